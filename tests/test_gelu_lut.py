"""The bf16 GELU table compiled into gp_ffn_fc1_gelu (csrc/gp_gelu_lut.h, made by tools/gen_gelu_lut.py)
against torch's F.gelu on the CPU -- the arithmetic of feedforward_network.py:134 -- entry by entry, and
the out-of-table rules the kernel applies, over every bf16 input (no GPU)."""
import importlib.util
import os
import re

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "prov-gigapath-replication_amd", "csrc", "gp_gelu_lut.h")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_gelu_lut", os.path.join(ROOT, "tools", "gen_gelu_lut.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _header():
    text = open(HEADER).read()
    lo = int(re.search(r"kGeluLutLo = (0x[0-9a-f]+)", text).group(1), 16)
    hi = int(re.search(r"kGeluLutHi = (0x[0-9a-f]+)", text).group(1), 16)
    n = int(re.search(r"kGeluLutN = (\d+)", text).group(1))
    body = text[text.index("= {"):]
    vals = [int(v, 16) for v in re.findall(r"0x([0-9a-f]{4})", body)]
    return lo, hi, n, vals


def test_table_is_torch_gelu():
    lo, hi, n, vals = _header()
    assert n == hi - lo + 1 and len(vals) == 2 * n
    gen = _gen()
    assert (gen.LO, gen.HI) == (lo, hi)
    assert vals == gen.table().tolist()


def test_out_of_table_rules():
    _gen().check_rules()


def test_kernel_rules_restated():
    """gelu_lut_pair + gelu_fix (gp_gemm.hip) restated on bit patterns, against torch for every finite bf16."""
    lo, hi, n, vals = _header()
    bits = torch.arange(0, 65536, dtype=torch.int64)
    m, neg = bits & 0x7FFF, (bits >> 15) & 1
    t = torch.clamp(m - lo, 0, n - 1)
    out = torch.tensor(vals)[neg * n + t]
    x = bits.to(torch.int16).view(torch.bfloat16).float()
    half = (x * 0.5).to(torch.bfloat16).view(torch.int16).to(torch.int64) & 0xFFFF
    big = torch.where(neg == 1, torch.where(m >= 0x7F80, 0x7FC0, 0x8000),
                      torch.where((m >= 0x7F00) & (m < 0x7F80), 0x7F80, bits))
    out = torch.where(m > hi, big, out)
    out = torch.where(m < lo, half, out)
    ref = torch.nn.functional.gelu(x).to(torch.bfloat16).view(torch.int16).to(torch.int64) & 0xFFFF
    finite = m < 0x7F80
    assert torch.equal(out[finite], ref[finite])
