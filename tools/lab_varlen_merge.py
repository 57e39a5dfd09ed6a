"""Packed-slide (varlen) merge: a lab build against the product -- the varlen GPU tests run on the lab build, then
the C5 batch's merge (32 slides, 675,587 tokens) timed interleaved on both builds, outputs compared bit for bit.

    python tools/lab_varlen_merge.py tools/attn_lab/liblab_x.so
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from gigapath import _hip, batch, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
prod = _hip.load_library()
lab = _hip.load_library(os.path.join(ROOT, sys.argv[1]))
_hip._lib = lab
import test_gpu_batch as t  # noqa: E402

for fmt in ("bf16", "bf16_overflow", "fp16_overflow"):
    t.test_varlen_attention_and_merge_bit_exact_per_slide(fmt)
    print("varlen bit-exact per slide", fmt, "ok (lab)", flush=True)
t.test_forward_packed_matches_individual_forwards(False)
print("packed forward == individual forwards ok (lab)", flush=True)

H, D, E = 16, 48, 768
Ls = [n + 1 for n in batch.mixed_batch_sizes(n_slides=32)]
T = sum(Ls)
g = torch.Generator(device="cuda").manual_seed(7)
qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
qkv[:, :E] *= 0.35
qkv = qkv.to(torch.bfloat16)
vs = runtime.VarlenScratch(torch.device("cuda"), Ls, H, D, SEGS, RATIOS, qkv)
_hip._lib = prod
_hip.dilated_attn_fwd_varlen(vs.plan, True)
ln_w = torch.rand(E, device="cuda") + 0.5
ln_b = torch.randn(E, device="cuda") * 0.1
outs = {}
times = {"prod": [], "lab": []}
for rnd in range(9):
    for name, lib in (("prod", prod), ("lab", lab)):
        _hip._lib = lib
        out = torch.empty(T, E, dtype=torch.bfloat16, device="cuda")
        _hip.branch_merge_ln_varlen(vs.plan, ln_w, ln_b, 1e-5, out)
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(5):
            _hip.branch_merge_ln_varlen(vs.plan, ln_w, ln_b, 1e-5, out)
        s1.record()
        s1.synchronize()
        times[name].append(s0.elapsed_time(s1) / 5)
        outs[name] = out
print("C5 varlen merge (%d tokens): prod median %.4f ms, lab median %.4f ms, bit-identical %s"
      % (T, statistics.median(times["prod"]), statistics.median(times["lab"]), torch.equal(outs["prod"], outs["lab"])),
      flush=True)
