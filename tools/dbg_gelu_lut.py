"""Debug: where gp_ffn_fc1_gelu's bf16 h differs from torch's CPU GELU of gp_linear's pre-activation."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip  # noqa: E402

_hip.load_library()
DEV = "cuda"
E, F = 768, 3072
for M in (1, 255, 1000):
    g = torch.Generator(device=DEV).manual_seed(M)
    a = (torch.randn(M, E, device=DEV, generator=g)).bfloat16()
    w1 = (torch.randn(F, E, device=DEV, generator=g) * E ** -0.5 * 1.5).bfloat16()
    b1 = torch.randn(F, device=DEV, generator=g) * 0.2
    hh = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    stats = torch.empty((F // 256 + 1) * M * 2, device=DEV)
    _hip.ffn_fc1_gelu(a, w1, b1, hh, stats)
    pre = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    _hip.linear(a, w1, b1, pre, None)
    torch.cuda.synchronize()
    ex = torch.nn.functional.gelu(pre.float().cpu()).bfloat16()
    exg = torch.nn.functional.gelu(pre.float()).bfloat16().cpu()
    hc = hh.cpu()
    bad = hc != ex
    idx = bad.nonzero()
    print(M, "mismatch vs cpu", int(bad.sum()), "vs gpu torch", int((hc != exg).sum()), "cpu vs gpu torch",
          int((ex != exg).sum()), flush=True)
    pc = pre.cpu()
    for r, c in idx[:12].tolist():
        print(f"  row {r} col {c} (tile col {c // 256}, wn {(c % 256) // 64}, r16 {r % 16}) pre {pc[r, c].item():.6g} "
              f"0x{pc[r, c].view(torch.int16).item() & 0xffff:04x} h 0x{hc[r, c].view(torch.int16).item() & 0xffff:04x} "
              f"exact 0x{ex[r, c].view(torch.int16).item() & 0xffff:04x}")
    if bad.any():
        rows = idx[:, 0].unique()
        cols = idx[:, 1]
        print("  rows", rows[:20].tolist(), "n rows", rows.numel(), "col%16 hist", torch.bincount(cols % 16, minlength=16).tolist(),
              "col//256 hist", torch.bincount(cols // 256, minlength=12).tolist())
