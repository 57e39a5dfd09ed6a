"""A/B timing of the GELU+LN row kernel (gp_gelu_layernorm) at the 70k-slide FFN shape.

    python tools/row_bench.py [--rows 70001] [--impls 3,2]
Interleaves GP_GELU_IMPL values in one process; reports ms, effective GB/s (bf16 read + write)
and each implementation's max |difference| from the first one and from the fp32 torch reference."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip  # noqa: E402

# the run-time variant switches (GP_ATTN_IMPL / GP_ATTN_VAR / GP_GELU_IMPL) live in the lab build only
_hip._lib = _hip.load_library(os.path.join(ROOT, "tools", "attn_lab", "liblab_r01.so"))

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=70001)
ap.add_argument("--cols", type=int, default=3072)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--impls", default="3,5")
args = ap.parse_args()
M, F = args.rows, args.cols
g = torch.Generator(device="cuda").manual_seed(0)
x = (torch.randn(M, F, device="cuda", generator=g) * 1.5).bfloat16()
w = 1 + 0.1 * torch.randn(F, device="cuda", generator=g)
b = 0.1 * torch.randn(F, device="cuda", generator=g)
out = torch.empty_like(x)
ref = torch.nn.functional.layer_norm(torch.nn.functional.gelu(x[:4096].float()).bfloat16().float(), (F,), w, b, 1e-5)
res, first = {}, {}
impls = args.impls.split(",")
for it in range(args.iters + 1):
    for impl in impls:
        os.environ["GP_GELU_IMPL"] = impl
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _hip.gelu_layernorm(x, w, b, 1e-5, out, M, F)
        e1.record()
        torch.cuda.synchronize()
        if it == 0:
            first[impl] = out.clone()
        else:
            res.setdefault(impl, []).append(e0.elapsed_time(e1))
for impl in impls:
    ts = sorted(res[impl])
    med = ts[len(ts) // 2]
    d0 = (first[impl].float() - first[impls[0]].float()).abs().max().item()
    dr = (first[impl][:4096].float() - ref).abs().max().item()
    neq = (first[impl] != first[impls[0]]).float().mean().item()
    print("impl %s: median %.4f ms  %.0f GB/s  max|d vs %s| %.3g (%.2e of elements differ)  max|d vs fp32 ref| %.3g"
          % (impl, med, 4.0 * M * F / med / 1e6, impls[0], d0, neq, dr))
