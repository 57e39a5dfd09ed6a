"""A/B timing of gp_dilated_attn_fwd implementations on one layer's worth of random QKV.

    python tools/attn_bench.py [--L 70001] [--iters 10]
Interleaves implementations (GP_ATTN_IMPL=1/2) in one process; reports TFLOP/s on the
algorithmic (valid-token) FLOPs of SURVEY §8(d)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

def _lab_stamps():
    import ctypes
    out = (ctypes.c_int64 * 8)()
    _hip._lib.gp_debug_attn_stamps(out, 1)
    return list(out)


# the run-time variant switches (GP_ATTN_IMPL / GP_ATTN_VAR / GP_GELU_IMPL) live in the lab build only
_hip._lib = _hip.load_library(os.path.join(ROOT, "tools", "attn_lab", "liblab_r01.so"))

ap = argparse.ArgumentParser()
ap.add_argument("--L", type=int, default=70001)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--impls", default="2p,3p")
ap.add_argument("--D", type=int, default=48)
ap.add_argument("--branches", default="0,1,2,3,4", help="subset of the 5 branches to run")
args = ap.parse_args()
H, D = 16, args.D
E = H * D
L = args.L
segs, ratios = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
_sel = [int(b) for b in args.branches.split(",")]
segs, ratios = [segs[b] for b in _sel], [ratios[b] for b in _sel]
g = torch.Generator(device="cuda").manual_seed(0)
qkv = torch.randn(L, 3 * E, device="cuda", generator=g)
qkv[:, :E] *= 0.35      # typical projected-q scale so pre-scaled logits stay in a realistic range
qkv = qkv.to(torch.bfloat16)
sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, segs, ratios)
flops = runtime.attention_valid_flops(L, segs, ratios, H, D)
res = {}
first = {}
for rnd in range(args.iters):
    for impl in args.impls.split(","):
        base, _, var = impl.partition("@")            # "2p@4": impl 2, prescaled q, GP_ATTN_VAR=4
        os.environ["GP_ATTN_IMPL"] = base.rstrip("p")
        os.environ["GP_ATTN_VAR"] = var or "0"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, segs, ratios, sc.outs, sc.lses,
                              0.0, base.endswith("p"))
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            res.setdefault(impl, []).append(e0.elapsed_time(e1))
        else:      # outputs of every impl, compared with the first one's after the loop
            first[impl] = ([o.clone() for o in sc.outs], [x.clone() for x in sc.lses])
ref_impl = next(iter(first))
for impl, (outs, lses) in first.items():
    # rows no impl writes (outside every valid query range) hold garbage: compare NaN-equal
    do = max(float(torch.nan_to_num(a.float() - b.float(), nan=0.0).abs().max()) +
             float((a.float().isnan() != b.float().isnan()).sum()) for a, b in zip(outs, first[ref_impl][0]))
    dl = max(float((a - b).abs().max()) for a, b in zip(lses, first[ref_impl][1]))
    print("impl %s vs %s: max|d out| %.3g  max|d lse| %.3g" % (impl, ref_impl, do, dl))
if any(i.endswith("@34818") for i in res):      # stamped build: cycles per segment per tile
    st = _lab_stamps()
    names = ["S MFMAs", "softmax", "PV", "stage store", "barrier"]
    tiles = max(st[6], 1)
    print("stamps: %d waves, %d tiles, %.0f wave-cycles/tile; per tile: %s" % (
        st[7], st[6], st[5] / tiles, ", ".join("%s %.0f" % (n, v / tiles) for n, v in zip(names, st[:5]))))
for impl, ts in res.items():
    ts.sort()
    med = ts[len(ts) // 2]
    print("impl %s: median %.3f ms  min %.3f ms  -> %.1f TFLOP/s (valid)  %.1f%% of 2.5 PF"
          % (impl, med, ts[0], flops / med / 1e9, 100 * flops / med / 1e9 / 2500))
