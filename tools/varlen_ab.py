"""Interleaved A/B timing of the varlen (packed C5 batch) attention launch across library builds.

    python tools/varlen_ab.py --libs prod,tools/attn_lab/liblab_vlold.so [--slides 32] [--rounds 7]

One process, one GPU: every round times each library's gp_dilated_attn_fwd_varlen (HIP events around
--iters launches) on the same random packed qkv of batch.mixed_batch_sizes(); reports median / min per
launch and valid TFLOP/s, and whether each build's outputs are bit-identical to the first build's.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, batch, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--slides", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]
    H, D = 16, 48
    E = H * D
    Ls = [n + 1 for n in batch.mixed_batch_sizes(n_slides=args.slides)]
    T = sum(Ls)
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    qkv = qkv.to(torch.bfloat16)
    flops = sum(runtime.attention_valid_flops(L, SEGS, RATIOS, H, D) for L in Ls)
    runs = {}
    for name, lib in libs:
        _hip._lib = lib
        plan = _hip.VarlenPlan(Ls, H, D, SEGS, RATIOS)
        outs = [torch.zeros(n, dtype=torch.bfloat16, device="cuda") for n in plan.o_elems]
        lses = [torch.zeros(n, dtype=torch.float32, device="cuda") for n in plan.lse_elems]
        plan.bind(qkv, outs, lses)
        runs[name] = (lib, plan, outs, lses)
    _hip._lib = prod
    times = {n: [] for n, _ in libs}
    for _ in range(args.rounds):
        for name, _ in libs:
            lib, plan, outs, lses = runs[name]
            _hip._lib = lib
            _hip.dilated_attn_fwd_varlen(plan)          # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                _hip.dilated_attn_fwd_varlen(plan)
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.iters)
    _hip._lib = prod
    ref = runs[libs[0][0]]
    res = {}
    for name, _ in libs:
        o, l = runs[name][2], runs[name][3]
        ident = all(torch.equal(a, b) for a, b in zip(o, ref[2])) and all(torch.equal(a, b) for a, b in zip(l, ref[3]))
        med, mn = statistics.median(times[name]), min(times[name])
        res[name] = {"median_ms": med, "min_ms": mn, "tflops": flops / med / 1e9, "ident": ident}
        print("%-40s median %.4f ms  min %.4f ms  %7.1f TF/s  ident=%s" % (name, med, mn, flops / med / 1e9, ident))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump({"T": T, "slides": len(Ls), "flops": flops, "results": res, "times": times}, fh, indent=1)


if __name__ == "__main__":
    main()
