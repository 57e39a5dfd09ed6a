"""Interleaved A/B timing of gp_branch_merge_ln (5-branch LSE merge + inner LN) at the 70k-slide shape
across library builds, on real attention outputs.  Median ms, algorithmic HBM rate
(runtime.merge_bytes) and bit-identity to the first build.

    python tools/merge_ab.py --libs prod,tools/attn_lab/liblab_merge_nt.so [--L 70001]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--L", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]
    H, D, E, L = 16, 48, 768, args.L
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn(L, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    qkv = qkv.to(torch.bfloat16)
    ln_w = torch.rand(E, device="cuda", generator=g) + 0.5
    ln_b = torch.randn(E, device="cuda", generator=g) * 0.1
    sc = runtime.AttentionScratch(dev, 1, L, H, D, SEGS, RATIOS)
    _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, sc.outs, sc.lses, 0.0, True)
    outs = {p: torch.empty(L, E, dtype=torch.bfloat16, device="cuda") for p, _ in libs}
    times = {p: [] for p, _ in libs}
    for rnd in range(args.rounds + 1):
        for p, lib in libs:
            _hip._lib = lib
            run = lambda: _hip.branch_merge_ln(sc.outs, sc.lses, SEGS, RATIOS, 1, L, H, D, ln_w, ln_b, 1e-5, outs[p])  # noqa
            if rnd == 0:
                run()
                torch.cuda.synchronize()
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) / args.iters)
    _hip._lib = prod
    nbytes = runtime.merge_bytes(L, SEGS, RATIOS, H, D)
    first = libs[0][0]
    res = []
    for p, ts in times.items():
        med = statistics.median(ts)
        ident = torch.equal(outs[p].view(torch.int16), outs[first].view(torch.int16))
        d = (outs[p].float() - outs[first].float()).abs()
        ulp = (outs[p].view(torch.int16).int() - outs[first].view(torch.int16).int()).abs()
        res.append({"lib": p, "median_ms": round(med, 4), "gbps": round(nbytes / med / 1e6, 1), "identical": ident,
                    "max_abs_diff": float(d.max()), "max_ulp_diff": int(ulp.max()),
                    "frac_diff": float((ulp > 0).float().mean())})
        print("%-44s median %.4f ms  %7.1f GB/s  identical=%s  max|d| %.3g  max ulp %d  frac %.2e" % (
            p, med, nbytes / med / 1e6, ident, float(d.max()), int(ulp.max()), float((ulp > 0).float().mean())),
            flush=True)
    if args.out:
        json.dump({"L": L, "results": res}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
