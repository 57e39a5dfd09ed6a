"""Interleaved A/B timing of gp_gelu_layernorm (fc1 output -> GELU -> LN(F)) across library builds.

    python tools/norm_ab.py --libs prod,tools/attn_lab/liblab_gelu1.so [--rows 70001] [--cols 3072]

Same protocol as tools/attn_ab.py: every round times every library once (HIP events around --iters
back-to-back launches), so clock drift hits all builds alike; reports median / min launch time, the
algorithmic HBM rate (read + write of the bf16 rows) and bit-identity to the first
build.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--rows", type=int, default=70001)
    ap.add_argument("--cols", type=int, default=3072)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]
    R, F = args.rows, args.cols
    g = torch.Generator(device="cuda").manual_seed(0)
    h = (torch.randn(R, F, device="cuda", generator=g) * 1.5).to(torch.bfloat16)
    w = 1 + 0.1 * torch.randn(F, device="cuda", generator=g)
    b = 0.1 * torch.randn(F, device="cuda", generator=g)
    outs = {p: torch.empty(R, F, device="cuda", dtype=torch.bfloat16) for p, _ in libs}
    times = {p: [] for p, _ in libs}
    for rnd in range(args.rounds + 1):
        for p, lib in libs:
            _hip._lib = lib
            run = lambda: _hip.gelu_layernorm(h, w, b, 1e-5, outs[p], R, F)  # noqa
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
    first = libs[0][0]
    nbytes = 2 * R * F * 2
    res = []
    for p, ts in times.items():
        med, mn = statistics.median(ts), min(ts)
        ident = torch.equal(outs[p].view(torch.int16), outs[first].view(torch.int16))
        if not ident:
            ne = outs[p].view(torch.int16) != outs[first].view(torch.int16)
            rr, cc = torch.nonzero(ne, as_tuple=True)
            print("%s: %d elements differ in %d rows; first rows %s cols %s; max|d| %.4g" % (
                p, int(ne.sum()), len(torch.unique(rr)), torch.unique(rr)[:6].tolist(), torch.unique(cc)[:6].tolist(),
                float((outs[p].float() - outs[first].float()).abs().max())), flush=True)
        res.append({"lib": p, "median_ms": round(med, 4), "min_ms": round(mn, 4),
                    "gbps_median": round(nbytes / med / 1e6, 1), "bit_identical_to_first": ident})
        print("%-40s median %.4f ms  min %.4f ms  %7.1f GB/s  ident=%s" % (p, med, mn, nbytes / med / 1e6, ident),
              flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"rows": R, "cols": F, "rounds": args.rounds, "iters": args.iters, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
