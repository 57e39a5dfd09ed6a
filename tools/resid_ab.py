"""Interleaved A/B timing of gp_residual_layernorm (x += y + b; out = LN(x)) across library builds, at
the 70k-slide shape.  Reports median ms and the algorithmic HBM rate (x fp32 read + write, y and out
16-bit), and whether each build's outputs equal the first's.

    python tools/resid_ab.py --libs prod,tools/attn_lab/liblab_resln_nt1.so [--rows 70001]
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
    ap.add_argument("--cols", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]
    R, E = args.rows, args.cols
    g = torch.Generator(device="cuda").manual_seed(0)
    x0 = torch.randn(R, E, device="cuda", generator=g)
    y = (torch.randn(R, E, device="cuda", generator=g) * 0.1).bfloat16()
    bias = 0.01 * torch.randn(E, device="cuda", generator=g)
    w = 1 + 0.1 * torch.randn(E, device="cuda", generator=g)
    b = 0.1 * torch.randn(E, device="cuda", generator=g)
    xs = {p: x0.clone() for p, _ in libs}
    outs = {p: torch.empty(R, E, device="cuda", dtype=torch.bfloat16) for p, _ in libs}
    times = {p: [] for p, _ in libs}
    for rnd in range(args.rounds + 1):
        for p, lib in libs:
            _hip._lib = lib
            run = lambda: _hip.residual_layernorm(xs[p], y, bias, w, b, 1e-5, outs[p], R, E)  # noqa
            if rnd == 0:
                xs[p].copy_(x0)
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
    nbytes = R * E * (4 + 4 + 2 + 2)
    res = []
    for p, ts in times.items():
        med = statistics.median(ts)
        ident = torch.equal(outs[p].view(torch.int16), outs[first].view(torch.int16)) and torch.equal(xs[p], xs[first])
        res.append({"lib": p, "median_ms": round(med, 4), "gbps": round(nbytes / med / 1e6, 1), "identical": ident})
        print("%-44s median %.4f ms  %7.1f GB/s  identical=%s" % (p, med, nbytes / med / 1e6, ident), flush=True)
    if args.out:
        json.dump({"rows": R, "cols": E, "results": res}, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
