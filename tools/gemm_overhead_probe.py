"""Per-tile overhead of gp_linear: time M x N x K for K = 768 / 1536 / 3072 (fit t_tile = NK * t_k + o),
and the same shapes with a lab library (e.g. one built with -DGP_EXP_NOSTORE: the epilogue without its
stores).  Median of interleaved rounds, HIP events on the launch stream.

    python tools/gemm_overhead_probe.py [--lab tools/attn_lab/liblab_gemm_nostore.so] [--out f.json]
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
    ap.add_argument("--lab", action="append", default=[])
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [("product", prod)] + [(os.path.basename(p), _hip.load_library(os.path.join(ROOT, p))) for p in args.lab]
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    for N, K in ((3072, 768), (3072, 1536), (3072, 3072), (768, 768), (2304, 768), (768, 3072)):
        a = torch.randn(args.M, K, device=dev, generator=g).bfloat16()
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
        c = torch.empty(args.M, N, dtype=torch.bfloat16, device=dev)
        ts = {name: [] for name, _ in libs}
        for _ in range(args.rounds):
            for name, lib in libs:
                _hip._lib = lib
                _hip.linear(a, w, None, c, None)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    _hip.linear(a, w, None, c, None)
                e1.record()
                torch.cuda.synchronize()
                ts[name].append(e0.elapsed_time(e1) / args.iters)
                _hip._lib = prod
        row = {"M": args.M, "N": N, "K": K}
        for name, v in ts.items():
            m = statistics.median(v)
            row[name + "_ms"] = round(m, 4)
            row[name + "_tflops"] = round(2.0 * args.M * N * K / m / 1e9, 1)
        print(row, flush=True)
        res.append(row)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
