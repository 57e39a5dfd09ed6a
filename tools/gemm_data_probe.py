"""Does the MFMA GEMM's time depend on its operand values?  gp_linear on the QKV shape (70k x 2304 x 768) with
the A operand scaled by several factors (same bits pattern family, different exponents), and with a
LayerNorm-normalised A, interleaved in one process.

    python tools/gemm_data_probe.py [--M 70001] [--rounds 7]
"""
import argparse
import json
import statistics
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--N", type=int, default=2304)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randn(args.M, args.K, device=dev, generator=g)
    w = (torch.randn(args.N, args.K, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    b = torch.zeros(args.N, device=dev)
    out = torch.empty(args.M, args.N, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(_hip.gemm_workspace_bytes(args.M, args.N, args.K) // 4 + 1, device=dev)
    shifted = base * 3.0 + 5.0 * torch.randn(args.M, 1, device=dev, generator=g)   # rows with a mean, std 3
    variants = {
        "A=N(0,1)": base.to(torch.bfloat16),
        "A=0.1*N(0,1)": (base * 0.1).to(torch.bfloat16),
        "A=10*N(0,1)": (base * 10).to(torch.bfloat16),
        "A=row-shifted (mean~5, std 3)": shifted.to(torch.bfloat16),
        "A=LN(row-shifted)": torch.nn.functional.layer_norm(shifted, (args.K,)).to(torch.bfloat16),
        "A=zeros": torch.zeros(args.M, args.K, device=dev, dtype=torch.bfloat16),
    }
    times = {k: [] for k in variants}
    for a in variants.values():
        _hip.linear(a, w, b, out, ws)
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for k, a in variants.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                _hip.linear(a, w, b, out, ws)
            e1.record()
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    res = {k: round(statistics.median(v), 1) for k, v in times.items()}
    for k, v in res.items():
        print("%-34s %8.1f us" % (k, v), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"shape": [args.M, args.N, args.K], "us_per_launch_median": res}, f, indent=1)


if __name__ == "__main__":
    main()
