"""What each GEMM epilogue costs on the 70k-token shapes: the product entry points of one projection timed
interleaved in one process against the same GEMM with the plain bias epilogue (gp_linear), plus the
fp32 residual stream's read + write alone (torch in-place add) as the HBM reference for the residual
epilogues.

    python tools/epi_cost.py [--M 70001] [--rounds 7] [--iters 10] [--out file.json]
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
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--E", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    M, E = args.M, args.E
    F = 4 * E
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16

    def rn(*s, scale=1.0, dtype=bf):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(dtype)

    a = rn(M, E)
    h_in = rn(M, F)
    w_qkv, w_out, w_fc1, w_fc2 = rn(3 * E, E, scale=0.03), rn(E, E, scale=0.03), rn(F, E, scale=0.03), rn(E, F, scale=0.02)
    b3, bE, bF = (torch.randn(n, device=dev, generator=g) * 0.1 for n in (3 * E, E, F))
    cE3, dE3 = torch.randn(3 * E, device=dev, generator=g), torch.randn(3 * E, device=dev, generator=g)
    cF, dF = torch.randn(F, device=dev, generator=g), torch.randn(F, device=dev, generator=g)
    cE, dE = torch.randn(E, device=dev, generator=g), torch.randn(E, device=dev, generator=g)
    gam = torch.ones(E, device=dev)

    def stats_planes(n):                 # n planes of (mean 0, M2 256 = unit variance) + the merged plane
        s = torch.zeros(n + 1, M, 2, device=dev)
        s[:n, :, 1] = 256.0
        return s

    xst, hst = stats_planes(E // 256), stats_planes(F // 256)
    s0, s1 = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
    x = torch.randn(M, E, device=dev, generator=g)
    xb = torch.empty(M, E, device=dev, dtype=bf)
    qkv = torch.empty(M, 3 * E, device=dev, dtype=bf)
    y = torch.empty(M, E, device=dev, dtype=bf)
    h = torch.empty(M, F, device=dev, dtype=bf)
    ws = torch.empty(max(_hip.gemm_workspace_bytes(M, n, k) for n, k in ((3 * E, E), (E, E), (F, E), (E, F))) // 4 + 1,
                     device=dev)
    xo = torch.randn(M, E, device=dev, generator=g)

    cases = {
        "qkv": [("linear_bias", lambda: _hip.linear(a, w_qkv, b3, qkv, ws)),
                ("linear_ln", lambda: _hip.linear_ln(a, w_qkv, xst, E // 256, cE3, dE3, 1e-5, s0, s1, qkv, ws))],
        "out": [("linear_bias", lambda: _hip.linear(a, w_out, bE, y, ws)),
                ("linear_resid_x_only", lambda: _hip.linear_resid(a, w_out, bE, x, None, None, None, None, ws)),
                ("linear_resid", lambda: _hip.linear_resid(a, w_out, bE, x, s0, gam, xb, xst, ws)),
                ("torch_x_add_(fp32 r+w)", lambda: x.add_(xo))],
        "fc1": [("linear_bias", lambda: _hip.linear(a, w_fc1, bF, h, ws)),
                ("fc1_gelu", lambda: _hip.ffn_fc1_gelu(a, w_fc1, bF, h, hst)),
                ("fc1_gelu_ln", lambda: _hip.ffn_fc1_gelu_ln(a, w_fc1, xst, E // 256, cF, dF, 1e-5, s0, s1, h, hst))],
        "fc2": [("linear_bias", lambda: _hip.linear(h_in, w_fc2, bE, y, ws)),
                ("fc2_ln", lambda: _hip.ffn_fc2_ln(h_in, w_fc2, hst, cE, dE, 1e-5, y, ws)),
                ("fc2_ln_resid", lambda: _hip.ffn_fc2_ln_resid(h_in, w_fc2, hst, cE, dE, 1e-5, x, s0, gam, xb, xst, ws))],
    }
    res = {}
    for shape, variants in cases.items():
        times = {n: [] for n, _ in variants}
        for fn in (f for _, f in variants):
            fn()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for n, fn in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                e1.synchronize()
                times[n].append(e0.elapsed_time(e1) * 1e3 / args.iters)
        res[shape] = {n: round(statistics.median(t), 1) for n, t in times.items()}
        base = res[shape]["linear_bias"]
        print(shape, "  ".join("%s %.1f us (%+.1f)" % (n, v, v - base) for n, v in res[shape].items()), flush=True)
    out = {"M": M, "E": E, "F": F, "unit": "us per launch (median of %d rounds x %d)" % (args.rounds, args.iters),
           "shapes": res}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
