"""Same-process, interleaved A/B of the product GEMM entry points (the 70k-token shapes of one layer) across
library builds of the same ABI: per round every build runs every entry point `iters` times; medians in us
per launch, plus each build's output distance to the first build's (timing-only lab ablations are
deliberately wrong; real variants must be ~0).

    python tools/gemm_ab.py --libs prod,tools/attn_lab/liblab_x.so [--M 70001] [--rounds 7] [--out f.json]
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
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--E", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--fmt", default="bf16")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    M, E = args.M, args.E
    F = 4 * E
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    act = torch.bfloat16 if args.fmt == "bf16" else torch.float16
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]

    def rn(*s, scale=1.0, dtype=act):
        return (torch.randn(*s, device=dev, generator=g) * scale).to(dtype)

    a = rn(M, E)
    h_in = torch.nn.functional.gelu(rn(M, F).float()).to(act)
    w_qkv, w_out, w_fc1, w_fc2 = rn(3 * E, E, scale=0.03), rn(E, E, scale=0.03), rn(F, E, scale=0.03), rn(E, F, scale=0.02)
    b3, bE, bF = (torch.randn(n, device=dev, generator=g) * 0.1 for n in (3 * E, E, F))
    cE3, dE3 = torch.randn(3 * E, device=dev, generator=g) * 0.01, torch.randn(3 * E, device=dev, generator=g)
    cF, dF = torch.randn(F, device=dev, generator=g) * 0.01, torch.randn(F, device=dev, generator=g)
    cE, dE = torch.randn(E, device=dev, generator=g) * 0.01, torch.randn(E, device=dev, generator=g)
    gam = torch.ones(E, device=dev)

    def stats_planes(n):                 # n planes of (mean 0, M2 256 = unit variance) + the merged plane
        s = torch.zeros(n + 1, M, 2, device=dev)
        s[:n, :, 1] = 256.0
        return s

    xst, hst = stats_planes(E // 256), stats_planes(F // 256)
    s0, s1 = torch.zeros(M, device=dev), torch.zeros(M, device=dev)
    x0 = torch.randn(M, E, device=dev, generator=g)
    x = x0.clone()
    xb = torch.empty(M, E, device=dev, dtype=act)
    qkv = torch.empty(M, 3 * E, device=dev, dtype=act)
    y = torch.empty(M, E, device=dev, dtype=act)
    h = torch.empty(M, F, device=dev, dtype=act)
    ws = torch.empty(max(_hip.gemm_workspace_bytes(M, n, k) for n, k in ((3 * E, E), (E, E), (F, E), (E, F))) // 4 + 1,
                     device=dev)

    def fresh_x():
        x.copy_(x0)

    cases = [
        ("qkv_bias", lambda: _hip.linear(a, w_qkv, b3, qkv, ws), lambda: qkv),
        ("qkv_ln", lambda: _hip.linear_ln(a, w_qkv, xst, E // 256, cE3, dE3, 1e-5, s0, s1, qkv, ws), lambda: qkv),
        ("out_bias", lambda: _hip.linear(a, w_out, bE, y, ws), lambda: y),
        ("out_resid", lambda: _hip.linear_resid(a, w_out, bE, x, s0, gam, xb, xst, ws), lambda: xb),
        ("fc1_bias", lambda: _hip.linear(a, w_fc1, bF, h, ws), lambda: h),
        ("fc1_gelu", lambda: _hip.ffn_fc1_gelu(a, w_fc1, bF, h, hst), lambda: h),
        ("fc1_gelu_ln", lambda: _hip.ffn_fc1_gelu_ln(a, w_fc1, xst, E // 256, cF, dF, 1e-5, s0, s1, h, hst), lambda: h),
        ("fc2_bias", lambda: _hip.linear(h_in, w_fc2, bE, y, ws), lambda: y),
        ("fc2_ln_resid", lambda: _hip.ffn_fc2_ln_resid(h_in, w_fc2, hst, cE, dE, 1e-5, x, s0, gam, xb, xst, ws),
         lambda: xb),
    ]
    if args.only:
        keep = args.only.split(",")
        cases = [c for c in cases if c[0] in keep]
    ref_out = {}
    times = {(p, n): [] for p, _ in libs for n, _, _ in cases}
    diffs = {}
    for p, lib in libs:                                      # correctness vs the first build, one call each
        _hip._lib = lib
        for n, fn, out in cases:
            fresh_x()
            fn()
            torch.cuda.synchronize()
            o = out().float().clone()
            if p == libs[0][0]:
                ref_out[n] = o
            diffs[(p, n)] = ((o - ref_out[n]).abs().max() / ref_out[n].abs().max()).item()
    for _ in range(args.rounds):
        for n, fn, _ in cases:
            for p, lib in libs:
                _hip._lib = lib
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                e1.synchronize()
                times[(p, n)].append(e0.elapsed_time(e1) * 1e3 / args.iters)
    _hip._lib = prod
    res = []
    for p, _ in libs:
        row = {"lib": p, "us": {n: round(statistics.median(times[(p, n)]), 1) for n, _, _ in cases},
               "rel_diff_vs_first": {n: diffs[(p, n)] for n, _, _ in cases}}
        print(json.dumps(row), flush=True)
        res.append(row)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"M": M, "E": E, "fmt": args.fmt, "rounds": args.rounds, "iters": args.iters, "results": res}, f,
                      indent=1)


if __name__ == "__main__":
    main()
