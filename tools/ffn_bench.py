"""The encoder FFN at the 70k-slide shape, interleaved in one process:

  unfused   hipBLASLt fc1 (bias epilogue) -> gp_gelu_layernorm -> hipBLASLt fc2    (round-2 product)
  fused     gp_ffn_fc1_gelu (GELU + LN statistics epilogue) -> gp_ffn_fc2_ln (LN folded into fc2)

and the plain projection GEMMs, gp_linear against tuned hipBLASLt.  Reports median ms per call over
`rounds` x `iters` launches (HIP events on the launch stream) and the max |difference| between the two
FFN outputs relative to max |y|.

    python tools/ffn_bench.py [--M 70001] [--rounds 7] [--iters 10] [--half] [--out file.json]
        [--lab tools/attn_lab/liblab_gemm9.so]   # also time a lab build of the same GEMM ABI, interleaved
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


def timed(fn, rounds, iters):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / iters)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--half", action="store_true", help="fp16 (the reference pipeline's autocast) instead of bf16")
    ap.add_argument("--out", default=None)
    ap.add_argument("--lab", default=None, help="a lab library exporting the GEMM ABI (liblab_gemm9.so)")
    args = ap.parse_args()
    prod = _hip.load_library()
    lab = _hip.load_library(os.path.join(ROOT, args.lab) if args.lab and not os.path.isabs(args.lab) else args.lab) \
        if args.lab else None

    def using(lib, fn):
        """fn() with the typed wrappers bound to lib (the product library otherwise)."""
        def run():
            _hip._lib = lib
            try:
                fn()
            finally:
                _hip._lib = prod
        return run
    dev = torch.device("cuda")
    runtime.use_tuned_gemms(dev)
    act = torch.float16 if args.half else torch.bfloat16
    M, E, F = args.M, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(0)
    rn = lambda *s, sc=1.0: torch.randn(*s, device=dev, generator=g) * sc  # noqa: E731
    a = rn(M, E).to(act)
    w1, b1 = rn(F, E, sc=E ** -0.5 * 1.5).to(act), rn(F, sc=0.2)
    gam, bet = 1 + rn(F, sc=0.3), rn(F, sc=0.1)
    w2, b2 = rn(E, F, sc=F ** -0.5).to(act), rn(E, sc=0.1)
    w2g = (w2.double() * gam.double()[None]).to(act)
    c2 = w2g.double().sum(1).float()
    d2 = (w2.double() @ bet.double() + b2.double()).float()
    b1a = b1.to(act)
    f = torch.empty(M, F, dtype=act, device=dev)
    y0 = torch.empty(M, E, dtype=act, device=dev)
    y1 = torch.empty(M, E, dtype=act, device=dev)
    stats, gws = runtime.ffn_buffers(dev, M, E, F)

    def unfused():
        torch.addmm(b1a, a, w1.t(), out=f)
        _hip.gelu_layernorm(f, gam, bet, 1e-5, f, M, F)
        torch.addmm(b2.to(act), f, w2.t(), out=y0)

    def fused():
        _hip.ffn_fc1_gelu(a, w1, b1, f, stats)
        _hip.ffn_fc2_ln(f, w2g, stats, c2, d2, 1e-5, y1, gws)

    unfused(); fused(); torch.cuda.synchronize()
    diff = ((y0.float() - y1.float()).abs().max() / y0.float().abs().max()).item()
    res = {"M": M, "act": str(act), "ffn_rel_diff": diff, "ffn": {}, "parts": {}, "linear": []}
    variants = [("unfused", unfused), ("fused", fused)]
    if lab is not None:
        y2 = y1.clone()
        using(lab, fused)()
        torch.cuda.synchronize()
        res["lab_vs_product_ffn_rel_diff"] = ((y1.float() - y2.float()).abs().max() / y2.float().abs().max()).item()
        variants.append(("lab_fused", using(lab, fused)))
    ts = {k: [] for k, _ in variants}
    for _ in range(args.rounds):
        for k, fn in variants:
            ts[k] += timed(fn, 1, args.iters)
    res["ffn"] = {k + "_ms": round(statistics.median(v), 4) for k, v in ts.items()}
    parts = {
        "hipblaslt_fc1": lambda: torch.addmm(b1a, a, w1.t(), out=f),
        "gelu_ln": lambda: _hip.gelu_layernorm(f, gam, bet, 1e-5, f, M, F),
        "hipblaslt_fc2": lambda: torch.mm(f, w2.t(), out=y0),
        "fc1_gelu": lambda: _hip.ffn_fc1_gelu(a, w1, b1, f, stats),
        "fc2_ln": lambda: _hip.ffn_fc2_ln(f, w2g, stats, c2, d2, 1e-5, y1, gws),
    }
    if lab is not None:
        parts["lab_fc1_gelu"] = using(lab, parts["fc1_gelu"])
        parts["lab_fc2_ln"] = using(lab, parts["fc2_ln"])
    for k, fn in parts.items():
        res["parts"][k + "_ms"] = round(statistics.median(timed(fn, args.rounds, args.iters)), 4)
    for name, N, K, has_bias in (("qkv", 3 * E, E, True), ("out", E, E, False), ("fc1", F, E, True),
                                 ("fc2", E, F, False), ("patch", E, 1536, True)):
        Mi = M - 1 if name == "patch" else M
        x = rn(Mi, K).to(act)
        w = rn(N, K, sc=K ** -0.5).to(act)
        b = rn(N, sc=0.1) if has_bias else None
        ba = b.to(act) if has_bias else None
        c0 = torch.empty(Mi, N, dtype=act, device=dev)
        c1 = torch.empty(Mi, N, dtype=act, device=dev)
        nb = _hip.gemm_workspace_bytes(Mi, N, K)
        ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
        ref = (lambda: torch.addmm(ba, x, w.t(), out=c0)) if has_bias else (lambda: torch.mm(x, w.t(), out=c0))
        ours = lambda: _hip.linear(x, w, b, c1, ws)  # noqa: E731
        ref(); ours(); torch.cuda.synchronize()
        d = ((c0.float() - c1.float()).abs().max() / c0.float().abs().max()).item()
        fns = [("hipblaslt", ref), ("gp_linear", ours)]
        row = {"gemm": name, "M": Mi, "N": N, "K": K, "rel_diff": d}
        if lab is not None:
            nbl = int(lab.gp_gemm_workspace_bytes(Mi, N, K))
            wsl = torch.empty(max(nbl, 16), dtype=torch.uint8, device=dev)
            c2 = torch.empty(Mi, N, dtype=act, device=dev)
            labf = using(lab, lambda: _hip.linear(x, w, b, c2, wsl))  # noqa: E731
            labf(); torch.cuda.synchronize()
            row["lab_rel_diff"] = ((c0.float() - c2.float()).abs().max() / c0.float().abs().max()).item()
            fns.append(("lab_linear", labf))
        tt = {k: [] for k, _ in fns}
        for _ in range(args.rounds):
            for k, fn in fns:
                tt[k] += timed(fn, 1, args.iters)
        fl = 2.0 * Mi * N * K
        for k, v in tt.items():
            m = statistics.median(v)
            row[k + "_ms"] = round(m, 4)
            row[k + "_tflops"] = round(fl / m / 1e9, 1)
        res["linear"].append(row)
        del x, w, c0, c1
    print(json.dumps(res, indent=1), flush=True)
    if args.out:
        with open(args.out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
