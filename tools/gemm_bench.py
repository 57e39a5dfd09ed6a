"""The lab GEMM (tools/attn_lab/liblab_gemm.so, gp_gemm_bf16_tn) vs torch.addmm (hipBLASLt, the tuned
solutions the product uses) on the slide encoder's GEMM shapes, interleaved in one process; reports
median ms, TFLOP/s and the max |difference| relative to max |C|.

    python tools/gemm_bench.py [--lib tools/attn_lab/liblab_gemm4.so] [--M 70001] [--rounds 5] [--iters 10]
        [--shapes qkv,out,fc1,fc2,patch] [--out file.json]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

import ctypes  # noqa: E402

from gigapath import runtime  # noqa: E402

_lab = None


def load_lab(path):
    global _lab
    _lab = ctypes.CDLL(path if os.path.isabs(path) else os.path.join(ROOT, path))
    _lab.gp_gemm_bf16_tn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                     ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                     ctypes.c_int64, ctypes.c_void_p]


def gemm_bf16_tn(a, w, b, out):
    rc = _lab.gp_gemm_bf16_tn(a.data_ptr(), a.stride(0), w.data_ptr(), w.stride(0),
                              None if b is None else b.data_ptr(), int(b is not None and b.dtype == torch.float32),
                              out.data_ptr(), out.stride(0), a.shape[0], w.shape[0], a.shape[1],
                              torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc

SHAPES = [("qkv", 2304, 768, True), ("out", 768, 768, False), ("fc1", 3072, 768, True), ("fc2", 768, 3072, False),
          ("patch", 768, 1536, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default="tools/attn_lab/liblab_gemm.so")
    ap.add_argument("--shapes", default="qkv,out,fc1,fc2,patch")
    args = ap.parse_args()
    load_lab(args.lib)
    dev = torch.device("cuda")
    runtime.use_tuned_gemms(dev)
    g = torch.Generator(device="cuda").manual_seed(0)
    res = []
    for name, N, K, has_bias in SHAPES:
        if name not in args.shapes.split(","):
            continue
        M = args.M - 1 if name == "patch" else args.M
        a = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).to(torch.bfloat16)
        b = (torch.randn(N, device=dev, generator=g) * 0.1).to(torch.bfloat16) if has_bias else None
        c0 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        c1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ref = lambda: torch.addmm(b, a, w.t(), out=c0) if b is not None else torch.mm(a, w.t(), out=c0)  # noqa
        ours = lambda: gemm_bf16_tn(a, w, b, c1)  # noqa
        ref(); ours(); torch.cuda.synchronize()
        d = (c0.float() - c1.float()).abs().max().item() / c0.float().abs().max().item()
        ts = {"hipblaslt": [], "gp_gemm": []}
        for _ in range(args.rounds):
            for nm, fn in (("hipblaslt", ref), ("gp_gemm", ours)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts[nm].append(e0.elapsed_time(e1) / args.iters)
        fl = 2.0 * M * N * K
        row = {"gemm": name, "M": M, "N": N, "K": K, "rel_diff": d}
        for nm, t in ts.items():
            med = statistics.median(t)
            row[nm + "_ms"] = round(med, 4)
            row[nm + "_tflops"] = round(fl / med / 1e9, 1)
        res.append(row)
        print(json.dumps(row), flush=True)
        del a, w, c0, c1
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
