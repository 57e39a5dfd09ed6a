"""Probe: do the encoder's GEMMs run faster with M padded to a multiple of 256 (TunableOp-tuned
both ways)?  python tools/gemm_align_probe.py"""
import os
import time

import torch

torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(30)
torch.cuda.tunable.set_max_tuning_iterations(20)
torch.cuda.tunable.set_filename("/tmp/probe_tunableop.csv")
dev = "cuda"
E, F = 768, 3072
shapes = {"qkv": (E, 3 * E, True), "out": (E, E, False), "fc1": (E, F, True), "fc2": (F, E, False)}
for M in (70001, 70144, 70400):
    tot = 0.0
    res = []
    for name, (K, N, bias) in shapes.items():
        a = torch.randn(M, K, device=dev).bfloat16()
        w = torch.randn(N, K, device=dev).bfloat16()
        b = torch.randn(N, device=dev).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        f = (lambda: torch.addmm(b, a, w.t(), out=out)) if bias else (lambda: torch.mm(a, w.t(), out=out))
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        tot += ms
        res.append("%s %.4f ms (%.0f TF/s)" % (name, ms, 2 * M * K * N / ms / 1e9))
    print("M=%d total %.4f ms: %s" % (M, tot, "; ".join(res)), flush=True)
