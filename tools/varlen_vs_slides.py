"""C5 attention: the packed varlen launch vs each slide's own single-slide launch, same qkv rows.

    python tools/varlen_vs_slides.py [--slides 32] [--rounds 5]

Reports the packed launch's time and valid TFLOP/s, the sum of the 32 single-slide launches (each the
product kernel on that slide's rows, with q pre-scaled as in the forward), and per-slide TFLOP/s by
size -- whether the C5 attention rate is set by the packing or by the slide-size mix.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, batch, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def timed(fn, iters):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slides", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    H, D = 16, 48
    E = H * D
    Ls = [n + 1 for n in batch.mixed_batch_sizes(n_slides=args.slides)]
    offs = [0]
    for L in Ls:
        offs.append(offs[-1] + L)
    T = offs[-1]
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    qkv = qkv.to(torch.bfloat16)
    plan = _hip.VarlenPlan(Ls, H, D, SEGS, RATIOS)
    outs = [torch.zeros(n, dtype=torch.bfloat16, device="cuda") for n in plan.o_elems]
    lses = [torch.zeros(n, dtype=torch.float32, device="cuda") for n in plan.lse_elems]
    plan.bind(qkv, outs, lses)
    scr = {L: runtime.AttentionScratch("cuda", 1, L, H, D, SEGS, RATIOS) for L in set(Ls)}
    flops = [runtime.attention_valid_flops(L, SEGS, RATIOS, H, D) for L in Ls]

    def one(i):
        L, o = Ls[i], offs[i]
        q = qkv[o:o + L]
        s = scr[L]
        _hip.dilated_attn_fwd(q, q[:, E:], q[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, s.outs, s.lses,
                              q_log2_prescaled=True)

    packed, per = [], [[] for _ in Ls]
    for _ in range(args.rounds):
        packed.append(timed(lambda: _hip.dilated_attn_fwd_varlen(plan), 3))
        for i in range(len(Ls)):
            per[i].append(timed(lambda i=i: one(i), 3))
    pk = statistics.median(packed)
    ps = [statistics.median(x) for x in per]
    res = {"T": T, "packed_ms": pk, "packed_tflops": sum(flops) / pk / 1e9,
           "sum_single_ms": sum(ps), "single_tflops": sum(flops) / sum(ps) / 1e9,
           "slides": sorted(({"L": L, "ms": round(t, 4), "tflops": round(f / t / 1e9, 1)}
                             for L, t, f in zip(Ls, ps, flops)), key=lambda d: d["L"])}
    print(json.dumps({k: v for k, v in res.items() if k != "slides"}))
    for d in res["slides"]:
        print("L %7d  %.4f ms  %6.1f TF/s" % (d["L"], d["ms"], d["tflops"]))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
