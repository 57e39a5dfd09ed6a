"""Interleaved A/B timing of gp_dilated_attn_fwd across library builds (one process, one GPU).

    python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_tune1.so [--L 70001] [--rounds 7]
        [--branches all,0,1,2,3,4] [--merge]

--merge times gp_branch_merge_ln (the five branches' LSE merge + inner LN of one 70k layer, fed by
the product attention's outputs) per library instead of the attention launches.

"prod" is the in-tree product library.  Every round times every (library, branch set) pair once
(HIP events around --iters back-to-back launches on random q/k/v of one layer), so clock drift and
device-to-device variance hit all variants alike (cdna_hip_programming.md §5.4 rule 24).  Reports
the median / min launch time and valid TFLOP/s per pair, plus whether each build's
outputs are bit-identical to the first build's.
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

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--L", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--branches", default="all")
    ap.add_argument("--out", default=None)
    ap.add_argument("--merge", action="store_true")
    ap.add_argument("--fp16", action="store_true", help="fp16 operands (the pipeline's autocast caller: the exact kernel)")
    ap.add_argument("--vbf16", action="store_true",
                    help="fp16 q / k with a bf16 V third (GP_FMT_F16_VBF16: the fp16 caller's fused-QKV product pair)")
    args = ap.parse_args()
    if args.merge:
        args.branches = "all"
    prod = _hip.load_library()
    libs = []
    for p in args.libs.split(","):
        libs.append((p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p) if not os.path.isabs(p) else p)))
    H, D, L = 16, 48, args.L
    E = H * D
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(L, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    act = torch.float16 if (args.fp16 or args.vbf16) else torch.bfloat16
    vb = qkv[:, 2 * E:].to(torch.bfloat16)
    qkv = qkv.to(act)
    if args.vbf16:      # the V third holds bf16 bits, as the fp16 caller's QKV GEMM writes them
        qkv[:, 2 * E:].view(torch.int16).copy_(vb.view(torch.int16))
    sets = []
    for b in args.branches.split(","):
        sel = list(range(5)) if b == "all" else [int(b)]
        sets.append((b, [SEGS[i] for i in sel], [RATIOS[i] for i in sel]))
    scratch = {name: runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, s, r, act) for name, s, r in sets}
    flops = {name: runtime.attention_valid_flops(L, s, r, H, D) for name, s, r in sets}
    if args.merge:     # report GB/s of the merge's algorithmic bytes instead
        flops = {name: 1e-3 * L * ((2 * E + 4 * H) * sum(1.0 / x for x in r) + 2 * E) for name, _, r in sets}
    times = {(p, name): [] for p, _ in libs for name, _, _ in sets}
    ident = {}
    ref = {}
    merge_out = {}
    ln_w = 1 + 0.1 * torch.randn(E, device="cuda", generator=g)
    ln_b = 0.1 * torch.randn(E, device="cuda", generator=g)
    for rnd in range(args.rounds + 1):
        for p, lib in libs:
            _hip._lib = lib
            for name, s, r in sets:
                sc = scratch[name]
                run = lambda: _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, s, r,  # noqa
                                                    sc.outs, sc.lses, 0.0, True, v_bf16=args.vbf16)
                if args.merge:
                    if name not in merge_out:       # attention outputs once, from the product build
                        _hip._lib = prod
                        run()
                        torch.cuda.synchronize()
                        _hip._lib = lib
                        merge_out[name] = torch.empty(L, E, device="cuda", dtype=torch.bfloat16)
                    mo = merge_out[name]
                    run = lambda: _hip.branch_merge_ln(sc.outs, sc.lses, s, r, 1, L, H, D, ln_w, ln_b, 1e-5, mo)  # noqa
                    if rnd == 0:
                        run()
                        torch.cuda.synchronize()
                        if name not in ref:
                            ref[name] = [mo.clone()]
                        else:
                            ident[(p, name)] = torch.equal(mo.view(torch.uint8), ref[name][0].view(torch.uint8))
                            if not ident[(p, name)]:
                                print("max |diff| vs first:", (mo.float() - ref[name][0].float()).abs().max().item())
                        continue
                if rnd == 0:       # warm-up + outputs
                    run()
                    torch.cuda.synchronize()
                    outs = [t.clone() for t in sc.outs + sc.lses]
                    if name not in ref:
                        ref[name] = outs
                    else:
                        ident[(p, name)] = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8))
                                               for a, b in zip(outs, ref[name]))
                        if not ident[(p, name)]:       # a variant with other arithmetic: how far off
                            no = len(sc.outs)
                            dif = [(a.float() - b.float()).abs().nan_to_num(0.0, 0.0, 0.0).max().item()
                                   for a, b in zip(outs, ref[name])]
                            print("%s br=%s: max |d o| %.3e, max |d lse| %.3e vs the first build" %
                                  (p, name, max(dif[:no]), max(dif[no:])))
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[(p, name)].append(e0.elapsed_time(e1) / args.iters)
    _hip._lib = prod
    res = []
    for (p, name), ts in times.items():
        med, mn = statistics.median(ts), min(ts)
        res.append({"lib": p, "branches": name, "median_ms": round(med, 4), "min_ms": round(mn, 4),
                    "tflops_median": round(flops[name] / med / 1e9, 1), "bit_identical_to_first": ident.get((p, name), True)})
        print("%-40s br=%-4s median %.4f ms  min %.4f ms  %7.1f %s  ident=%s" % (
            p, name, med, mn, flops[name] / med / 1e9, "GB/s" if args.merge else "TF/s",
            ident.get((p, name), True)), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"L": L, "rounds": args.rounds, "iters": args.iters, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
