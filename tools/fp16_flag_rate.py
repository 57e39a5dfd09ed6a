"""Rows the no-max / tile-0-offset fast attention kernels flag for the exact fixup pass, and what the
fixup then costs (ADVICE r02 on gp_attn.hip's fixup pass).

    make -C tools/attn_lab tune NAME=f16fast DEFS="-DGP_ATTN_FP16_EXACT=0"
    make -C tools/attn_lab tune NAME=fix32 DEFS="-DGP_ATTN_FIX_ITEMS=32"
    make -C tools/attn_lab tune NAME=nofix DEFS="-DGP_ATTN_FP16_EXACT=0 -DGP_ATTN_NOFIX=1"
    python tools/fp16_flag_rate.py [--fmt fp16|bf16] [--L 70001] [--out file.json]

Builds of the same source, one process, interleaved rounds:
  prod      the product: fp16 = kModeExact (exact running max, no fixup; round 3); bf16 = kModeFast
            (p = 2^s, no max, no offset) + kModeFix with one block per work item (round 3);
  f16fast   (fp16 only) the fp16 fast mode: kModeFast with p = 2^(s - m0), m0 = tile 0's row max,
            + kModeFix (one block per item);
  fix32     (bf16 only) round 2's fixup pass: 32 items per block, flagged ones recomputed in turn;
  nofix     kModeFast alone: flagged rows keep the lse marker 0x7fc0dead, which this tool counts.
Inputs (one 70k layer's q / k / v, q pre-scaled by D^-1/2 log2 e as the product's QKV weight):
  random-init   q, k, v ~ N(0, 1), q x 0.35 (the scale the model's random-init q projection gives);
  sharp x s     the same with q x 0.35 s (scores s times larger, as trained attention can be sharper);
  worst         every head's scores climb per 64-key tile past the fast kernel's range (fp16: +24
                log2 units per tile over tile 0's max; bf16: +120), so nearly every row is flagged.
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
MARK = 0x7fc0dead


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=70001)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--libs", default=None, help="comma-separated lab builds (tools/attn_lab/liblab_<name>.so) "
                    "to time beside prod; default f16fast,nofix (fp16) / fix32,nofix (bf16); nofix is required")
    ap.add_argument("--scales", default=None, help="comma-separated q sharpness factors")
    ap.add_argument("--fmt", choices=["fp16", "bf16"], default="fp16",
                    help="bf16: the product's no-max bf16 kernel (flags rows whose sum leaves [2^-100, 2^100])")
    args = ap.parse_args()
    act = torch.float16 if args.fmt == "fp16" else torch.bfloat16
    prod = _hip.load_library()
    libs = [("prod", prod)]
    names = args.libs.split(",") if args.libs else (["f16fast", "nofix"] if args.fmt == "fp16" else ["fix32", "nofix"])
    assert "nofix" in names
    for name in names:
        libs.append((name, _hip.load_library(os.path.join(ROOT, "tools", "attn_lab", "liblab_%s.so" % name))))
    H, D, L = 16, 48, args.L
    E = H * D
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(L, 3 * E, device="cuda", generator=g)
    cases = []
    scales = ((1.0, 2.0, 4.0, 8.0) if args.fmt == "fp16" else (1.0, 4.0, 8.0, 12.0, 16.0))
    if args.scales:
        scales = tuple(float(x) for x in args.scales.split(","))
    for s in scales:
        x = base.clone()
        x[:, :E] *= 0.35 * s
        cases.append(("random-init" if s == 1.0 else "sharp x%g" % s, x.to(act)))
    w = base.clone()
    w[:, :E] = 0.0
    w[:, E:2 * E] = 0.0
    for h in range(H):
        w[:, h * D] = 8.0
        w[:, E + h * D] = (torch.arange(L, device="cuda") % 1024 // 64).float() * 3.0   # +24 log2 per tile
    if args.fmt == "bf16":       # bf16 flags only past 2^100: climb 120 log2 units per tile instead
        for h in range(H):
            w[:, E + h * D] = (torch.arange(L, device="cuda") % 1024 // 64).float() * 15.0
    cases.append(("worst", w.to(act)))
    sc = runtime.AttentionScratch(dev, 1, L, H, D, SEGS, RATIOS, act)
    res = []
    for nm, qkv in cases:
        # flag count: the nofix build leaves the marker in every flagged row
        _hip._lib = dict(libs)["nofix"]
        for t in sc.lses:
            t.zero_()
        _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, sc.outs, sc.lses,
                              0.0, True)
        torch.cuda.synchronize()
        flagged = sum(int((t.view(torch.int32) == MARK).sum().item()) for t in sc.lses)
        rows_total = sum(int((t != 0).sum().item()) for t in sc.lses)    # rows the kernel wrote
        times = {p: [] for p, _ in libs}
        outs = {}
        for rnd in range(args.rounds + 1):
            for p, lib in libs:
                _hip._lib = lib
                run = lambda: _hip.dilated_attn_fwd(qkv, qkv[:, E:], qkv[:, 2 * E:], 3 * E, 1, L, H, D, SEGS,  # noqa
                                                    RATIOS, sc.outs, sc.lses, 0.0, True)
                if rnd == 0:
                    run()
                    torch.cuda.synchronize()
                    outs[p] = [t.clone() for t in sc.outs + sc.lses]
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / args.iters)
        _hip._lib = prod
        n = len(sc.outs)
        row = {"input": nm, "flagged_rows": flagged, "rows": rows_total, "flagged_frac": flagged / rows_total}
        for p, _ in libs[1:]:
            if p == "nofix":
                continue
            row["prod_vs_%s_max_abs_o" % p] = max((a.float() - b.float()).abs().max().item()
                                                  for a, b in zip(outs["prod"][:n], outs[p][:n]))
            row["prod_vs_%s_max_abs_lse" % p] = max((a - b).abs().max().item()
                                                    for a, b in zip(outs["prod"][n:], outs[p][n:]))
        for p, ts in times.items():
            row[p + "_ms"] = round(statistics.median(ts), 4)
        res.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"L": L, "rounds": args.rounds, "iters": args.iters, "results": res}, f, indent=1)


if __name__ == "__main__":
    main()
