"""Where two builds' (or the varlen and single-slide) branch merges disagree, for one packed batch.

    python tools/merge_diff.py --libs prod,tools/attn_lab/liblab_premerge.so

For each library: the packed (varlen) merge and the per-slide merge of the same attention outputs;
prints, per slide, how many rows / columns differ between every pair and the first few positions.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="prod")
    ap.add_argument("--sizes", default="1025,2897,700")
    args = ap.parse_args()
    prod = _hip.load_library()
    libs = [(p, prod if p == "prod" else _hip.load_library(os.path.join(ROOT, p))) for p in args.libs.split(",")]
    H, D, E = 16, 48, 768
    Ls = [int(x) for x in args.sizes.split(",")]
    T = sum(Ls)
    g = torch.Generator(device="cuda").manual_seed(5)
    qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
    qkv[:, :E] *= 0.35
    qkv = qkv.to(torch.bfloat16)
    ln_w = torch.rand(E, device="cuda", generator=g) + 0.5
    ln_b = torch.randn(E, device="cuda", generator=g) * 0.1
    vs = runtime.VarlenScratch(torch.device("cuda"), Ls, H, D, SEGS, RATIOS, qkv)
    for t in vs.outs + vs.lses:
        t.zero_()
    _hip.dilated_attn_fwd_varlen(vs.plan, True)
    scs = []
    t0 = 0
    for L in Ls:
        rows = qkv[t0:t0 + L]
        sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, SEGS, RATIOS)
        for t in sc.outs + sc.lses:
            t.zero_()
        _hip.dilated_attn_fwd(rows, rows[:, E:], rows[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, sc.outs, sc.lses,
                              0.0, True)
        scs.append(sc)
        t0 += L
    res = {}
    for p, lib in libs:
        _hip._lib = lib
        packed = torch.empty(T, E, dtype=torch.bfloat16, device="cuda")
        _hip.branch_merge_ln_varlen(vs.plan, ln_w, ln_b, 1e-5, packed)
        single = []
        for L, sc in zip(Ls, scs):
            o = torch.empty(L, E, dtype=torch.bfloat16, device="cuda")
            _hip.branch_merge_ln(sc.outs, sc.lses, SEGS, RATIOS, 1, L, H, D, ln_w, ln_b, 1e-5, o)
            single.append(o)
        torch.cuda.synchronize()
        res[(p, "varlen")] = torch.split(packed, Ls)
        res[(p, "single")] = single
    _hip._lib = prod
    keys = list(res)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            for s, L in enumerate(Ls):
                a, b = res[keys[i]][s].float(), res[keys[j]][s].float()
                ne = (a != b) & ~(torch.isnan(a) & torch.isnan(b))
                if ne.any():
                    r, c = torch.nonzero(ne, as_tuple=True)
                    print("%s vs %s  L=%d: %d elems differ in %d rows, max|d| %.4g, nan a/b %d/%d, rows %s cols %s" % (
                        keys[i], keys[j], L, int(ne.sum()), len(torch.unique(r)), float((a - b)[ne].abs().max()),
                        int(torch.isnan(a).sum()), int(torch.isnan(b).sum()), torch.unique(r)[:8].tolist(),
                        torch.unique(c)[:8].tolist()), flush=True)
                else:
                    print("%s vs %s  L=%d: identical" % (keys[i], keys[j], L), flush=True)


if __name__ == "__main__":
    main()
