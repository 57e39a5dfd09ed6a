"""Debug: where the varlen merge differs from the single-slide merge (tests/test_gpu_batch.py
test_varlen_attention_and_merge_bit_exact_per_slide), with the inputs of the first differing token."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip, runtime  # noqa: E402

SEGS, RATIOS = [1024, 5792, 32768, 185363, 1048576], [1, 2, 4, 8, 16]
H, D, E = 16, 48, 768
Ls = [1025, 2897, 700, 6001, 12000]
T = sum(Ls)
g = torch.Generator(device="cuda").manual_seed(5)
qkv = torch.randn(T, 3 * E, device="cuda", generator=g)
qkv[:, :E] *= 0.35
qkv = qkv.to(torch.bfloat16)
vs = runtime.VarlenScratch(torch.device("cuda"), Ls, H, D, SEGS, RATIOS, qkv)
for t in vs.outs + vs.lses:
    t.zero_()
_hip.dilated_attn_fwd_varlen(vs.plan, True)
ln_w = torch.rand(E, device="cuda") + 0.5
ln_b = torch.randn(E, device="cuda") * 0.1
for use_ln in (False, True):
    merged = torch.empty(T, E, dtype=qkv.dtype, device="cuda")
    _hip.branch_merge_ln_varlen(vs.plan, ln_w if use_ln else None, ln_b if use_ln else None, 1e-5, merged)
    t0 = 0
    for L in Ls:
        rows = qkv[t0:t0 + L]
        sc = runtime.AttentionScratch(torch.device("cuda"), 1, L, H, D, SEGS, RATIOS, qkv.dtype)
        for t in sc.outs + sc.lses:
            t.zero_()
        _hip.dilated_attn_fwd(rows, rows[:, E:], rows[:, 2 * E:], 3 * E, 1, L, H, D, SEGS, RATIOS, sc.outs, sc.lses,
                              0.0, True)
        ref = torch.empty(L, E, dtype=qkv.dtype, device="cuda")
        _hip.branch_merge_ln(sc.outs, sc.lses, SEGS, RATIOS, 1, L, H, D, ln_w if use_ln else None,
                             ln_b if use_ln else None, 1e-5, ref)
        torch.cuda.synchronize()
        got = merged[t0:t0 + L]
        bad = (got.view(torch.int16) != ref.view(torch.int16))
        nb = int(bad.sum())
        print("ln=%s L=%d differing elements %d rows %d" % (use_ln, L, nb, int(bad.any(1).sum())))
        if nb:
            r, c = [int(v) for v in bad.nonzero()[0]]
            cols = bad[r].nonzero().flatten().tolist()
            print("   first row %d cols %s ... (%d)" % (r, cols[:16], len(cols)))
            print("   got", got[r, cols[:6]].float().tolist(), "ref", ref[r, cols[:6]].float().tolist())
        t0 += L
