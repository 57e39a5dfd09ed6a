import sys, os
sys.path.insert(0, "tests"); sys.path.insert(0, "."); sys.path.insert(0, "prov-gigapath-replication_amd")
import numpy as np, torch
import test_gpu_kernels as T
import oracle as orc
h = T._hip()
for impl in ("1", "2"):
    os.environ["GP_ATTN_IMPL"] = impl
    for name, B, L, segs, ratios in T.ATTN_CASES:
        H, D = 16, 48; E = H * D
        qkv = T._rand_qkv(B, L, E, seed=L)
        outs, lses = T._run_attn(h, qkv, B, L, H, D, segs, ratios)
        q, k, v = (qkv[:, i * E:(i + 1) * E].float().view(B, L, H, D) for i in range(3))
        for b, (sl, r) in enumerate(zip(segs, ratios)):
            o_ref, l_ref = orc.branch_attention(q, k, v, sl, r)
            geo = orc.branch_geometry(L, sl, r, H); nseg, m = geo["nseg"], geo["m"]
            o = outs[b].float().cpu().view(B, nseg, m, H, D).permute(0, 1, 3, 2, 4)
            l = lses[b].cpu().view(B, nseg, H, m)
            need = T._rows_needed(L, sl, r, H)
            mask = torch.from_numpy(np.arange(m)[None, None, :] < need[:, :, None]).unsqueeze(0).expand(B, -1, -1, -1)
            dl = (l - l_ref).abs()[mask]
            print(impl, name, b, "do %.2e" % (o - o_ref).abs()[mask].max().item(), "dl max %.2e mean %.2e" % (dl.max().item(), dl.mean().item()),
                  "nan", int((~torch.isfinite(l[mask])).sum()))
