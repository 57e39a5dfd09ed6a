"""CPU stand-ins for the HIP entry points the sequence-parallel forward calls (TEST ONLY).

They restate each kernel's contract in torch fp32 from its header comment
(include/gigapath_hip.h) and ASSERT every access the kernel would make is inside the tensor
it was given, and that the merge only reads branch rows the attention wrote.  Installed with
`install(monkeypatch)`, they let tests run LongNetViT._forward_sp end to end on CPU under a gloo
world (tests/test_seqpar.py) -- a check of the host-side sharding logic, not of the kernels.
"""
import math

import numpy as np
import torch

import oracle as orc

LN2 = math.log(2.0)
_written = {}      # o.data_ptr() -> bool tensor [rows of (segment, row, head)] written by attention


def _ln(x, w, b, eps):
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)


def coords_to_pos(coords, grid, tile_size, pos_out, err_count):
    c = coords.reshape(-1, 2).double().numpy() if coords.dtype == torch.float64 else coords.reshape(-1, 2).numpy()
    pos = orc.coords_to_pos(c[None], grid, tile_size)[0]
    assert pos_out.numel() >= len(pos)
    pos_out.view(-1)[:len(pos)] = torch.from_numpy(pos)
    if err_count is not None:
        nrows = grid * grid + 1
        err_count += int(((pos < -nrows) | (pos >= nrows)).sum())


def posembed_cls_ln(xp, pos, tab, cls, B, N, E, G, ln_w, ln_b, eps, x_out, ln_out, row_mean=None):
    has = cls is not None
    rows = B * (N + has)
    assert x_out.shape[0] >= rows and (ln_out is None or ln_out.shape[0] >= rows)
    assert xp.shape[0] >= B * N and pos.numel() >= B * N
    tabn = tab.numpy()
    pe = torch.from_numpy(orc.pos_embed_rows(pos.view(-1)[:B * N].numpy()[None], tabn, G)[0])
    v = xp[:B * N].float() + pe
    out = torch.cat([cls.view(1, E).float(), v], 0) if has else v
    x_out[:rows] = out
    if row_mean is not None:
        assert row_mean.numel() >= rows
        row_mean.view(-1)[:rows] = out.mean(1)
    if ln_w is not None:
        ln_out[:rows] = _ln(out, ln_w, ln_b, eps).to(ln_out.dtype)


def layernorm_f32(x, row_stride, ln_w, ln_b, eps, out, rows, cols):
    flat = x.reshape(-1)
    assert (rows - 1) * row_stride + cols <= flat.numel()
    src = torch.stack([flat[r * row_stride:r * row_stride + cols] for r in range(rows)])
    out.view(-1)[:rows * cols] = _ln(src, ln_w, ln_b, eps).reshape(-1)


def mean_tokens(x, B, L, E, start, out):
    assert x.numel() >= B * L * E
    out.view(B, E)[:] = x.reshape(-1)[:B * L * E].view(B, L, E)[:, start:].mean(1)


def residual_layernorm(x, y, bias, ln_w, ln_b, eps, ln_out, rows, cols):
    assert x.shape[0] >= rows and y.shape[0] >= rows
    v = x[:rows] + y[:rows].float() + (bias.float() if bias is not None else 0)
    x[:rows] = v
    if ln_w is not None:
        ln_out[:rows] = _ln(v, ln_w, ln_b, eps).to(ln_out.dtype)


def residual2_layernorm(x, y1, b1, y2, b2, ln_w, ln_b, eps, ln_out, rows, cols):
    """gp_residual2_layernorm: x1 = x + (y1 + b1) (x unchanged unless y2), x2 = x1 + (y2 + b2) -> x."""
    assert x.shape[0] >= rows and y1.shape[0] >= rows
    v = x[:rows] + (y1[:rows].float() + (b1.float() if b1 is not None else 0))
    if y2 is not None:
        v = v + (y2[:rows].float() + (b2.float() if b2 is not None else 0))
        x[:rows] = v
    if ln_w is not None:
        ln_out[:rows] = _ln(v, ln_w, ln_b, eps).to(ln_out.dtype)


def gelu_layernorm(h, ln_w, ln_b, eps, out, rows, cols):
    v = torch.nn.functional.gelu(h[:rows].float())
    out[:rows] = _ln(v, ln_w, ln_b, eps).to(out.dtype)


def ffn_fc1_gelu(a, w1, b1, h, stats):
    """gp_ffn_fc1_gelu: h = act(gelu(act(a . w1^T + b1))), stats[g][m] = (mean, M2) of h's 256-column group g."""
    M, F = a.shape[0], w1.shape[0]
    assert h.shape[0] >= M and h.shape[1] == F and F % 256 == 0 and stats.numel() >= (F // 256 + 1) * M * 2
    v = (a.float() @ w1.float().t() + (b1.float() if b1 is not None else 0)).to(h.dtype)
    g = torch.nn.functional.gelu(v.float()).to(h.dtype)
    h[:M] = g
    gf = g.float().view(M, F // 256, 256)
    mean = gf.mean(-1)
    st = stats.view(-1)[:(F // 256) * M * 2].view(F // 256, M, 2)
    st[..., 0] = mean.t()
    st[..., 1] = ((gf - mean[..., None]) ** 2).sum(-1).t()


def ffn_fc2_ln(h, w2g, stats, c, d, eps, y, ws=None):
    """gp_ffn_fc2_ln: y = act(rstd (h . w2g^T - mean c) + d), the row statistics Chan-merged from stats."""
    M, F = h.shape
    N = w2g.shape[0]
    assert y.shape[0] >= M and y.shape[1] == N and c.numel() == N and d.numel() == N
    st = stats.view(-1)[:(F // 256) * M * 2].view(F // 256, M, 2)
    mg = st[..., 0]
    mean = mg.mean(0)
    m2 = st[..., 1].sum(0) + 256.0 * ((mg - mean) ** 2).sum(0)
    rstd = torch.rsqrt(m2 / F + eps)
    acc = h.float() @ w2g.float().t()
    y[:M] = (rstd[:, None] * (acc - mean[:, None] * c.float()[None]) + d.float()[None]).to(y.dtype)


def _merge_stats(stats, nst, M, eps, s_in, s_out):
    """row_stats_kernel: Chan-merge planes 0 .. nst-1 into plane nst; s_out = s_in + mean."""
    st = stats.view(-1)[:(nst + 1) * M * 2].view(nst + 1, M, 2)
    mg = st[:nst, :, 0]
    mean = mg.mean(0)
    m2 = st[:nst, :, 1].sum(0) + 256.0 * ((mg - mean) ** 2).sum(0)
    rstd = torch.rsqrt(m2 / (256 * nst) + eps)
    st[nst, :, 0] = mean
    st[nst, :, 1] = rstd
    if s_out is not None:
        s_out.view(-1)[:M] = (s_in.view(-1)[:M] if s_in is not None else 0) + mean
    return mean, rstd


def _resid_out(x, v, shift, gamma, xb, xstats):
    """The residual epilogue: x = v; xb = act(gamma (x - shift)); xstats[g][m] = (mean, M2) of x - shift."""
    M, N = v.shape
    x[:M, :N] = v
    if gamma is None:
        return
    assert shift.numel() >= M and xb.shape[0] >= M and xb.shape[1] >= N and xstats.numel() >= N // 256 * M * 2
    dlt = v - shift.view(-1)[:M, None]
    xb[:M, :N] = (dlt * gamma.float()[None]).to(xb.dtype)
    dg = dlt.view(M, N // 256, 256)
    mean = dg.mean(-1)
    st = xstats.view(-1)[:(N // 256) * M * 2].view(N // 256, M, 2)
    st[..., 0] = mean.t()
    st[..., 1] = ((dg - mean[..., None]) ** 2).sum(-1).t()


def _producer_merge(xstats, N, M, shift, eps_next, s_out):
    """ABI 9: the residual producer merges the next LN's statistics itself when s_out is given."""
    if s_out is not None:
        assert eps_next is not None and eps_next > 0
        _merge_stats(xstats, N // 256, M, eps_next, shift, s_out)


def _merged_plane(stats, nst, M):
    """(mean, rstd) of plane nst, already merged by the producer (merged=True)."""
    st = stats.view(-1)[:(nst + 1) * M * 2].view(nst + 1, M, 2)
    return st[nst, :, 0].clone(), st[nst, :, 1].clone()


def linear_resid(a, w, bias, x, shift, gamma, xb, xstats, ws=None, eps_next=None, s_out=None):
    M, N = a.shape[0], w.shape[0]
    y = a.float() @ w.float().t() + (bias.float() if bias is not None else 0)
    _resid_out(x, x[:M, :N] + y, shift, gamma, xb, xstats)
    _producer_merge(xstats, N, M, shift, eps_next, s_out)


def linear_ln(a, w, stats, nst, c, d, eps, s_in, s_out, out, ws=None, v_bf16=False, merged=False):
    assert not v_bf16          # (the bf16 model: no bf16 V third in an fp16 buffer)
    M = a.shape[0]
    mean, rstd = _merged_plane(stats, nst, M) if merged else _merge_stats(stats, nst, M, eps, s_in, s_out)
    acc = a.float() @ w.float().t()
    out[:M] = (rstd[:, None] * (acc - mean[:, None] * c.float()[None]) + d.float()[None]).to(out.dtype)


def ffn_fc1_gelu_ln(a, w1, xstats, nst, c1, d1, eps, s_in, s_out, h, hstats, merged=False):
    M, F = a.shape[0], w1.shape[0]
    mean, rstd = _merged_plane(xstats, nst, M) if merged else _merge_stats(xstats, nst, M, eps, s_in, s_out)
    v = (rstd[:, None] * (a.float() @ w1.float().t() - mean[:, None] * c1.float()[None]) + d1.float()[None])
    g = torch.nn.functional.gelu(v.to(h.dtype).float()).to(h.dtype)
    h[:M] = g
    gf = g.float().view(M, F // 256, 256)
    gm = gf.mean(-1)
    st = hstats.view(-1)[:(F // 256) * M * 2].view(F // 256, M, 2)
    st[..., 0] = gm.t()
    st[..., 1] = ((gf - gm[..., None]) ** 2).sum(-1).t()


def ffn_fc2_ln_resid(h, w2g, hstats, c, d, eps, x, shift, gamma, xb, xstats, ws=None, eps_next=None, s_out=None):
    M, F = h.shape
    N = w2g.shape[0]
    mean, rstd = _merge_stats(hstats, F // 256, M, eps, None, None)
    y = rstd[:, None] * (h.float() @ w2g.float().t() - mean[:, None] * c.float()[None]) + d.float()[None]
    _resid_out(x, x[:M, :N] + y, shift, gamma, xb, xstats)
    _producer_merge(xstats, N, M, shift, eps_next, s_out)


def dilated_sparsify(src, src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, segs, ratios, dsts, dst_bases=None):
    assert src.shape[0] >= n_tok and src.shape[1] == src_row_stride
    p = torch.arange(tok_lo, tok_lo + n_tok)
    for b, (sl, r) in enumerate(zip(segs, ratios)):
        base = 0 if dst_bases is None else dst_bases[b]
        s, C = min(sl, L), (H // r) * D
        j = (p % s) % r
        cols = j[:, None] * C + torch.arange(C)[None, :]
        rows = p - base
        assert rows.min() >= 0 and rows.max() < dsts[b].shape[0] and dsts[b].shape[1] == 2 * C
        dsts[b][rows, :C] = torch.gather(src[:n_tok, k_col:k_col + H * D], 1, cols)
        dsts[b][rows, C:] = torch.gather(src[:n_tok, v_col:v_col + H * D], 1, cols)


def dilated_sparsify_dests(src, src_row_stride, k_col, v_col, tok_lo, n_tok, L, H, D, segs, ratios, dests):
    assert src.shape[0] >= n_tok and src.shape[1] == src_row_stride
    p = torch.arange(tok_lo, tok_lo + n_tok)
    for b, (sl, r) in enumerate(zip(segs, ratios)):
        s, C = min(sl, L), (H // r) * D
        j = (p % s) % r
        cols = j[:, None] * C + torch.arange(C)[None, :]
        krow = torch.gather(src[:n_tok, k_col:k_col + H * D], 1, cols)
        vrow = torch.gather(src[:n_tok, v_col:v_col + H * D], 1, cols)
        for lo, hi, t, off in dests[b]:
            sel = (p >= lo) & (p < hi)
            rows = off + (p[sel] - lo)
            assert t.shape[1] == 2 * C and (len(rows) == 0 or (rows.min() >= 0 and rows.max() < t.shape[0]))
            t[rows, :C] = krow[sel].to(t.dtype)
            t[rows, C:] = vrow[sel].to(t.dtype)


def attn_branch(sl, r, k, v, kv_row_stride, kv_tok_base, kv_sparse_cols, o, lse, key_part=0, key_parts=1):
    return dict(sl=sl, r=r, k=k, v=v, stride=kv_row_stride, base=kv_tok_base, sparse=kv_sparse_cols, o=o, lse=lse,
                kp=key_part, kparts=key_parts)


def _kv_tensor(k, v, stride, sparse, H, D, r):
    """Resolve (k tensor, v pointer) into two [rows, cols] views of the same buffer."""
    assert isinstance(k, torch.Tensor) and k.stride(0) == stride and k.stride(1) == 1
    C = (H // r) * D if sparse else H * D
    vp = v if isinstance(v, int) else v.data_ptr()
    off = (vp - k.data_ptr()) // k.element_size()
    assert 0 <= off and off + C <= k.shape[1]
    return k[:, :C], k[:, off:off + C]


def dilated_attn_fwd_ex(q, q_row_stride, q_tok_base, B, L, H, D, win_lo, win_hi, branches, softmax_scale=0.0,
                        q_log2_prescaled=False, v_bf16=False):
    assert B == 1 and not v_bf16 and q.shape[1] == q_row_stride
    scale = 1.0 if q_log2_prescaled else (softmax_scale or D ** -0.5) / LN2   # -> log2-domain logits
    for br in branches:
        geo = orc.branch_geometry(L, br["sl"], br["r"], H)
        s, r, m, g, nseg, hpg = geo["s"], geo["r"], geo["m"], geo["g"], geo["nseg"], geo["hpg"]
        kt, vt = _kv_tensor(br["k"], br["v"], br["stride"], br["sparse"], H, D, r)
        o = br["o"].view(nseg, m, H, D)
        lse = br["lse"].view(nseg, H, m)
        wr = _written.setdefault(br["o"].data_ptr(), torch.zeros(nseg, m, H, dtype=torch.bool))
        for n in range(win_lo // g, (win_hi - 1) // g + 1):
            for h in range(H):
                j = h // hpg
                base = n * g + j
                i_lo = max(0, -(-(win_lo - base) // r)) if win_lo > base else 0
                i_hi = min(m, -(-(win_hi - base) // r)) if win_hi > base else 0
                if i_hi <= i_lo:
                    continue
                rem = min(L - n * s, s) - j
                c = -(-rem // r) if rem > 0 else 0
                col = (h % hpg) * D if br["sparse"] else h * D
                # key part kp of kparts (GpAttnBranch.key_parts): 64-key tiles [t_lo, t_hi); pads in the last
                P, kp = max(1, br["kparts"]), br["kp"]
                nt = -(-c // 64)
                k_lo, k_hi = 64 * (nt * kp // P), min(c, 64 * (nt * (kp + 1) // P))
                last = kp == P - 1
                ktok = n * s + j + r * torch.arange(k_lo, max(k_lo, k_hi))
                krow = ktok - br["base"]
                assert len(krow) == 0 or (krow.min() >= 0 and krow.max() < kt.shape[0]), ("k rows", n, h)
                K, V = kt[krow, col:col + D].float(), vt[krow, col:col + D].float()
                i = torch.arange(i_lo, i_hi)
                qtok = n * s + j + r * i
                valid = (i * r + j < min(L - n * s, s))
                qrow = (qtok - q_tok_base)
                assert (qrow[valid] >= 0).all() and (qrow[valid] < q.shape[0]).all(), ("q rows", n, h)
                Q = torch.zeros(len(i), D)
                Q[valid] = q[qrow[valid], h * D:(h + 1) * D].float()
                s2 = (Q @ K.T) * scale                               # log2-domain logits
                npad = m - c if last else 0
                full = torch.cat([s2 * LN2, torch.zeros(len(i), npad)], 1)
                if full.shape[1] == 0:                               # an empty part: o = 0, lse = -inf
                    o[n, i_lo:i_hi, h] = 0
                    lse[n, h, i_lo:i_hi] = -float("inf")
                    wr[n, i_lo:i_hi, h] = True
                    continue
                l_ = torch.logsumexp(full, 1)
                p = torch.exp(s2 * LN2 - l_[:, None])
                o[n, i_lo:i_hi, h] = (p @ V).to(o.dtype)
                lse[n, h, i_lo:i_hi] = l_
                wr[n, i_lo:i_hi, h] = True


def branch_merge_ln_window(outs, lses, segs, ratios, B, L, tok_lo, n_tok, H, D, ln_w, ln_b, eps, out):
    assert B == 1 and out.shape[0] >= n_tok
    E = H * D
    p = np.arange(tok_lo, tok_lo + n_tok)
    o_d, l_d = [], []
    for o, l, sl, r in zip(outs, lses, segs, ratios):
        geo = orc.branch_geometry(L, sl, r, H)
        nseg, m, g, hpg = geo["nseg"], geo["m"], geo["g"], geo["hpg"]
        n, t = p // g, p % g
        i, jj = t // r, t % r
        ov = torch.zeros(n_tok, H, D)
        lv = torch.full((n_tok, H), -1e8)
        wr = _written[o.data_ptr()]
        for h in range(H):
            cov = (h // hpg) == jj
            nn_, ii = torch.from_numpy(n[cov]), torch.from_numpy(i[cov])
            assert wr[nn_, ii, h].all(), "merge reads a branch row the attention did not write"
            ov[torch.from_numpy(cov), h] = o.view(nseg, m, H, D)[nn_, ii, h].float()
            lvals = l.view(nseg, H, m)[nn_, h, ii]
            lv[torch.from_numpy(cov), h] = torch.where(lvals == 0, torch.full_like(lvals, -1e8), lvals)
        o_d.append(ov)
        l_d.append(lv)
    st = torch.stack(l_d, 0)
    w = torch.softmax(st, 0)
    acc = sum(od * wi[..., None] for od, wi in zip(o_d, w))
    acc = acc.reshape(n_tok, E)
    if ln_w is not None:
        acc = _ln(acc, ln_w, ln_b, eps)
    out[:n_tok] = acc.to(out.dtype)


def install():
    """Replace the _hip entry points in this process (call in a test subprocess only)."""
    from gigapath import _hip
    for name in ("coords_to_pos", "posembed_cls_ln", "layernorm_f32", "mean_tokens", "residual_layernorm", "residual2_layernorm",
                 "gelu_layernorm", "ffn_fc1_gelu", "ffn_fc2_ln", "linear_resid", "linear_ln", "ffn_fc1_gelu_ln",
                 "ffn_fc2_ln_resid", "dilated_sparsify", "dilated_sparsify_dests", "attn_branch", "dilated_attn_fwd_ex",
                 "branch_merge_ln_window"):
        setattr(_hip, name, globals()[name])
    _written.clear()
