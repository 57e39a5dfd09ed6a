"""CPU fp32 restatement of the Prov-GigaPath slide encoder (LongNet dilated attention).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Integer bookkeeping is numpy;
floating-point math is torch fp32 on the CPU.  Every function cites the reference
file:line it restates (paths relative to the reference repo root).

The attention here is deliberately *literal*: zero-padded keys/queries are materialised
as zero vectors and take part in the softmax exactly as they do in the reference
(``dilated_attention.py:85-91`` pads, ``multihead_attention.py:103`` runs flash-attention
without a mask).  The HIP product treats the padded keys analytically; this oracle
checks that shortcut instead of sharing it.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

__all__ = [
    "ARCHS", "arch_config", "segment_schedule", "padding_to_multiple_of",
    "sincos_axis_table", "coords_to_pos", "pos_embed_rows", "branch_geometry",
    "gather_index", "scatter_index", "dilated_gather", "branch_attention",
    "merge_branches", "dilated_attention", "encoder_layer", "slide_encoder_forward",
    "state_dict_keys", "make_weights", "synthetic_slide", "weights_sha256",
]

# gigapath/slide_encoder.py:255-270 + torchscale/model/LongNetConfig.py (16 heads, FFN = 4E)
ARCHS = {
    "gigapath_slide_enc12l768d": dict(embed_dim=768, depth=12, heads=16),
    "gigapath_slide_enc24l1024d": dict(embed_dim=1024, depth=24, heads=16),
    "gigapath_slide_enc12l1536d": dict(embed_dim=1536, depth=12, heads=16),
}


def arch_config(arch: str, max_wsi_size: int = 262144, tile_size: int = 256,
                slide_ngrids: int = 1000, in_chans: int = 1536) -> dict:
    a = dict(ARCHS[arch])
    a["ffn_dim"] = 4 * a["embed_dim"]
    a["segment_length"] = segment_schedule(max_wsi_size, tile_size)
    a["dilated_ratio"] = [1, 2, 4, 8, 16]          # LongNet.py:92 default
    a["slide_ngrids"] = slide_ngrids
    a["tile_size"] = tile_size
    a["in_chans"] = in_chans
    a["ln_eps"] = 1e-5                             # architecture/config.py:44 (layernorm_eps)
    a["norm_eps"] = 1e-6                           # slide_encoder.py:258 (final norm)
    return a


def segment_schedule(max_wsi_size: int = 262144, tile_size: int = 256) -> List[int]:
    """slide_encoder.py:137-154 — 5 segment lengths, 2**linspace(10, log2(max_seq_len), 5)."""
    max_seq_len = (max_wsi_size // tile_size) ** 2
    seg = np.linspace(np.log2(1024), int(np.log2(max_seq_len)), 5)
    seg = np.power(2, seg).astype(int)
    return [int(v) for v in seg]


def padding_to_multiple_of(n: int, mult: int) -> int:
    """torchscale/component/utils.py:7-11."""
    rem = n % mult
    return 0 if rem == 0 else mult - rem


# ----------------------------------------------------------------------------------------------
# positional embedding (slide_encoder.py:104,121-125,166-179 ; pos_embed.py:30-77)
# ----------------------------------------------------------------------------------------------
def sincos_axis_table(embed_dim: int, grid: int) -> np.ndarray:
    """One axis of get_2d_sincos_pos_embed (pos_embed.py:59-77), fp64 math, fp32 result.

    Row v = [sin(v*w_k) | cos(v*w_k)], w_k = 10000**(-k/(E/4)), k < E/4.  The 2-D table row
    p>0 is [T[(p-1) % grid] | T[(p-1) // grid]] (pos_embed.py:36-56 with meshgrid(w, h)).
    """
    half = embed_dim // 2
    omega = np.arange(half // 2, dtype=float)
    omega /= half / 2.0
    omega = 1.0 / 10000 ** omega
    pos = np.arange(grid, dtype=np.float32).reshape(-1)
    out = np.einsum("m,d->md", pos, omega)
    return np.concatenate([np.sin(out), np.cos(out)], axis=1).astype(np.float32)


def coords_to_pos(coords, grid: int = 1000, tile_size: int = 256) -> np.ndarray:
    """slide_encoder.py:166-179: p = long(floor(x/t)*G + floor(y/t)) + 1, in fp32."""
    c = np.asarray(coords, dtype=np.float32)
    c_ = np.floor(c / np.float32(tile_size))
    pos = c_[..., 0] * np.float32(grid) + c_[..., 1]
    return pos.astype(np.int64) + 1


def pos_embed_rows(pos: np.ndarray, table: np.ndarray, grid: int) -> np.ndarray:
    """pos_embed[:, pos, :] (slide_encoder.py:200) from the factorised table; torch index rules."""
    n_rows = grid * grid + 1
    p = np.where(pos < 0, pos + n_rows, pos)
    if np.any((p < 0) | (p >= n_rows)):
        raise IndexError("pos index out of range for pos_embed of %d rows" % n_rows)
    q = np.maximum(p - 1, 0)
    rows = np.concatenate([table[q % grid], table[q // grid]], axis=-1)
    rows[p == 0] = 0.0
    return rows.astype(np.float32)


# ----------------------------------------------------------------------------------------------
# dilated bookkeeping (dilated_attention.py:16-53, 76-131)
# ----------------------------------------------------------------------------------------------
def branch_geometry(L: int, sl: int, r: int, H: int) -> dict:
    s = min(sl, L)                                   # :86
    nseg = -(-L // s)                                # :88-90
    m = -(-s // r)                                   # :18-22
    Hp = H + padding_to_multiple_of(H, r)            # :19-22 head padding
    return dict(s=s, r=r, nseg=nseg, m=m, g=m * r, hpg=Hp // r, L=L, H=H)


def gather_index(L: int, sl: int, r: int, H: int) -> np.ndarray:
    """Token feeding sparse row i of (segment n, head h); -1 where the reference reads a zero pad.

    dense_to_sparse (:16-31): row i of head h = r2*(Hp/r)+h' reads segment position i*r + r2.
    """
    g = branch_geometry(L, sl, r, H)
    s, nseg, m, hpg = g["s"], g["nseg"], g["m"], g["hpg"]
    n = np.arange(nseg)[:, None, None]
    h = np.arange(H)[None, :, None]
    i = np.arange(m)[None, None, :]
    t = i * r + h // hpg
    tok = n * s + t
    ok = (t < s) & (tok < L)
    return np.where(ok, tok, -1).astype(np.int64)


def scatter_index(L: int, sl: int, r: int, H: int) -> Tuple[np.ndarray, np.ndarray]:
    """For dense position p and head h: which sparse (segment, row) sparse_to_dense +
    scattering (:33-53, :100-131) put there, or -1 (uncovered: out 0, lse -1e8).

    The dense layout is (n, l*r + r1) with per-segment length g = m*r, cropped to [0, L);
    g != s when s % r != 0, and then segments n>0 land shifted (reference behaviour).
    """
    geo = branch_geometry(L, sl, r, H)
    gg, hpg = geo["g"], geo["hpg"]
    p = np.arange(L)[:, None]
    h = np.arange(H)[None, :]
    n = p // gg
    t = p % gg
    i = t // r
    jj = t % r
    cov = (h // hpg) == jj
    return np.where(cov, n, -1).astype(np.int64), np.where(cov, i, -1).astype(np.int64)


def dilated_gather(x: torch.Tensor, sl: int, r: int) -> torch.Tensor:
    """gathering (:76-98) for x [B, L, H, D] -> [B, nseg, H, m, D], zeros at pads."""
    B, L, H, D = x.shape
    tok = torch.from_numpy(gather_index(L, sl, r, H))
    xp = torch.cat([x, x.new_zeros(B, 1, H, D)], dim=1)
    tok = torch.where(tok < 0, torch.full_like(tok, L), tok)
    hidx = torch.arange(H).view(1, H, 1).expand_as(tok)
    return xp[:, tok, hidx]                       # [B, nseg, H, m, D]


def branch_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, sl: int, r: int,
                     scale: Optional[float] = None, chunk: int = 1024):
    """One (segment, dilation) branch: gather + flash_attn_func semantics (flash_attention.py:13-16)
    with literal zero pads.  Returns o [B, nseg, H, m, D], lse [B, nseg, H, m] (natural log)."""
    B, L, H, D = q.shape
    scale = D ** -0.5 if scale is None else scale
    qg, kg, vg = (dilated_gather(t.float(), sl, r) for t in (q, k, v))
    _, nseg, _, m, _ = qg.shape
    o = torch.empty_like(qg)
    lse = torch.empty(B, nseg, H, m, dtype=torch.float32)
    for b in range(B):
        for n in range(nseg):
            kk, vv = kg[b, n], vg[b, n]
            for i0 in range(0, m, chunk):
                s_ = torch.matmul(qg[b, n, :, i0:i0 + chunk], kk.transpose(1, 2)) * scale
                l_ = torch.logsumexp(s_, dim=-1)
                o[b, n, :, i0:i0 + chunk] = torch.matmul(torch.exp(s_ - l_[..., None]), vv)
                lse[b, n, :, i0:i0 + chunk] = l_
    return o, lse


def merge_branches(outs: Sequence[torch.Tensor], lses: Sequence[torch.Tensor], L: int,
                   segs: Sequence[int], ratios: Sequence[int]) -> torch.Tensor:
    """scattering (:100-131): densify every branch, lse==0 -> -1e8 (:46), softmax over branch
    LSEs in fp32, weighted sum in branch order.  Returns [B, L, H*D]."""
    B, _, H, _, D = outs[0].shape
    dense_o, dense_l = [], []
    hidx = torch.arange(H).view(1, H).expand(L, H)
    for o, l, sl, r in zip(outs, lses, segs, ratios):
        n_idx, i_idx = (torch.from_numpy(a) for a in scatter_index(L, sl, r, H))
        cov = n_idx >= 0
        nn_, ii = n_idx.clamp(min=0), i_idx.clamp(min=0)
        od = o[:, nn_, hidx, ii] * cov[None, :, :, None]           # [B, L, H, D]
        ld = torch.where(cov[None], l[:, nn_, hidx, ii], torch.full((), -1e8))
        ld = torch.where(ld == 0, torch.full((), -1e8), ld)
        dense_o.append(od)
        dense_l.append(ld)
    st = torch.stack(dense_l, 0)
    mx = st.max(0)[0]
    w = [torch.exp(l - mx) for l in dense_l]
    ws = torch.stack(w, 0).sum(0)
    w = [x / ws for x in w]
    out = 0
    for od, wi in zip(dense_o, w):
        out = out + od * wi[..., None]
    return out.reshape(B, L, H * D)


# ----------------------------------------------------------------------------------------------
# layers (dilated_attention.py:133-217 ; encoder.py:116-162 ; feedforward_network.py:131-142)
# ----------------------------------------------------------------------------------------------
def _lin(x, W, pre):
    return F.linear(x, W[pre + ".weight"], W[pre + ".bias"])


def _ln(x, W, pre, eps):
    return F.layer_norm(x, (x.shape[-1],), W[pre + ".weight"], W[pre + ".bias"], eps)


def dilated_attention(x: torch.Tensor, W: Dict[str, torch.Tensor], pre: str, segs, ratios,
                      H: int, eps: float = 1e-5, return_branches: bool = False):
    """DilatedAttention.forward (dilated_attention.py:133-217), eval mode, no incremental state."""
    B, L, E = x.shape
    D = E // H
    q = _lin(x, W, pre + ".q_proj").view(B, L, H, D)
    k = _lin(x, W, pre + ".k_proj").view(B, L, H, D)
    v = _lin(x, W, pre + ".v_proj").view(B, L, H, D)
    outs, lses = [], []
    for sl, r in zip(segs, ratios):
        o, l = branch_attention(q, k, v, sl, r)
        outs.append(o)
        lses.append(l)
    attn = merge_branches(outs, lses, L, segs, ratios)
    attn = _ln(attn, W, pre + ".inner_attn_ln", eps)
    out = _lin(attn, W, pre + ".out_proj")
    if return_branches:
        return out, dict(q=q, k=k, v=v, outs=outs, lses=lses)
    return out


def encoder_layer(x, W, pre, segs, ratios, H, eps=1e-5):
    """EncoderLayer.forward (encoder.py:116-162) with subln (pre-LN), alpha = 1, eval."""
    h = _ln(x, W, pre + ".self_attn_layer_norm", eps)
    x = x + dilated_attention(h, W, pre + ".self_attn", segs, ratios, H, eps)
    h = _ln(x, W, pre + ".final_layer_norm", eps)
    h = _lin(h, W, pre + ".ffn.fc1")
    h = F.gelu(h.float())
    h = _ln(h, W, pre + ".ffn.ffn_layernorm", eps)
    h = _lin(h, W, pre + ".ffn.fc2")
    return x + h


def slide_encoder_forward(W: Dict[str, torch.Tensor], x, coords, cfg: dict,
                          all_layer_embed: bool = False, global_pool: bool = False,
                          layers: Optional[int] = None) -> List[torch.Tensor]:
    """LongNetViT.forward (slide_encoder.py:181-223) + Encoder.forward (encoder.py:327-399)."""
    x = torch.as_tensor(np.asarray(x, dtype=np.float32))
    B, N, _ = x.shape
    E, H = cfg["embed_dim"], cfg["heads"]
    G = cfg["slide_ngrids"]
    h = _lin(x, W, "patch_embed.proj")
    pos = coords_to_pos(coords, G, cfg["tile_size"])
    table = sincos_axis_table(E, G)
    h = h + torch.from_numpy(pos_embed_rows(pos, table, G))
    cls = W["cls_token"].view(1, 1, E).expand(B, 1, E)   # + pos_embed[:, :1] == zeros
    h = torch.cat([cls, h], dim=1)
    states = [h]
    depth = cfg["depth"] if layers is None else layers
    for li in range(depth):
        h = encoder_layer(h, W, "encoder.layers.%d" % li, cfg["segment_length"],
                          cfg["dilated_ratio"], H, cfg["ln_eps"])
        states.append(h)
    if all_layer_embed:
        xs = states
    else:
        xs = [_ln(h, W, "encoder.layer_norm", cfg["ln_eps"])]
    outs = []
    for t in xs:
        if global_pool:
            outs.append(_ln(t[:, 1:, :].mean(dim=1), W, "norm", cfg["norm_eps"]))
        else:
            outs.append(_ln(t, W, "norm", cfg["norm_eps"])[:, 0])
    return outs


# ----------------------------------------------------------------------------------------------
# seeded weights / synthetic inputs — identical arrays in oracle, golden and tests
# ----------------------------------------------------------------------------------------------
def state_dict_keys(cfg: dict) -> List[Tuple[str, Tuple[int, ...]]]:
    """The 247-key state-dict layout of LongNetViT (for 12 layers), in module order."""
    E, F_, C = cfg["embed_dim"], cfg["ffn_dim"], cfg["in_chans"]
    keys = [("cls_token", (1, 1, E)), ("patch_embed.proj.weight", (E, C)),
            ("patch_embed.proj.bias", (E,))]
    for li in range(cfg["depth"]):
        p = "encoder.layers.%d." % li
        for nm in ("k_proj", "v_proj", "q_proj", "out_proj"):
            keys += [(p + "self_attn.%s.weight" % nm, (E, E)), (p + "self_attn.%s.bias" % nm, (E,))]
        keys += [(p + "self_attn.inner_attn_ln.weight", (E,)), (p + "self_attn.inner_attn_ln.bias", (E,)),
                 (p + "self_attn_layer_norm.weight", (E,)), (p + "self_attn_layer_norm.bias", (E,)),
                 (p + "ffn.fc1.weight", (F_, E)), (p + "ffn.fc1.bias", (F_,)),
                 (p + "ffn.fc2.weight", (E, F_)), (p + "ffn.fc2.bias", (E,)),
                 (p + "ffn.ffn_layernorm.weight", (F_,)), (p + "ffn.ffn_layernorm.bias", (F_,)),
                 (p + "final_layer_norm.weight", (E,)), (p + "final_layer_norm.bias", (E,))]
    keys += [("encoder.layer_norm.weight", (E,)), ("encoder.layer_norm.bias", (E,)),
             ("norm.weight", (E,)), ("norm.bias", (E,))]
    return keys


def make_weights(cfg: dict, seed: int = 0, perturb: bool = True) -> "OrderedDict[str, np.ndarray]":
    """numpy PCG64 weights in the reference's init distributions (slide_encoder.py:121-164):
    xavier-uniform Linear weights, normal(0, .02) cls.  ``perturb`` also randomises biases and
    LayerNorm affines (the reference inits them to 0/1) so parity tests exercise them."""
    rng = np.random.Generator(np.random.PCG64(seed))
    W = OrderedDict()
    for name, shape in state_dict_keys(cfg):
        if name == "cls_token":
            a = rng.normal(0.0, 0.02, size=shape)
        elif name.endswith(".weight") and len(shape) == 2:
            bound = math.sqrt(6.0 / (shape[0] + shape[1]))
            a = rng.uniform(-bound, bound, size=shape)
        elif name.endswith(".bias"):
            a = rng.normal(0.0, 0.05, size=shape) if perturb else np.zeros(shape)
        else:  # LayerNorm weight
            a = 1.0 + rng.normal(0.0, 0.1, size=shape) if perturb else np.ones(shape)
        W[name] = a.astype(np.float32)
    return W


def weights_sha256(W) -> str:
    import hashlib
    h = hashlib.sha256()
    for k, v in W.items():
        h.update(k.encode())
        h.update(np.ascontiguousarray(np.asarray(v, dtype=np.float32)).tobytes())
    return h.hexdigest()


def synthetic_slide(N: int, in_chans: int = 1536, seed_x: int = 1, seed_c: int = 2,
                    B: int = 1, tile: int = 256) -> Tuple[np.ndarray, np.ndarray]:
    """x ~ PCG64(1) N(0,1) [B,N,C]; N distinct cells of an S x S grid
    (S = ceil(sqrt(N/0.7)), PCG64(2)), raster-sorted, coords = 256*cell (fp32)."""
    rx = np.random.Generator(np.random.PCG64(seed_x))
    x = rx.standard_normal((B, N, in_chans), dtype=np.float32)
    rc = np.random.Generator(np.random.PCG64(seed_c))
    S = int(math.ceil(math.sqrt(N / 0.7)))
    S = max(S, int(math.ceil(math.sqrt(N))))
    coords = np.empty((B, N, 2), dtype=np.float32)
    for b in range(B):
        cells = np.sort(rc.choice(S * S, size=N, replace=False))
        cx, cy = cells // S, cells % S
        coords[b, :, 0] = cx * tile
        coords[b, :, 1] = cy * tile
    return x, coords
