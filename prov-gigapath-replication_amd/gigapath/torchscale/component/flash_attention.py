"""Operator seam of the reference: ``flash_attn_func`` (torchscale/component/flash_attention.py:13-16).

On the reference this binds flash-attn 2.5.8 (CUDA) or xformers; here it binds the gfx950
MFMA kernel behind ``gp_seg_attn_fwd`` (bf16) / ``gp_seg_attn_fwd_f16`` (fp16).  Same contract:
q, k, v [B, L, H, D], non-causal, no mask, dropout 0; returns (out [B, L, H, D] in q's dtype,
softmax_lse [B, H, L] fp32, natural log).  fp16 inputs (the reference pipeline's autocast,
pipeline.py:186-187) compute in fp16 as flash-attn does; bf16 in bf16; fp32 inputs (which flash-attn
rejects) are computed in bf16.
"""
from __future__ import annotations

import torch

from ... import _hip


def flash_attn_func(q, k, v, dropout=0.0, bias=None, softmax_scale=None, is_causal=False):
    if bias is not None or is_causal or dropout != 0.0:
        raise NotImplementedError("gp_seg_attn_fwd: bias / causal / dropout are not on the slide-encoder path")
    if q.device.type != "cuda":
        raise RuntimeError("flash_attn_func (MI355X path) needs ROCm device tensors")
    B, L, H, D = q.shape
    dt = torch.float16 if q.dtype == torch.float16 else torch.bfloat16
    qb, kb, vb = (t.to(dt).contiguous() for t in (q, k, v))
    out = torch.empty_like(qb)
    lse = torch.empty(B, H, L, dtype=torch.float32, device=q.device)
    _hip.seg_attn_fwd(qb, kb, vb, out, lse, softmax_scale or 0.0)
    return out.to(q.dtype), lse
