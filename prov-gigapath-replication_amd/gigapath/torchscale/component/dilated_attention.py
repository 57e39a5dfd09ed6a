"""DilatedAttention for the MI355X path (reference: torchscale/component/dilated_attention.py).

Same constructor, parameter names (k_proj, v_proj, q_proj, out_proj, inner_attn_ln) and
forward signature as the reference module.  The forward runs the fused HIP pipeline:
one fused QKV GEMM, ONE gp_dilated_attn_fwd launch for every (segment, dilation) branch
(gather folded into the kernel's addressing, zero-pad keys analytic), gp_branch_merge_ln
(LSE merge + inner_attn_ln), and the out_proj GEMM.  Inference only (eval mode).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import runtime


class DilatedAttention(nn.Module):
    def __init__(self, args, embed_dim, num_heads, dropout=0.0, self_attention=False,
                 encoder_decoder_attention=False, subln=False):
        super().__init__()
        if not self_attention or encoder_decoder_attention:
            raise NotImplementedError("the slide encoder uses self-attention only")
        if not subln:
            raise NotImplementedError("the slide encoder uses subln (inner_attn_ln)")
        self.args = args
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = embed_dim // num_heads
        self.scaling = self.head_dim ** -0.5
        self.dropout = dropout
        self.self_attention = True
        # registration order = reference state-dict order (multihead_attention.py:43-53)
        self.k_proj = nn.Linear(embed_dim, embed_dim, bias=True)
        self.v_proj = nn.Linear(embed_dim, embed_dim, bias=True)
        self.q_proj = nn.Linear(embed_dim, embed_dim, bias=True)
        self.out_proj = nn.Linear(embed_dim, embed_dim, bias=True)
        self.inner_attn_ln = nn.LayerNorm(embed_dim, eps=args.layernorm_eps)
        self._packed = None
        self._packed_sig = None
        self._scratch = None

    def packed(self, dev, act: torch.dtype = torch.bfloat16) -> runtime.PackedAttention:
        sig = (str(dev), runtime.param_signature(self), act)
        if sig != self._packed_sig:
            self._packed = runtime.PackedAttention.from_module(self, dev, act)
            self._packed_sig = sig
        return self._packed

    @runtime.compute_format
    def forward(self, query, key, value, incremental_state=None, key_padding_mask=None, attn_mask=None,
                rel_pos=None, is_first_step=False, is_causal=False):
        if incremental_state is not None or is_causal or rel_pos is not None or attn_mask is not None:
            raise NotImplementedError("incremental/causal/rel_pos/attn_mask are not on the slide-encoder path")
        if self.training and self.dropout > 0:
            raise RuntimeError("DilatedAttention (MI355X path) is inference-only: call .eval()")
        B, L, E = query.shape
        if E != self.embed_dim or key.shape != query.shape or value.shape != query.shape:
            raise ValueError("query/key/value must all be [B, L, %d]" % self.embed_dim)
        dev = query.device
        if dev.type != "cuda":
            raise RuntimeError("DilatedAttention (MI355X path) needs ROCm device tensors")
        act = runtime.act_dtype()
        pa = self.packed(dev, act)
        M = B * L
        qkv = torch.empty(M, 3 * E, dtype=act, device=dev)
        if key is query and value is query:
            torch.addmm(pa.b_qkv, query.reshape(M, E).to(act), pa.w_qkv.t(), out=qkv)
        else:
            for i, t in enumerate((query, key, value)):
                torch.addmm(pa.b_qkv[i * E:(i + 1) * E], t.reshape(M, E).to(act),
                            pa.w_qkv[i * E:(i + 1) * E].t(), out=qkv[:, i * E:(i + 1) * E])
        key_ = (B, L, pa.H, pa.D, tuple(pa.segs), tuple(pa.ratios), act)
        if self._scratch is None or self._scratch.key != key_:
            self._scratch = runtime.AttentionScratch(dev, B, L, pa.H, pa.D, pa.segs, pa.ratios, act)
        merged = torch.empty(M, E, dtype=act, device=dev)
        runtime.dilated_attention_core(pa, qkv, B, L, self._scratch, merged)
        out = torch.addmm(pa.b_o_act, merged, pa.w_o.t())
        return out.view(B, L, E).to(query.dtype), None
