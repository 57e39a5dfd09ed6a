"""LongNet encoder stack (reference: torchscale/architecture/encoder.py:25-399), eval-mode, subln.

Module tree and parameter names match the reference (layers.{i}.self_attn.*,
self_attn_layer_norm, ffn.{fc1,fc2,ffn_layernorm}, final_layer_norm, layer_norm) so
reference state dicts load unchanged.  ``Encoder.forward`` keeps the reference's signature
and return dict; the arithmetic runs through runtime.EncoderEngine (HIP kernels + hipBLASLt).
LongNetViT bypasses it to fuse the embedding with the first LayerNorm.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ... import _hip, runtime
from ..component.dilated_attention import DilatedAttention
from ..component.feedforward_network import FeedForwardNetwork


def _ln_to_act(x32: torch.Tensor, ln: nn.LayerNorm, out_act: torch.Tensor):
    """out = LayerNorm(x) for an fp32 [M, E] residual stream, rounded to the 16-bit activation format
    (standalone-module entry only)."""
    dev = x32.device
    tmp = torch.empty_like(x32)
    _hip.layernorm_f32(x32, x32.shape[1], runtime._f32(ln.weight, dev), runtime._f32(ln.bias, dev), float(ln.eps),
                       tmp, x32.shape[0], x32.shape[1])
    out_act.copy_(tmp)


class EncoderLayer(nn.Module):
    def __init__(self, args, depth, is_moe_layer=False, is_encoder_decoder=False):
        super().__init__()
        if is_moe_layer or is_encoder_decoder:
            raise NotImplementedError("MoE / encoder-decoder layers are outside the slide-encoder path")
        self.args = args
        self.embed_dim = args.encoder_embed_dim
        self.self_attn = self.build_self_attention(self.embed_dim, args)
        self.self_attn_layer_norm = nn.LayerNorm(self.embed_dim, eps=args.layernorm_eps)
        self.dropout = args.dropout
        self.drop_path_prob = (float(np.linspace(0, args.drop_path_rate, args.encoder_layers)[depth])
                               if args.drop_path_rate > 0 else 0.0)
        self.ffn_dim = args.encoder_ffn_embed_dim
        self.ffn = FeedForwardNetwork(self.embed_dim, self.ffn_dim, args.activation_fn, args.dropout,
                                      args.activation_dropout, args.layernorm_eps, args.subln)
        self.final_layer_norm = nn.LayerNorm(self.embed_dim, eps=args.layernorm_eps)

    def build_self_attention(self, embed_dim, args):
        return DilatedAttention(args, embed_dim, args.encoder_attention_heads, dropout=args.attention_dropout,
                                self_attention=True, subln=args.subln)

    @runtime.compute_format
    def forward(self, x, encoder_padding_mask=None, attn_mask=None, rel_pos=None, multiway_split_position=None,
                incremental_state=None):
        if self.training and (self.dropout > 0 or self.drop_path_prob > 0):
            raise RuntimeError("EncoderLayer (MI355X path) is inference-only: call .eval()")
        B, L, E = x.shape
        dev = x.device
        if dev.type != "cuda":
            raise RuntimeError("EncoderLayer (MI355X path) needs ROCm device tensors")
        eng = runtime.EncoderEngine()
        act = runtime.act_dtype()
        pl = runtime.PackedLayer.from_module(self, dev, act)
        eng.layers = [pl]
        ws = runtime.Workspace(dev, B, L, E, self.ffn_dim, pl.attn.H, pl.attn.segs, pl.attn.ratios, act)
        ws.x.copy_(x.reshape(B * L, E))
        _ln_to_act(ws.x, self.self_attn_layer_norm, ws.a)
        eng.run_layers(ws, B, L)
        return ws.x.view(B, L, E).to(x.dtype), None


class Encoder(nn.Module):
    def __init__(self, args, embed_tokens=None, embed_positions=None, output_projection=None,
                 is_encoder_decoder=False, **kwargs):
        super().__init__(**kwargs)
        if embed_tokens is not None or embed_positions is not None or output_projection is not None:
            raise NotImplementedError("token/position embeddings and output projections are not used by LongNetViT")
        self.args = args
        self.layers = nn.ModuleList([self.build_encoder_layer(args, depth=i) for i in range(args.encoder_layers)])
        self.num_layers = len(self.layers)
        self.layer_norm = (nn.LayerNorm(args.encoder_embed_dim, eps=args.layernorm_eps)
                           if args.encoder_normalize_before and args.normalize_output else None)
        self.engine = runtime.EncoderEngine()

    def build_encoder_layer(self, args, depth, is_moe_layer=False, is_encoder_decoder=False):
        return EncoderLayer(args, depth, is_moe_layer=is_moe_layer, is_encoder_decoder=is_encoder_decoder)

    def check_eval(self):
        if self.training and (self.args.dropout > 0 or self.args.drop_path_rate > 0):
            raise RuntimeError("the MI355X slide encoder is inference-only: call model.eval()")

    @runtime.compute_format
    def forward(self, src_tokens, encoder_padding_mask=None, attn_mask=None, return_all_hiddens=False,
                token_embeddings=None, multiway_split_position=None, features_only=False,
                incremental_state=None, positions=None, **kwargs):
        if token_embeddings is None:
            raise NotImplementedError("LongNetViT feeds token_embeddings; src_tokens lookup is not on the path")
        if attn_mask is not None or incremental_state is not None:
            raise NotImplementedError("attn_mask / incremental_state are not on the slide-encoder path")
        self.check_eval()
        x_in = token_embeddings
        B, L, E = x_in.shape
        dev = x_in.device
        if dev.type != "cuda":
            raise RuntimeError("Encoder (MI355X path) needs ROCm device tensors")
        if encoder_padding_mask is None:
            encoder_padding_mask = torch.zeros(B, L, dtype=torch.bool, device=dev)
        else:
            # encoder.py:358: masked embeddings are zeroed before the first layer (and in
            # encoder_states[0]); the flash attention path does not see the mask
            # (multihead_attention.py:103), so padded tokens stay keys of every branch
            if encoder_padding_mask.shape != (B, L):
                raise ValueError("encoder_padding_mask must be [B, L] = [%d, %d], got %s"
                                 % (B, L, tuple(encoder_padding_mask.shape)))
            x_in = x_in * (1 - encoder_padding_mask.to(dev).unsqueeze(-1).type_as(x_in))
        layers = self.engine.pack(self, dev)
        pa = layers[0].attn
        ws = self.engine.workspace(dev, B, L, E, self.args.encoder_ffn_embed_dim, pa.H, pa.segs, pa.ratios)
        ws.x.copy_(x_in.reshape(B * L, E))
        _ln_to_act(ws.x, self.layers[0].self_attn_layer_norm, ws.a)
        states = [x_in] if return_all_hiddens else []

        def hook(i):
            if return_all_hiddens:
                states.append(ws.x.view(B, L, E).to(x_in.dtype, copy=True))

        self.engine.run_layers(ws, B, L, hook)
        x = ws.x
        if self.layer_norm is not None:
            out = torch.empty_like(x)
            _hip.layernorm_f32(x, E, runtime._f32(self.layer_norm.weight, dev), runtime._f32(self.layer_norm.bias, dev),
                               float(self.layer_norm.eps), out, B * L, E)
            x = out
        return {"encoder_out": x.view(B, L, E).to(x_in.dtype), "encoder_embedding": token_embeddings,
                "encoder_padding_mask": encoder_padding_mask, "encoder_states": states, "l_aux": [None] * self.num_layers}
