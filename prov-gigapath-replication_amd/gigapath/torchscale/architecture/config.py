"""Encoder hyper-parameters for the LongNet slide encoder.

Mirrors the fields of the reference ``EncoderConfig`` (torchscale/architecture/config.py:5-84)
that the slide-encoder path reads.  Segment lengths and dilation ratios may be given as
lists or as the reference's string form ("[1024, 5792, ...]"), parsed with ast.literal_eval
instead of eval.  Options the reference supports but the slide encoder never enables (MoE,
xPos, relative position buckets, deepnorm, multiway, sequence-parallel K/V gather) are
accepted and must stay at their defaults; anything else raises.
"""
from __future__ import annotations

import ast
from typing import List, Sequence, Union

_UNSUPPORTED_IF_SET = {
    "moe_freq": 0, "moe_expert_count": 0, "use_xmoe": False, "xpos_rel_pos": False,
    "rel_pos_buckets": 0, "max_rel_pos": 0, "deepnorm": False, "multiway": False,
    "layernorm_embedding": False, "bert_init": False,
}


def _as_int_list(v: Union[str, Sequence[int], None]) -> List[int]:
    if v is None or v == "":
        return []
    if isinstance(v, str):
        v = ast.literal_eval(v)
    return [int(x) for x in v]


class EncoderConfig:
    def __init__(self, **kw):
        self.encoder_embed_dim = kw.pop("encoder_embed_dim", 768)
        self.encoder_attention_heads = kw.pop("encoder_attention_heads", 12)
        self.encoder_ffn_embed_dim = kw.pop("encoder_ffn_embed_dim", 3072)
        self.encoder_layers = kw.pop("encoder_layers", 12)
        self.activation_fn = kw.pop("activation_fn", "gelu")
        self.dropout = kw.pop("dropout", 0.0)
        self.drop_path_rate = kw.pop("drop_path_rate", 0.0)
        self.attention_dropout = kw.pop("attention_dropout", 0.0)
        self.activation_dropout = kw.pop("activation_dropout", 0.0)
        self.layernorm_eps = kw.pop("layernorm_eps", 1e-5)
        self.subln = kw.pop("subln", True)
        self.normalize_output = kw.pop("normalize_output", True)
        self.no_scale_embedding = kw.pop("no_scale_embedding", True)
        self.flash_attention = kw.pop("flash_attention", False)
        self.seq_parallel = kw.pop("seq_parallel", False)
        self.segment_length = _as_int_list(kw.pop("segment_length", None))
        self.dilated_ratio = _as_int_list(kw.pop("dilated_ratio", None))
        for k, default in _UNSUPPORTED_IF_SET.items():
            v = kw.pop(k, default)
            if v != default:
                raise NotImplementedError("EncoderConfig.%s=%r is outside the slide-encoder path" % (k, v))
        # remaining reference keys (vocab/img sizes, fsdp, checkpointing, block_shift, ...) are inert here
        self.extra = dict(kw)
        if self.activation_fn != "gelu":
            raise NotImplementedError("only gelu FFN is on the slide-encoder path")
        if len(self.segment_length) != len(self.dilated_ratio):
            raise ValueError("segment_length and dilated_ratio must have the same length")
        if not self.no_scale_embedding:
            raise NotImplementedError("embed scaling is not used by LongNetViT")
        if not self.subln:
            raise NotImplementedError("LongNet slide encoders use subln (pre-LN + inner LNs)")
        self.encoder_normalize_before = True   # subln forces pre-LN (reference config.py:78-80)
