"""LongNet encoder assembly (reference: torchscale/model/LongNet.py:47-128)."""
from __future__ import annotations

import copy

from ..architecture.config import EncoderConfig
from ..architecture.encoder import Encoder, EncoderLayer
from ..component.dilated_attention import DilatedAttention
from . import LongNetConfig


class LongNetEncoderLayer(EncoderLayer):
    def build_self_attention(self, embed_dim, args):
        return DilatedAttention(args, embed_dim, args.encoder_attention_heads, dropout=args.attention_dropout,
                                self_attention=True, encoder_decoder_attention=False, subln=args.subln)


class LongNetEncoder(Encoder):
    def build_encoder_layer(self, args, depth, is_moe_layer=False, is_encoder_decoder=False):
        return LongNetEncoderLayer(args, depth, is_moe_layer=is_moe_layer, is_encoder_decoder=is_encoder_decoder)


def make_longnet_from_name(config_name: str, dilated_ratio: str = "[1, 2, 4, 8, 16]",
                           segment_length: str = "[1024, 2048, 4096, 8192, 16384]",
                           drop_path_rate: float = 0.1, dropout: float = 0.1):
    """Build a LongNetEncoder from a named config with the given dilation schedule."""
    if config_name not in LongNetConfig.CONFIGS:
        raise KeyError("unknown LongNet config %r" % config_name)
    kw = copy.deepcopy(LongNetConfig.CONFIGS[config_name])
    kw.update(dropout=dropout, drop_path_rate=drop_path_rate, dilated_ratio=dilated_ratio,
              segment_length=segment_length)
    print("dilated_ratio: ", dilated_ratio)
    print("segment_length: ", segment_length)
    model = LongNetEncoder(EncoderConfig(**kw))
    print("Number of trainable LongNet parameters: ", sum(p.numel() for p in model.parameters() if p.requires_grad))
    return model
