"""Named LongNet encoder configurations used by the registered slide encoders
(reference: torchscale/model/LongNetConfig.py:166-275).  All use 16 heads and FFN = 4E;
segment lengths / dilation ratios are overridden by make_longnet_from_name."""


def _cfg(layers, dim):
    return {
        "encoder_layers": layers,
        "encoder_embed_dim": dim,
        "encoder_ffn_embed_dim": 4 * dim,
        "encoder_attention_heads": 16,
        "dilated_ratio": "[1, 2, 4, 8, 16]",
        "segment_length": "[1024, 2048, 4096, 8192, 16384]",
        "flash_attention": True,
        "block_shift": True,
        "use_xmoe": False,
        "moe_top1_expert": False,
        "moe_freq": 0,
        "moe_expert_count": 0,
    }


LongNet_8_layers_768_dim = _cfg(8, 768)
LongNet_12_layers_768_dim = _cfg(12, 768)
LongNet_8_layers_1024_dim = _cfg(8, 1024)
LongNet_24_layers_1024_dim = _cfg(24, 1024)
LongNet_3_layers_1536_dim = _cfg(3, 1536)
LongNet_6_layers_1536_dim = _cfg(6, 1536)
LongNet_8_layers_1536_dim = _cfg(8, 1536)
LongNet_12_layers_1536_dim = _cfg(12, 1536)

CONFIGS = {k: v for k, v in dict(globals()).items() if k.startswith("LongNet_")}
