"""FFN of the LongNet encoder layer (reference: torchscale/component/feedforward_network.py:105-142).

fc1 -> exact-erf GELU in fp32 -> ffn_layernorm -> fc2.  fc1/fc2 run on hipBLASLt in bf16 (fp16 under
the caller's fp16 autocast);
GELU and the 3072-wide LayerNorm are one HIP kernel (gp_gelu_layernorm).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import _hip, runtime


class FeedForwardNetwork(nn.Module):
    def __init__(self, embed_dim, ffn_dim, activation_fn="gelu", dropout=0.0, activation_dropout=0.0,
                 layernorm_eps=1e-5, subln=True):
        super().__init__()
        if str(activation_fn) != "gelu" or not subln:
            raise NotImplementedError("the slide encoder FFN is gelu + subln")
        self.embed_dim = embed_dim
        self.dropout = dropout
        self.activation_dropout = activation_dropout
        self.fc1 = nn.Linear(embed_dim, ffn_dim)
        self.fc2 = nn.Linear(ffn_dim, embed_dim)
        self.ffn_layernorm = nn.LayerNorm(ffn_dim, eps=layernorm_eps)

    @runtime.compute_format
    def forward(self, x):
        if x.device.type != "cuda":
            raise RuntimeError("FeedForwardNetwork (MI355X path) needs ROCm device tensors")
        shape = x.shape
        dev = x.device
        act = runtime.act_dtype()
        h = torch.addmm(self.fc1.bias.to(dev, act), x.reshape(-1, shape[-1]).to(act), self.fc1.weight.to(dev, act).t())
        _hip.gelu_layernorm(h, runtime._f32(self.ffn_layernorm.weight, dev), runtime._f32(self.ffn_layernorm.bias, dev),
                            float(self.ffn_layernorm.eps), h, h.shape[0], h.shape[1])
        y = torch.addmm(self.fc2.bias.to(dev, act), h, self.fc2.weight.to(dev, act).t())
        return y.view(shape).to(x.dtype)
