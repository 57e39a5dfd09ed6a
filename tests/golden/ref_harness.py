"""Import the *reference* slide encoder in the build container (never on the GPU box).

Used only by ``make_golden.py`` to produce the committed golden vectors.  Nothing here is
copied from the reference: the stubs stand in for absent third-party packages (timm,
fairscale) and for the CUDA-only ``flash_attn_func`` seam, which is restated from its
published definition in fp32.  Recipe: SURVEY.md §8(c).
"""
import os
import sys
import types

import numpy as np
import torch

REF_ROOT = "/root/reference"


def _install_stubs():
    registry = {}

    timm = types.ModuleType("timm")
    timm_models = types.ModuleType("timm.models")
    timm_registry = types.ModuleType("timm.models.registry")
    timm_layers = types.ModuleType("timm.models.layers")

    def register_model(fn):
        registry[fn.__name__] = fn
        return fn

    def create_model(name, pretrained=False, **kw):
        return registry[name](**kw)

    def drop_path(x, drop_prob=0.0, training=False):
        assert not training, "oracle runs in eval mode"
        return x

    timm.create_model = create_model
    timm.models = timm_models
    timm_models.registry = timm_registry
    timm_models.layers = timm_layers
    timm_registry.register_model = register_model
    timm_layers.drop_path = drop_path
    sys.modules.update({"timm": timm, "timm.models": timm_models,
                        "timm.models.registry": timm_registry, "timm.models.layers": timm_layers})

    fs = types.ModuleType("fairscale")
    fs_nn = types.ModuleType("fairscale.nn")
    fs_nn.checkpoint_wrapper = lambda m, *a, **k: m
    fs_nn.wrap = lambda m, *a, **k: m
    fs.nn = fs_nn
    sys.modules.update({"fairscale": fs, "fairscale.nn": fs_nn})


def flash_attn_fp32(q, k, v, dropout=0.0, bias=None, softmax_scale=None, is_causal=False, chunk=1024):
    """Restatement of flash_attn_func (torchscale/component/flash_attention.py:13-16):
    q,k,v [B, L, H, D] -> (out [B, L, H, D] in q.dtype, lse [B, H, L] fp32, natural log)."""
    assert bias is None and not is_causal and dropout == 0.0
    B, L, H, D = q.shape
    scale = D ** -0.5 if softmax_scale is None else softmax_scale
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 3, 1)
    vf = v.float().permute(0, 2, 1, 3)
    out = torch.empty(B, H, L, D, dtype=torch.float32)
    lse = torch.empty(B, H, L, dtype=torch.float32)
    # chunked over query rows AND over the batch (segments) so one score block stays <= ~256 MB (the
    # 256k slide's 251 x 1,024-token segments would otherwise need 17 GB per block)
    bc = max(1, (64 << 20) // (H * min(chunk, L) * L))
    for b0 in range(0, B, bc):
        for i0 in range(0, L, chunk):
            s = torch.matmul(qf[b0:b0 + bc, :, i0:i0 + chunk], kf[b0:b0 + bc]) * scale
            l_ = torch.logsumexp(s, dim=-1)
            out[b0:b0 + bc, :, i0:i0 + chunk] = torch.matmul(torch.exp(s - l_[..., None]), vf[b0:b0 + bc])
            lse[b0:b0 + bc, :, i0:i0 + chunk] = l_
    return out.permute(0, 2, 1, 3).to(q.dtype).contiguous(), lse


_loaded = None


def load_reference():
    """Returns (slide_encoder module, dilated_attention module, config module)."""
    global _loaded
    if _loaded is not None:
        return _loaded
    sys.dont_write_bytecode = True
    _install_stubs()
    np.set_printoptions(legacy="1.25")   # config.py:71 eval()s str(list(np.int64...))
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import gigapath.slide_encoder as se                      # noqa: E402
    import torchscale.component.multihead_attention as mha   # noqa: E402
    import torchscale.component.dilated_attention as da      # noqa: E402
    import torchscale.architecture.config as cfgmod          # noqa: E402
    mha.flash_attn_func = flash_attn_fp32
    _loaded = (se, da, cfgmod)
    return _loaded
