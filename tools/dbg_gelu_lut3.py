"""Debug: bf16 h of gp_ffn_fc1_gelu vs torch's CPU GELU of gp_linear's pre-activation, for the product
library and the lab variants named on the command line."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
import torch  # noqa: E402

from gigapath import _hip  # noqa: E402

prod = _hip.load_library()
libs = [("product", prod)] + [(p, _hip.load_library(os.path.join(ROOT, p))) for p in sys.argv[1:]]
_hip._lib = prod
DEV = "cuda"
E, F = 768, 3072
for M in (255, 1000):
    g = torch.Generator(device=DEV).manual_seed(M)
    a = (torch.randn(M, E, device=DEV, generator=g)).bfloat16()
    w1 = (torch.randn(F, E, device=DEV, generator=g) * E ** -0.5 * 1.5).bfloat16()
    b1 = torch.randn(F, device=DEV, generator=g) * 0.2
    stats = torch.empty((F // 256 + 1) * M * 2, device=DEV)
    pre = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
    _hip.linear(a, w1, b1, pre, None)
    torch.cuda.synchronize()
    ex = torch.nn.functional.gelu(pre.float().cpu()).bfloat16()
    for name, lib in libs:
        _hip._lib = lib
        hh = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
        _hip.ffn_fc1_gelu(a, w1, b1, hh, stats)
        _hip._lib = prod
        torch.cuda.synchronize()
        bad = hh.cpu() != ex
        idx = bad.nonzero()
        rows = idx[:, 0].unique()[:12].tolist() if bad.any() else []
        print(M, name, "mismatch", int(bad.sum()), "rows", rows, flush=True)
