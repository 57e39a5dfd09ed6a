"""Worst per-vector max-rel / min-cos of the product forward against the reference's own fp32 goldens
(tests/golden/e2e_N*_B1.npz) for the headline slides, without asserting -- the parity headroom a
design switch spends (e.g. GIGAPATH_RESID_FUSED=0).  One JSON line per slide.

    python tools/golden_rel.py [--N 70000,256000] [--tag label]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from conftest import load_golden  # noqa: E402


def worst(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    wr, wc = 0.0, 1.0
    for idx in np.ndindex(*got.shape[:-1]):
        g, r = got[idx], ref[idx]
        wr = max(wr, float(np.abs(g - r).max() / np.abs(r).max()))
        wc = min(wc, float((g * r).sum() / np.sqrt((g * g).sum() * (r * r).sum())))
    return wr, wc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", default="70000,256000")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from gigapath import runtime, slide_encoder
    for N in [int(v) for v in args.N.split(",")]:
        mw = 262144 if N > 100000 else None
        kw = {"max_wsi_size": mw} if mw else {}
        cfg = orc.arch_config("gigapath_slide_enc12l768d", **kw)
        m = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536, **kw)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in orc.make_weights(cfg, seed=0).items()}, strict=True)
        m = m.cuda().eval()
        g = load_golden("e2e_N%d_B1.npz" % N)
        x, coords = orc.synthetic_slide(N)
        with torch.no_grad():
            xt, ct = torch.from_numpy(x).cuda(), torch.from_numpy(coords).cuda()
            allv = torch.stack(m(xt, ct, all_layer_embed=True)).cpu().numpy()
            last = m(xt, ct)[0].cpu().numpy()
        ra, ca = worst(allv, g["all_layer"])
        rl, cl = worst(last, g["last"])
        print(json.dumps({"tag": args.tag, "N": N, "resid_fused": runtime.RESID_FUSED,
                          "all_layer_max_rel": ra, "all_layer_min_cos": ca, "last_max_rel": rl,
                          "last_min_cos": cl}), flush=True)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
