"""Tune the slide encoder's hipBLASLt GEMMs with PyTorch TunableOp on the GPU box and write the
winning solutions to prov-gigapath-replication_amd/gigapath/tuned/tunableop_results.csv, which
runtime.py loads (tuning disabled) on every later run.

    python tools/tune_gemms.py [--tiles 70000 16384 ...]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "prov-gigapath-replication_amd", "gigapath", "tuned", "tunableop_results.csv")

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tiles", type=int, nargs="+", default=[70000])
ap.add_argument("--out", default=OUT)
args = ap.parse_args()

os.environ["GIGAPATH_NO_TUNED_GEMMS"] = "1"       # do not load an old file while tuning
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_max_tuning_duration(60)
torch.cuda.tunable.set_max_tuning_iterations(30)
torch.cuda.tunable.set_filename(args.out)

import bench  # noqa: E402
from gigapath import slide_encoder  # noqa: E402

model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).cuda().eval()
with torch.no_grad():
    for n in args.tiles:
        x, c = bench.make_slide(n)
        model(torch.from_numpy(x).cuda(), torch.from_numpy(c).cuda(), all_layer_embed=True)
        torch.cuda.synchronize()
        print("tuned shapes for", n, "tiles", flush=True)
# TunableOp writes the file at interpreter exit (set_filename above)
print("tuned", len(torch.cuda.tunable.get_results()), "GEMM shapes ->", args.out)
