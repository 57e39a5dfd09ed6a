"""Host-side issue time of one forward vs its GPU time (is a small slide launch-bound?).

    python tools/host_overhead.py [--tiles 2000 8750 70000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prov-gigapath-replication_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from gigapath import slide_encoder  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--graphs", action="store_true")
ap.add_argument("--tiles", type=int, nargs="+", default=[2000, 8750, 70000])
args = ap.parse_args()
model = slide_encoder.create_model("", "gigapath_slide_enc12l768d", 1536).cuda().eval()
model.validate_positions = False
model.use_hip_graphs = "--graphs" in sys.argv
if "--graphs" in sys.argv:
    sys.argv.remove("--graphs")
with torch.no_grad():
    for n in args.tiles:
        x, c = bench.make_slide(n)
        xt, ct = torch.from_numpy(x).cuda(), torch.from_numpy(c).cuda()
        for _ in range(3):
            model(xt, ct, all_layer_embed=True)
        torch.cuda.synchronize()
        # host issue time with the GPU kept busy (a big sleep kernel is not available: queue
        # 3 forwards and time the Python side of the 2nd/3rd)
        t0 = time.perf_counter()
        for _ in range(5):
            model(xt, ct, all_layer_embed=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("tiles %6d: host issue %.2f ms/forward, wall %.2f ms/forward" % (n, (t1 - t0) / 5 * 1e3, (t2 - t0) / 5 * 1e3),
              flush=True)
