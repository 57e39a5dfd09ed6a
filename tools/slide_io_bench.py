"""Read throughput of slide files (gigapath/slide_io.py) for a C3-sized slide: 70,000 tiles x 1536 fp32
features + int64 coords, written by the spec writer in tests/ as contiguous and as chunked+shuffle+deflate,
then read back with read_assets_from_h5 (file in the page cache: this times the parser and the copy, not
the disk).  With a GPU, also times the host->HBM copy that feeds the encoder.

    python tools/slide_io_bench.py [--tiles 70000] [--reps 3]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "prov-gigapath-replication_amd"), os.path.join(ROOT, "tests")]

from gigapath import slide_io          # noqa: E402
from h5_spec_writer import Writer      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=70000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    feats = rng.standard_normal((args.tiles, 1536), dtype=np.float32)
    coords = rng.integers(0, 1000, size=(args.tiles, 2)).astype(np.int64) * 256
    nbytes = feats.nbytes + coords.nbytes
    out = {"tiles": args.tiles, "bytes": nbytes}
    with tempfile.TemporaryDirectory() as d:
        for name, kw in (("contiguous", {}),
                         ("chunked_one_tile_per_chunk", {"layout": "chunked", "chunks": (1, 1536)}),
                         ("chunked_shuffle_deflate", {"layout": "chunked", "chunks": (1024, 1536),
                                                      "filters": ("shuffle", "deflate")})):
            w = Writer()
            w.dataset("features", feats, **kw)
            w.dataset("coords", coords)
            p = os.path.join(d, name + ".h5")
            w.save(p)
            del w
            best = 1e9
            for _ in range(args.reps):
                t0 = time.perf_counter()
                a, _ = slide_io.read_assets_from_h5(p)
                best = min(best, time.perf_counter() - t0)
            assert np.array_equal(a["features"], feats)
            out[name] = {"file_bytes": os.path.getsize(p), "seconds": round(best, 4),
                         "GB_per_s": round(nbytes / best / 1e9, 2)}
            del a
        try:
            import torch
            if torch.cuda.is_available():
                y = torch.empty(feats.shape, dtype=torch.float32, device="cuda")
                for name, x in (("h2d_pinned", torch.from_numpy(feats).pin_memory()),
                                ("h2d_pageable", torch.from_numpy(feats))):
                    y.copy_(x, non_blocking=True)          # warm: allocation, mappings
                    torch.cuda.synchronize()
                    best = 1e9
                    for _ in range(args.reps):
                        t0 = time.perf_counter()
                        y.copy_(x, non_blocking=True)
                        torch.cuda.synchronize()
                        best = min(best, time.perf_counter() - t0)
                    out[name] = {"seconds": round(best, 4), "GB_per_s": round(feats.nbytes / best / 1e9, 2)}
                del y
        except ImportError:
            pass
    print(json.dumps(out))


if __name__ == "__main__":
    main()
