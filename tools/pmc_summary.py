"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch, per kernel (short names).

    python tools/pmc_summary.py gpurun_out/<tag>        # every */run_counter_collection.csv below it
FETCH_SIZE / WRITE_SIZE are in KiB; HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
(gfx950: FETCH_SIZE reports half the bytes of wide coalesced reads, MI355X_MICROARCH.md §HBM).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel)(<[^>(]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:60]


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in sorted(acc.items()):
        items = ["%s=%.4g(n=%d)" % (c, sum(v) / len(v), len(v)) for c, v in sorted(cs.items())]
        print(k, " ".join(items))


if __name__ == "__main__":
    main(sys.argv[1])


def traffic_json(root, out, tiles, tag):
    """Write per-kernel HBM bytes per launch ((2*FETCH_SIZE + WRITE_SIZE) KiB -> bytes) for bench.py."""
    import json
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            res[k] = {"hbm_bytes_per_launch": (2 * fetch + write) * 1024, "fetch_kib_raw": fetch, "write_kib": write}
    with open(out, "w") as fh:
        json.dump({"tiles": tiles, "source": tag, "kernels": res}, fh, indent=1, sort_keys=True)
