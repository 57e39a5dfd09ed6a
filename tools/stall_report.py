"""Stall attribution from the rocprofv3 --pmc passes of tools/pmc_stall.sh (verdict r03 item 1).

    python tools/stall_report.py gpurun_out/<tag>_pmc [kernel-prefix ...]

Per kernel (mean per dispatch): the wave-cycle split SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on
s_waitcnt / s_barrier) + SQ_WAIT_INST_ANY (ready but not issued: dependency / pipe busy) +
SQ_ACTIVE_INST_ANY (issuing), as fractions; the MFMA pipe's busy share of SIMD-cycles
(SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE/XCDs)); the effective clock is not derivable
without the wall time, so it is left to the caller; VALU and LDS instructions per MFMA.
SQ_* wave / wait / active counters count quad-cycles (MI355X_MICROARCH.md, cycle-constants table).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402

import csv  # noqa: E402
import glob  # noqa: E402
from collections import defaultdict  # noqa: E402

SIMDS = 1024
XCDS = 8


def load(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                acc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def report(k, c):
    out = {"kernel": k}
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_SCA",
                     "SQ_ACTIVE_INST_VMEM"):
            if name in c:
                out[name.replace("SQ_", "").lower() + "_frac"] = round(c[name] / wc, 4)
    g = c.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        out["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / (g / XCDS), 4)
        out["kernel_cycles"] = round(g / XCDS)
    mf = c.get("SQ_INSTS_MFMA")
    if mf:
        for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
            if name in c:
                out[name.replace("SQ_INSTS_", "").lower() + "_per_mfma"] = round(c[name] / mf, 3)
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_conflict_frac"] = round(c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"], 4)
    out["raw"] = {n: float("%.4g" % v) for n, v in sorted(c.items())}
    return out


def main():
    root = sys.argv[1]
    prefixes = sys.argv[2:] or ["dilated_attn32_kernel<48, true, 0", "gemm_kernel", "branch_merge_kernel"]
    data = load(root)
    res = [report(k, c) for k, c in sorted(data.items()) if any(k.startswith(p) for p in prefixes)]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
