#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) over tools/merge_ab.py: L1 -> L2 request counts and
# latencies, L1 stalls, wave states of the merge kernels of the given builds.  bash tools/pmc_merge.sh <tag> [libs]
TAG=${1:-pmc_merge}; LIBS=${2:-prod,tools/attn_lab/liblab_mold.so}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
pass() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python tools/merge_ab.py --libs $LIBS --rounds 1 --iters 3 > $OUT/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum \
 && pass stall TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE \
 && pass ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_avr GRBM_GUI_ACTIVE \
 && pass fetch FETCH_SIZE \
 && pass write WRITE_SIZE \
 && pass wave SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU \
 && pass valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES
rc=$?
python - "$OUT" <<'PY'
import csv, glob, os, sys, collections, json
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "merge" not in k:
            continue
        k = k[k.find("branch_merge"):][:48]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
for k, cs in sorted(res.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-36s %.4g" % (c, v))
json.dump(res, open(os.path.join(root, "pmc_merge.json"), "w"), indent=1, sort_keys=True)
PY
exit $rc
