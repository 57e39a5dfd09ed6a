#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) over tools/gemm_ab.py on selected GEMM entry points:
# memory-pipeline latency / stall / TLB counters per kernel.  bash tools/pmc_gemm.sh <tag> <gemm_ab --only list>
TAG=${1:-pmc_gemm}; ONLY=${2:-out_bias,out_resid}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
pass() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python tools/gemm_ab.py --libs prod --rounds 1 --iters 3 --only $ONLY > $OUT/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
pass tlb TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum GRBM_GUI_ACTIVE \
 && pass lat TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum \
 && pass stall TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum \
 && pass ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE \
 && pass tcc TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_sum \
 && pass wave SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES
rc=$?
python - "$OUT" <<'PY'
import csv, glob, os, sys, collections
root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = k[k.find("gemm_kernel"):][:40] if "gemm_kernel" in k else k[:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print("   %-45s %.4g" % (c, sum(v) / len(v)))
PY
exit $rc
