#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench.py run.
# Usage on the GPU box: bash tools/pmc_bench.sh <tag> [bench args...]
TAG=${1:-pmc}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python bench.py --no-cpu-baseline --steps 1 --warmup 1 $BENCH_ARGS > $OUT/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
BENCH_ARGS="$*"
pass fetch FETCH_SIZE && pass write WRITE_SIZE && pass mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
  && pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS
