#!/bin/bash
# Stall attribution (verdict r03 item 1): the counter list, then one rocprofv3 --pmc pass per counter
# group over a short 70k bench.py run (every kernel of the forward is profiled; tools/pmc_summary.py
# averages per kernel).  SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES (quad-cycles).
# Usage on the GPU box: bash tools/pmc_stall.sh <tag> [bench args...]
TAG=${1:-pmc_stall}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
echo "list rc=$?"
pass() {
  name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python bench.py --no-cpu-baseline --steps 1 --warmup 1 --timing-steps 1 $BENCH_ARGS > $OUT/$name.log 2>&1
  rc=$?; echo "pass $name rc=$rc"; return $rc
}
BENCH_ARGS="$*"
pass wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  && pass inst SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE \
  && pass lds SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH
rc=$?
python tools/pmc_summary.py $OUT > $OUT/summary.txt
exit $rc
