#!/bin/bash
# PMC passes over the attention kernel (tools/attn_bench.py, impl 2 only). One pass per counter group.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_attn_${IMPL:-2p}
mkdir -p $OUT
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pass() {
  name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python tools/attn_bench.py --impls ${IMPL:-2p} --iters 3 > $OUT/$name.log 2>&1
  echo "pass $name rc=$?"
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA
pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM
pass c GRBM_GUI_ACTIVE GRBM_COUNT FETCH_SIZE
pass d SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_LDS_UNALIGNED_STALL SQ_INSTS_BRANCH
