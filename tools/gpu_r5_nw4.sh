#!/bin/bash
# Round-5 under-filled-launch check: attention kernel tests, then the SP rank probe (W = 8, ranks 0, 6, 7)
# with the product and with the lab build without the 4-wave switch.  Usage: bash tools/gpu_r5_nw4.sh <tag>
set -o pipefail
TAG=${1:-r05_nw4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
for L in "" tools/attn_lab/liblab_nonw4.so "" tools/attn_lab/liblab_nonw4.so; do
  n=${L:+lab}; n=${n:-prod}
  timeout -k 10 600 python -u tools/sp_rank_probe.py --worlds 8 --ranks 0,6,7 --local-first 1 ${L:+--lib $L} > $OUT/probe_$n.log 2>&1
  rc=$?; echo "probe $n rc=$rc"; grep '"W"' $OUT/probe_$n.log; [ $rc -eq 0 ] || exit $rc
  tail -1 $OUT/probe_$n.log >> $OUT/probes.jsonl
done
