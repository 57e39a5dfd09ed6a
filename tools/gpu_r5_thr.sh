#!/bin/bash
# SP probe A/B: product vs a lab build (W = 8, ranks 0, 6, 7, two repeats).  Usage: bash tools/gpu_r5_thr.sh <tag> <lab.so>
set -o pipefail
TAG=$1; LAB=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in "" $LAB "" $LAB; do
  n=${L:+lab}; n=${n:-prod}
  timeout -k 10 600 python -u tools/sp_rank_probe.py --worlds 8 --ranks 0,6,7 --local-first 1 ${L:+--lib $L} > $OUT/probe_$n.log 2>&1
  rc=$?; echo "probe $n rc=$rc"; grep '"W"' $OUT/probe_$n.log; [ $rc -eq 0 ] || exit $rc
  tail -1 $OUT/probe_$n.log >> $OUT/probes.jsonl
done
