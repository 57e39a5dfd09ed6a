#!/bin/bash
# Round 4: rocprofv3 kernel stats of the 70k bench with and without the residual epilogues, same box
set -o pipefail
TAG=${1:-r04_o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fused -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/fused.log 2>&1
rc=$?; echo "fused rc=$rc"; [ $rc -eq 0 ] || exit $rc
GIGAPATH_RESID_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/unfused -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/unfused.log 2>&1
rc=$?; echo "unfused rc=$rc"; exit $rc
