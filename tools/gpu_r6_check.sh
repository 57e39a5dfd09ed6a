#!/bin/bash
# Round-6 quick check of a host-path change: selected GPU tests (-k expression), then a graph-replay bench A/B
# of an environment switch (unset vs =0, alternating processes).  bash tools/gpu_r6_check.sh <tag> "<-k expr>" <VAR> [rounds]
set -o pipefail
TAG=$1; K=$2; VAR=$3; N=${4:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null; [ $rc -eq 0 ] || exit $rc
[ -z "$VAR" ] && exit 0
bash tools/gpu_r5_benchab.sh $TAG/ab $VAR $N
