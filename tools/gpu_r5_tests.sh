#!/bin/bash
# Round-5 targeted GPU tests: bash tools/gpu_r5_tests.sh <tag> "<pytest -k expression>" [test files...]
set -o pipefail
TAG=${1:-r05_t}; K=${2:-}
shift 2
FILES=${@:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
fi
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null; exit $rc
