#!/bin/bash
# One GPU-box pass: parity tests, bench (70k, C3), rocprofv3 kernel-trace summary of the bench.
# Usage (from the repo root on the box): bash tools/gpu_check.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/lab_check.py --out $OUT/lab_check.json > $OUT/lab_check.log 2>&1; echo "lab_check rc=$?"; tail -2 $OUT/lab_check.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline "$@" > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*stats*"
exit $rc
