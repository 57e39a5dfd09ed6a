#!/bin/bash
# Round-5 pass: all GPU tests, smoke, default bench, rocprof stats, fp16 caller.  bash tools/gpu_r5_full.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r05_full}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cut -c1-300 $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c4-ref > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fp16_caller_bench.py > $OUT/fp16_caller.log 2>&1
rc=$?; echo "fp16 caller rc=$rc"; tail -4 $OUT/fp16_caller.log; exit $rc
