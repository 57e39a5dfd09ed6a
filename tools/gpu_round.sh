#!/bin/bash
# Round-end style GPU pass: GPU tests, smoke, the 70k bench (C3) + rocprof, the 256k single-GPU
# slide and the C5 packed mixed batch.  Usage: bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cat $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --tiles 256000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_256k.json 2> $OUT/bench_256k.err
rc=$?; echo "bench256k rc=$rc"; cat $OUT/bench_256k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode mixed --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?; echo "benchC5 rc=$rc"; cat $OUT/bench_c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
