#!/bin/bash
# Round-3 first pass: GPU tests (minus the 8-rank 256k golden test, golden pending, and the 4-stream
# concurrency test, run on its own), then the 8-rank gloo bench rehearsal of the driver's N = 8 run.
set -o pipefail
OUT=gpurun_out/r03_a
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
    -k "not eight_ranks and not four_stream" > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
GP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 > $OUT/bench_sp8_gloo.json 2> $OUT/bench_sp8_gloo.err
rc=$?; echo "sp8 gloo rc=$rc"; cat $OUT/bench_sp8_gloo.json; tail -5 $OUT/bench_sp8_gloo.err; exit $rc
