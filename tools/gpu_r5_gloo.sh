#!/bin/bash
# bench.py's multi-rank path rehearsed on one GPU (gloo, host-staged exchange: the time means nothing) with
# the round-5 product (key parts at W = 8).  Usage: bash tools/gpu_r5_gloo.sh <tag>
set -o pipefail
TAG=${1:-r05_gloo}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GP_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 8 --steps 2 --warmup 1 > $OUT/bench_gpus8.json 2> $OUT/bench_gpus8.err
rc=$?; echo "gpus8 rc=$rc"; cut -c1-400 $OUT/bench_gpus8.json; [ $rc -eq 0 ] || exit $rc
GP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 4 --steps 2 --warmup 1 > $OUT/bench_gpus4.json 2> $OUT/bench_gpus4.err
rc=$?; echo "gpus4 rc=$rc"; cut -c1-400 $OUT/bench_gpus4.json; exit $rc
