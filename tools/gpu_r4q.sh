#!/bin/bash
# Round 4: the driver's N = 2 and N = 4 scaling commands rehearsed with gloo ranks on the one GPU (host-staged
# transport: times mean nothing; the point is that every rank runs the round-4 product to the JSON line)
set -o pipefail
TAG=${1:-r04_q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 2 4; do
  GP_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus $n --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_sp${n}_gloo.json 2> $OUT/bench_sp${n}_gloo.err
  rc=$?; echo "sp$n gloo rc=$rc"; tail -c 300 $OUT/bench_sp${n}_gloo.json; echo; [ $rc -eq 0 ] || exit $rc
done
