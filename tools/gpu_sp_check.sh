#!/bin/bash
# Sequence-parallel rehearsal on a one-GPU box: bench.py with W ranks on cuda:0 over gloo.
TAG=${1:-sp}; W=${2:-2}; TILES=${3:-70000}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GP_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $W \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus $W --steps 2 --warmup 1 --tiles $TILES \
    > $OUT/bench_sp$W.json 2> $OUT/bench_sp$W.err
rc=$?; echo "sp bench rc=$rc"; cat $OUT/bench_sp$W.json; [ $rc -eq 0 ] || tail -30 $OUT/bench_sp$W.err
exit $rc
