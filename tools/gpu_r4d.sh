#!/bin/bash
# Round 4: the 8-GPU path re-rehearsed on the shipped product (verdict r03 item 6): per-rank compute of the
# W = 8 plan against W = 1 (sp_rank_probe, HIP graphs, exchange replaced by nothing), then the driver's
# `bench.py --gpus 8` command with 8 gloo ranks on the one GPU (host-staged transport: its time means nothing).
set -o pipefail
TAG=${1:-r04_d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/sp_rank_probe.py --worlds 1,8 --reps 3 > $OUT/sp_rank_probe.log 2> $OUT/sp_rank_probe.err
rc=$?; echo "probe rc=$rc"; tail -2 $OUT/sp_rank_probe.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
tail -1 $OUT/sp_rank_probe.log > $OUT/sp_rank_probe_w8.json
GP_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_sp8_gloo.json 2> $OUT/bench_sp8_gloo.err
rc=$?; echo "sp8 gloo rc=$rc"; tail -c 600 $OUT/bench_sp8_gloo.json; exit $rc
