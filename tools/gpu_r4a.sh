#!/bin/bash
# Round 4, first call: the shipped binary's 70k bench + rocprofv3 kernel stats, then the stall PMC passes.
set -o pipefail
TAG=${1:-r04_a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cat $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_stall.sh ${TAG}_pmc
