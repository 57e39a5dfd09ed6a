#!/bin/bash
# Round-5 baseline on this round's box: the default 70k bench (no CPU leg), rocprof kernel stats of the
# same command, and the per-epilogue GEMM cost probe.
set -o pipefail
TAG=${1:-r05_base}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-c4-ref > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cut -c1-400 $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c4-ref > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/epi_cost.py --out $OUT/epi_cost.json > $OUT/epi_cost.log 2>&1
rc=$?; echo "epi rc=$rc"; tail -20 $OUT/epi_cost.log; exit $rc
