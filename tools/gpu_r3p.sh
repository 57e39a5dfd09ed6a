#!/bin/bash
# A/B: projections on gp_linear (GIGAPATH_OWN_GEMMS=1) vs hipBLASLt, alternating; then the 4-stream
# concurrent-replay test with every GEMM of the forward on gp_linear / the fused FFN (no stream-K kernel).
set -o pipefail
TAG=${1:-r03_p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for own in 1 0; do
    GIGAPATH_OWN_GEMMS=$own timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_own${own}_$i.json 2> $OUT/bench_own${own}_$i.err
    rc=$?; echo "own=$own $i rc=$rc $(python -c "import json;d=json.load(open('$OUT/bench_own${own}_$i.json'));print(d['ms_per_step'], d['kernel_ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
  done
done
GIGAPATH_OWN_GEMMS=1 timeout -k 10 170 python -u -m pytest tests/test_gpu_concurrent.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_concurrent_own.log 2>&1
rc=$?; echo "4-stream (own GEMMs) rc=$rc"; tail -5 $OUT/pytest_concurrent_own.log; exit $rc
