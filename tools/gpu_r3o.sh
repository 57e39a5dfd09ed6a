#!/bin/bash
# Forward A/B on one box: fused FFN (default) vs GIGAPATH_FFN_FUSED=0 (hipBLASLt fc1 + GELU+LN + fc2),
# alternating, then the 4-stream concurrent graph-replay test once, on its own.
set -o pipefail
TAG=${1:-r03_o}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_fused_$i.json 2> $OUT/bench_fused_$i.err
  rc=$?; echo "fused $i rc=$rc $(python -c "import json;d=json.load(open('$OUT/bench_fused_$i.json'));print(d['ms_per_step'], d['kernel_ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
  GIGAPATH_FFN_FUSED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_unfused_$i.json 2> $OUT/bench_unfused_$i.err
  rc=$?; echo "unfused $i rc=$rc $(python -c "import json;d=json.load(open('$OUT/bench_unfused_$i.json'));print(d['ms_per_step'], d['kernel_ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_concurrent.py -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_concurrent.log 2>&1
rc=$?; echo "4-stream rc=$rc"; tail -3 $OUT/pytest_concurrent.log; exit $rc
