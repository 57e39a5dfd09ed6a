#!/bin/bash
# Non-temporal residual stream: GPU model / kernel tests, then the 70k bench twice.
set -o pipefail
TAG=${1:-r03_y}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k_$i.json 2> $OUT/bench_70k_$i.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_70k_$i.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_70k_$i.json'));print(d['ms_per_step'], d.get('kernel_ms_per_step'))"
done
