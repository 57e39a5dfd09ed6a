#!/bin/bash
# Fused FFN bring-up: GEMM / FFN kernel tests, FFN + linear A/B timing (bf16, fp16), e2e model tests, 70k bench.
set -o pipefail
TAG=${1:-r03_k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ffn_bench.py --out $OUT/ffn_bf16.json > $OUT/ffn_bf16.log 2>&1
rc=$?; echo "ffn bf16 rc=$rc"; grep -A3 '"ffn"\|"parts"' $OUT/ffn_bf16.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ffn_bench.py --half --out $OUT/ffn_f16.json > $OUT/ffn_f16.log 2>&1
rc=$?; echo "ffn f16 rc=$rc"; grep -A3 '"ffn"' $OUT/ffn_f16.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_model.log 2>&1
rc=$?; echo "model tests rc=$rc"; tail -3 $OUT/pytest_model.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cat $OUT/bench_70k.json; exit $rc
