#!/bin/bash
# Round 4: the residual epilogues -- GEMM + model tests, then the 70k bench + rocprof, then the stall PMC passes.
set -o pipefail
TAG=${1:-r04_b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
rc=$?; echo "pytest gemm rc=$rc"; tail -3 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 700 --timeout-method thread > $OUT/pytest_model.log 2>&1
rc=$?; echo "pytest model rc=$rc"; tail -3 $OUT/pytest_model.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_concurrent.py -x -v --timeout 400 --timeout-method thread > $OUT/pytest_concurrent.log 2>&1
rc=$?; echo "pytest concurrent rc=$rc"; tail -3 $OUT/pytest_concurrent.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cat $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/forward_ab.py --libs prod,prod:noresid,tools/attn_lab/liblab_st2.so,tools/attn_lab/liblab_st4.so --rounds 5 --out $OUT/forward_ab.json > $OUT/forward_ab.log 2>&1
rc=$?; echo "forward ab rc=$rc"; cat $OUT/forward_ab.log | grep forward_ms | cut -c1-300
