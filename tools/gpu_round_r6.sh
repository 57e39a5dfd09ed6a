#!/bin/bash
# Round-6 pass: every GPU test, smoke, the default bench (70k C3, CPU baseline on the usable cores),
# rocprof kernel stats, the 256k single-GPU slide, the C5 packed batch, the fp16 caller timing, the
# FETCH_SIZE / WRITE_SIZE passes that give bench.py its roofline.traffic, and the SP rank probe.
# Usage: bash tools/gpu_round_r6.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r06_fin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; cp gpurun_out/parity_metrics.json $OUT/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench70k rc=$rc"; cut -c1-400 $OUT/bench_70k.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c4-ref > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/fetch -o run -- python bench.py --no-cpu-baseline --no-c4-ref --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/write -o run -- python bench.py --no-cpu-baseline --no-c4-ref --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --tiles 256000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_256k.json 2> $OUT/bench_256k.err
rc=$?; echo "bench256k rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --mode mixed --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err
rc=$?; echo "benchC5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fp16_caller_bench.py > $OUT/fp16_caller.log 2>&1
rc=$?; echo "fp16 caller rc=$rc"; tail -4 $OUT/fp16_caller.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/sp_rank_probe.py --worlds 1,8 --local-first 1 --product-ref > $OUT/sp_probe.log 2>&1
rc=$?; echo "sp probe rc=$rc"; exit $rc
