#!/bin/bash
# r02_s6: full GPU test suite (no -x: see every failure), then the 70k bench if the tests ended
# normally (exit 0 or 1 = test failures; anything else -- fault, abort, timeout -- stops here)
OUT=gpurun_out/s6c; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_gpu.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc2=$?; echo "bench rc=$rc2"; cat $OUT/bench_70k.json; exit $(( rc > rc2 ? rc : rc2 ))
