#!/bin/bash
# Round-6 SP planner check 2: the sequence-parallel GPU tests, then the planners (sim vs r5) on the 70k slide at
# W = 8 and the 256k slide at W = 2 / 8, one process each.
set -o pipefail
TAG=${1:-r06_sp2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_seqpar.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_seqpar.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_seqpar.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/sp_rank_probe.py --tiles 70000 --worlds 8 --local-first 1 --planner sim,r5 > $OUT/sp_probe_70k.log 2>&1
rc=$?; echo "sp probe 70k rc=$rc"; grep '"W"' $OUT/sp_probe_70k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/sp_rank_probe.py --worlds 2,8 --local-first 1 --planner sim,r5 --product-ref > $OUT/sp_probe_256k.log 2>&1
rc=$?; echo "sp probe 256k rc=$rc"; grep '"W"' $OUT/sp_probe_256k.log; exit $rc
