#!/bin/bash
# Round-5 SP pass: the sequence-parallel GPU tests, then the per-rank probe (W = 1 and 8, local-first off and
# on) with the product's one-GPU encoder as the denominator.  bash tools/gpu_r5_sp.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r05_sp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "skip-tests" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_seqpar.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu_seqpar.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu_seqpar.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u tools/sp_rank_probe.py --worlds 1,8 --local-first 0,1 --product-ref > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -1 $OUT/probe.log | cut -c1-300; exit $rc
