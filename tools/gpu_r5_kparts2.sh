#!/bin/bash
# Round-5 key parts (ABI 10), the engine's rule: full GPU test suite, then the SP rank probe at W = 8 (every
# rank) with the rule and without parts, and W = 4 with the rule.  Usage: bash tools/gpu_r5_kparts2.sh <tag>
set -o pipefail
TAG=${1:-r05_kp2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/sp_rank_probe.py --worlds 8 --local-first 1 --key-parts default,none > $OUT/probe_w8.log 2>&1
rc=$?; echo "probe w8 rc=$rc"; grep '"W"' $OUT/probe_w8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/sp_rank_probe.py --worlds 4 --local-first 1 --key-parts default,none > $OUT/probe_w4.log 2>&1
rc=$?; echo "probe w4 rc=$rc"; grep '"W"' $OUT/probe_w4.log; exit $rc
