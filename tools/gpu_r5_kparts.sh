#!/bin/bash
# Round-5 key parts (ABI 10): attention kernel tests, then the SP rank probe (W = 8) over key-part settings
# in one process.  Usage: bash tools/gpu_r5_kparts.sh <tag> [ranks] [settings]
set -o pipefail
TAG=${1:-r05_kp}
RANKS=${2:-0,5,7}
KP=${3:-none,3=2/4=2,1=2,1=2/3=2/4=2,3=2,1=4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/sp_rank_probe.py --worlds 8 --ranks $RANKS --local-first 1 --key-parts $KP > $OUT/probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep '"W"' $OUT/probe.log; exit $rc
