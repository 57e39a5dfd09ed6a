#!/bin/bash
# Round-5 A/B: bash tools/gpu_r5_ab.sh <tag> <tool.py> <args...>   (one GPU step, own time limit)
set -o pipefail
TAG=$1; TOOL=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u $TOOL "$@" --out $OUT/ab.json > $OUT/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -12 $OUT/ab.log; exit $rc
