#!/bin/bash
# quick GPU check of selected tests: bash tools/gpu_quick.sh <tag> <pytest -k expression>
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$*" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -12; exit $rc
