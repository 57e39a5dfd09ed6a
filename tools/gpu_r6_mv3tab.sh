#!/bin/bash
# Round-6 lab: the v3 merge over packed slides (GP_MERGE_V3_TAB) -- varlen tests on the lab build + C5 merge A/B.
set -o pipefail
TAG=${1:-r06_mv3tab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/lab_varlen_merge.py tools/attn_lab/liblab_mv3tab.so > $OUT/varlen.log 2>&1
rc=$?; echo "varlen rc=$rc"; tail -6 $OUT/varlen.log; exit $rc
