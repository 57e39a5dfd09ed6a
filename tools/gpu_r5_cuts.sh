#!/bin/bash
# Shard-cut check: the SP rank probe at W = 2 with the plan's cut and explicit ones.  bash tools/gpu_r5_cuts.sh <tag>
set -o pipefail
TAG=${1:-r05_cuts}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/sp_rank_probe.py --worlds 2 --local-first 1 --bounds plan,cuts:124928,cuts:126976,plan > $OUT/probe_w2.log 2>&1
rc=$?; echo "probe w2 rc=$rc"; grep '"W"' $OUT/probe_w2.log; exit $rc
