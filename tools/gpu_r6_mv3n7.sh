#!/bin/bash
# Round-6 lab: the 7-entry (SP key parts) merge on the v3 kernel vs v2 -- SP rank probe, W = 8, ranks 0 and 7,
# product library then the lab build, one GPU call.
set -o pipefail
TAG=${1:-r06_mv3n7}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/sp_rank_probe.py --worlds 8 --ranks 0,7 --local-first 1 > $OUT/sp_prod.log 2>&1
rc=$?; echo "prod rc=$rc"; grep '"W"' $OUT/sp_prod.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sp_rank_probe.py --worlds 8 --ranks 0,7 --local-first 1 --lib tools/attn_lab/liblab_mv3n7.so > $OUT/sp_lab.log 2>&1
rc=$?; echo "lab rc=$rc"; grep '"W"' $OUT/sp_lab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/sp_rank_probe.py --worlds 8 --ranks 0,7 --local-first 1 > $OUT/sp_prod2.log 2>&1
rc=$?; echo "prod2 rc=$rc"; grep '"W"' $OUT/sp_prod2.log; exit $rc
