#!/bin/bash
# Round-6 SP planner check: per-rank compute of the W = 8 / 4 / 2 plans of the C4 slide, the simulated-launch
# planner (sim, sim0 = without the phase variant) against round 5's (r5), one process, + the product 1-GPU ref.
set -o pipefail
TAG=${1:-r06_sp1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u tools/sp_rank_probe.py --worlds 8,4,2 --local-first 1 --planner sim,r5 --product-ref > $OUT/sp_probe.log 2>&1
rc=$?; echo "sp probe rc=$rc"; grep '"W"' $OUT/sp_probe.log; exit $rc
