#!/bin/bash
# Round 4: stall-attribution PMC passes on the 70k bench (tools/pmc_stall.sh + tools/stall_report.py), then the
# 8-GPU path re-rehearsed (tools/gpu_r4d.sh: sp_rank_probe W = 1 / 8, bench.py --gpus 8 over gloo on one GPU).
set -o pipefail
TAG=${1:-r04_c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_stall.sh ${TAG}_pmc && python tools/stall_report.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc/stall_report.json
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4d.sh ${TAG}_sp
