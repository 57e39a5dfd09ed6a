#!/bin/bash
# Round 4: stall attribution PMC passes on the 70k bench (tools/pmc_stall.sh) + the summary.
set -o pipefail
TAG=${1:-r04_c}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_stall.sh ${TAG}_pmc && python tools/stall_report.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc/stall_report.json
