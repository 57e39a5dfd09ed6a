#!/bin/bash
# Round 4: the 70k kernel-trace pass alone (bench line + rocprof summary from the same run, no 256k block)
set -o pipefail
TAG=${1:-r04_z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c4-ref > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep '"metric"' $OUT/prof.log | cut -c1-300; exit $rc
