#!/bin/bash
# Round-6 baseline pass: golden headroom with the residual fusion on / off, the graph-replay bench A/B of
# that switch, and rocprofv3 kernel stats of the default bench.  bash tools/gpu_r6_base.sh <tag>
set -o pipefail
TAG=${1:-r06_base}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/golden_rel.py --tag fused > $OUT/golden_rel.jsonl 2> $OUT/golden_rel.err || exit $?
timeout -k 10 300 env GIGAPATH_RESID_FUSED=0 python tools/golden_rel.py --tag unfused >> $OUT/golden_rel.jsonl 2>> $OUT/golden_rel.err || exit $?
cat $OUT/golden_rel.jsonl
bash tools/gpu_r5_benchab.sh $TAG/rf GIGAPATH_RESID_FUSED 3 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --no-c4-ref > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
