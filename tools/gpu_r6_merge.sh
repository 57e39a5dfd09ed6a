#!/bin/bash
# Round-6 merge pass: the merge / batch / key-part kernel tests on the new merge kernel, then the same-process
# A/B of the 70k merge against the round-5 kernel (liblab_mold) and the x8 lane mapping (liblab_mx8).
# bash tools/gpu_r6_merge.sh <tag> [ab-only]
set -o pipefail
TAG=${1:-r06_merge}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "$2" != "ab-only" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_batch.py -m gpu -q --timeout 300 --timeout-method thread -k "merge or batch or packed or varlen or key_parts" > $OUT/pytest_merge.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_merge.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 300 python tools/merge_ab.py --libs ${LIBS:-prod,tools/attn_lab/liblab_mold.so} --out $OUT/merge_ab.json > $OUT/merge_ab.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/merge_ab.log; exit $rc
