#!/bin/bash
# Round-5 occupancy change check: attention GPU tests + fp16 (V-bf16) attention A/B + forward A/B vs the
# round-4-order build (tools/attn_lab/liblab_r4a.so: GP_ATTN_FAST_WPS=4).  Usage: bash tools/gpu_r5_occ.sh <tag>
set -o pipefail
TAG=${1:-r05_occ}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_kernels.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_r4a.so --rounds 9 --vbf16 --out $OUT/ab_vbf16.json > $OUT/ab_vbf16.log 2>&1
rc=$?; echo "ab vbf16 rc=$rc"; tail -2 $OUT/ab_vbf16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/forward_ab.py --libs prod,tools/attn_lab/liblab_r4a.so --rounds 7 --out $OUT/fwd.json > $OUT/fwd.log 2>&1
rc=$?; echo "fwd rc=$rc"; tail -2 $OUT/fwd.log | cut -c1-300; exit $rc
