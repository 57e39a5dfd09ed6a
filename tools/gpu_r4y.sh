#!/bin/bash
# Round 4: out-proj (K = 768) without the split-K tail (liblab_s12.so: GP_GEMM_SPLIT_SHORT=1) against the
# product's split 2 -- same-process forward A/B in both orders
set -o pipefail
TAG=${1:-r04_y}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=tools/attn_lab
timeout -k 10 400 python tools/forward_ab.py --libs prod,$L/liblab_s12.so --rounds 9 --out $OUT/forward_ab1.json > $OUT/forward_ab1.log 2>&1
rc=$?; echo "forward ab1 rc=$rc"; grep forward_ms $OUT/forward_ab1.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/forward_ab.py --libs $L/liblab_s12.so,prod --rounds 9 --out $OUT/forward_ab2.json > $OUT/forward_ab2.log 2>&1
rc=$?; echo "forward ab2 rc=$rc"; grep forward_ms $OUT/forward_ab2.log | cut -c1-200; exit $rc
