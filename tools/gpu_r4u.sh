#!/bin/bash
# Round 4: the LN-folded consumers (QKV, fc1) walking their tiles newest-written rows first (GP_GEMM_REVERSE
# lab build) vs the product, same process
set -o pipefail
TAG=${1:-r04_u}
LAB=${2:-tools/attn_lab/liblab_rev.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python tools/forward_ab.py --libs prod,$LAB --rounds 9 --out $OUT/forward_ab.json > $OUT/forward_ab.log 2>&1
rc=$?; echo "forward ab rc=$rc"; grep forward_ms $OUT/forward_ab.log | cut -c1-250; exit $rc
