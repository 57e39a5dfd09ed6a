#!/bin/bash
# Round 4: two-group ping-pong attention (GP_ATTN_PINGPONG lab build) vs the product, same process
set -o pipefail
TAG=${1:-r04_m}
LAB=${2:-tools/attn_lab/liblab_pp.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --libs prod,$LAB --branches all,0,2,3 --rounds 7 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn ab rc=$rc"; grep "br=\|max |d" $OUT/attn_ab.log; exit $rc
