#!/bin/bash
# Round 4: persistent attention workgroups (GP_ATTN_PERSIST lab build) vs the product, same process.
set -o pipefail
TAG=${1:-r04_h}
LAB=${2:-tools/attn_lab/liblab_persist.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --libs prod,$LAB --branches all,0,1,2,3,4 --rounds 7 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn ab rc=$rc"; grep "br=\|max |d" $OUT/attn_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/forward_ab.py --libs prod,$LAB --rounds 5 --out $OUT/forward_ab.json > $OUT/forward_ab.log 2>&1
rc=$?; echo "forward ab rc=$rc"; grep forward_ms $OUT/forward_ab.log | cut -c1-250; exit $rc
