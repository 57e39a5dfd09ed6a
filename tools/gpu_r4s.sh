#!/bin/bash
# Round 4: XCD grouping G = 2 / 4 vs the product's 8, more rounds, whole launch and branches 0 / 2
set -o pipefail
TAG=${1:-r04_s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_xg4.so,tools/attn_lab/liblab_xg2.so --branches all,0,2 --rounds 15 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn ab rc=$rc"; grep "br=\|max |d" $OUT/attn_ab.log; exit $rc
