#!/bin/bash
# Round 4: attention launch tunables re-checked on the round-4 kernel (XCD grouping G, static priority)
set -o pipefail
TAG=${1:-r04_r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_kfirst.so,tools/attn_lab/liblab_xg4.so,tools/attn_lab/liblab_xg16.so,tools/attn_lab/liblab_prio0.so --branches all --rounds 9 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn ab rc=$rc"; grep "br=\|max |d" $OUT/attn_ab.log; exit $rc
