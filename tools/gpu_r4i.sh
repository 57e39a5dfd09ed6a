#!/bin/bash
# Round 4: persistent attention variants (2: K/V tile 0 staged ahead, Q in the prologue; 3: no staging ahead)
set -o pipefail
TAG=${1:-r04_i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_persist2.so,tools/attn_lab/liblab_persist3.so --branches all,0,2 --rounds 7 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn ab rc=$rc"; grep "br=\|max |d" $OUT/attn_ab.log; exit $rc
