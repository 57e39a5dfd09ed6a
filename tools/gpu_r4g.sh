#!/bin/bash
# Round 4: per-branch attention rates of the product kernel (which branch's work items run below the
# whole-launch rate) and the merge kernel's rate.
set -o pipefail
TAG=${1:-r04_g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --libs prod --branches all,0,1,2,3,4 --rounds 7 --out $OUT/attn_branches.json > $OUT/attn_branches.log 2>&1
rc=$?; echo "attn branches rc=$rc"; grep "br=" $OUT/attn_branches.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/attn_ab.py --libs prod --merge --rounds 7 --out $OUT/merge.json > $OUT/merge.log 2>&1
rc=$?; echo "merge rc=$rc"; grep "br=" $OUT/merge.log; exit $rc
