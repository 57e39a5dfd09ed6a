#!/bin/bash
# Round-6 lab: the merge with block-staged LSEs (GP_MERGE_V3) against the product's v2 merge, 70k and 256k shapes.
set -o pipefail
TAG=${1:-r06_mv3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/merge_ab.py --libs prod,tools/attn_lab/liblab_mv3e32.so,tools/attn_lab/liblab_mv3e24.so,tools/attn_lab/liblab_mv3e16.so --rounds 9 --out $OUT/merge_ab_70k.json > $OUT/merge_ab_70k.log 2>&1
rc=$?; echo "merge_ab 70k rc=$rc"; tail -4 $OUT/merge_ab_70k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/merge_ab.py --libs prod,tools/attn_lab/liblab_mv3e32.so,tools/attn_lab/liblab_mv3e24.so,tools/attn_lab/liblab_mv3e16.so --rounds 5 --L 256001 --out $OUT/merge_ab_256k.json > $OUT/merge_ab_256k.log 2>&1
rc=$?; echo "merge_ab 256k rc=$rc"; tail -4 $OUT/merge_ab_256k.log; exit $rc
