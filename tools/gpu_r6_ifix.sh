#!/bin/bash
# Round-6 lab: the fixup pass folded into the fast kernel (GP_ATTN_INLINE_FIX, out-of-line call / inlined) --
# the fixup tests on each lab build, then the 70k attention launch A/B against the product (fast + fixup launch).
set -o pipefail
TAG=${1:-r06_ifix}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
for L in ifix ifix2; do
  timeout -k 10 300 python -u tools/lab_fixup_check.py tools/attn_lab/liblab_$L.so > $OUT/check_$L.log 2>&1
  rc=$?; echo "check $L rc=$rc"; tail -2 $OUT/check_$L.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_ifix.so,tools/attn_lab/liblab_ifix2.so --rounds 9 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn_ab rc=$rc"; tail -12 $OUT/attn_ab.log; exit $rc
