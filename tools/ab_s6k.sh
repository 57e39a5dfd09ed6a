#!/bin/bash
# r02_s6 A/B: P.V on 16x16x32 over the 3 real d-blocks (GP_ATTN_PV16 lab build) vs the product
set -o pipefail
OUT=gpurun_out/s6k; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_pv16.so --rounds 9 --out $OUT/ab_pv16.json > $OUT/ab_pv16.log 2>&1
rc=$?; tail -5 $OUT/ab_pv16.log; exit $rc
