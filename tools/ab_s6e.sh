#!/bin/bash
# r02_s6 A/B: GELU+LN with the LN affine in registers (GP_GELU_WREG=1, lab) vs LDS (product)
set -o pipefail
OUT=gpurun_out/s6e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/norm_ab.py --libs prod,tools/attn_lab/liblab_wreg.so --rounds 11 --out $OUT/ab_wreg.json > $OUT/ab_wreg.log 2>&1
rc=$?; tail -4 $OUT/ab_wreg.log; exit $rc
