#!/bin/bash
# r02_s6 A/B: sparse ones row in the V image (GP_ATTN_ONES_SPARSE) vs product; MFMA shape probe
set -o pipefail
OUT=gpurun_out/s6ab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/mfma_probe > $OUT/mfma_probe.txt 2>&1 || exit $?
cat $OUT/mfma_probe.txt
timeout -k 10 400 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_ones.so --rounds 9 --out $OUT/ab_ones.json > $OUT/ab_ones.log 2>&1
rc=$?; tail -8 $OUT/ab_ones.log; exit $rc
