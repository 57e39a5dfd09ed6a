#!/bin/bash
# Attention A/B: product (2-slot K/V buffers) vs GP_ATTN_RING3 (3-slot ring, counted waits, asm V reads).
set -o pipefail
TAG=${1:-r03_s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_ring3.so --rounds 9 --out $OUT/ab_ring3.json > $OUT/ab_ring3.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab_ring3.log | tail -30; exit $rc
