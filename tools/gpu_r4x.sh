#!/bin/bash
# Round 4: split-K factor of the last, partial tile round (K = 768: out-proj; K = 3072: fc2) vs the product's 2 / 4
set -o pipefail
TAG=${1:-r04_x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=tools/attn_lab
timeout -k 10 600 python tools/forward_ab.py --libs prod,$L/liblab_s13.so,$L/liblab_s33.so,$L/liblab_l2.so,$L/liblab_l8.so --rounds 7 --out $OUT/forward_ab.json > $OUT/forward_ab.log 2>&1
rc=$?; echo "forward ab rc=$rc"; grep forward_ms $OUT/forward_ab.log | cut -c1-230; exit $rc
