#!/bin/bash
# Round-6 lab: attention work items run in pairs per workgroup (GP_ATTN_PAIR=2) vs the product, 70k launch A/B.
set -o pipefail
TAG=${1:-r06_pair}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_pair2.so --rounds 9 --out $OUT/attn_ab.json > $OUT/attn_ab.log 2>&1
rc=$?; echo "attn_ab rc=$rc"; tail -4 $OUT/attn_ab.log; exit $rc
