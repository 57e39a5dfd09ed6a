#!/bin/bash
# Round 4: upper bound of the GELU table's LDS bank conflicts in the fc1 epilogue (timing-only lab build
# whose lookups use conflict-free, wrong addresses) vs the product
set -o pipefail
TAG=${1:-r04_l}
LAB=${2:-tools/attn_lab/liblab_lutnc.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python tools/forward_ab.py --libs prod,$LAB --rounds 7 --out $OUT/forward_ab.json > $OUT/forward_ab.log 2>&1
rc=$?; echo "forward ab rc=$rc"; grep forward_ms $OUT/forward_ab.log | cut -c1-250; exit $rc
