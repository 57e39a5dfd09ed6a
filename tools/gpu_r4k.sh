#!/bin/bash
# Round 4: the fp16 exact attention kernel with its -m_run start from one MFMA (GP_ATTN_EXACT_MI lab build)
set -o pipefail
TAG=${1:-r04_k}
LAB=${2:-tools/attn_lab/liblab_exmi.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --fp16 --libs prod,$LAB --branches all,0,2 --rounds 7 --out $OUT/attn_ab_fp16.json > $OUT/attn_ab_fp16.log 2>&1
rc=$?; echo "attn ab fp16 rc=$rc"; grep "br=\|max |d" $OUT/attn_ab_fp16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/attn_ab.py --libs prod,$LAB --branches all --rounds 5 --out $OUT/attn_ab_bf16.json > $OUT/attn_ab_bf16.log 2>&1
rc=$?; echo "attn ab bf16 rc=$rc"; grep "br=\|max |d" $OUT/attn_ab_bf16.log; exit $rc
