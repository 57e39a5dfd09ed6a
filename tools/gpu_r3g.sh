#!/bin/bash
# Fixup-pass granularity: no-flag overhead (attn_ab, random data) and flagged-row cost (flag tool, bf16).
set -o pipefail
OUT=gpurun_out/r03_g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/attn_ab.py --libs prod,tools/attn_lab/liblab_fix2.so,tools/attn_lab/liblab_fix4.so,tools/attn_lab/liblab_fix8.so,tools/attn_lab/liblab_fix32.so \
   --rounds 9 --out $OUT/ab_fix.json > $OUT/ab_fix.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/ab_fix.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/fp16_flag_rate.py --fmt bf16 --libs fix4,fix8,fix32,nofix --scales 1,8,16 \
   --out $OUT/flag_bf16.json > $OUT/flag_bf16.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/flag_bf16.log; exit $rc
