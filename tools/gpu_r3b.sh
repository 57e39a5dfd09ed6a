#!/bin/bash
# GEMM v8 vs hipBLASLt, then the fp16 flag-rate / worst-case fixup tool.
set -o pipefail
OUT=gpurun_out/r03_b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in gemm8 gemm8np; do
timeout -k 10 300 python tools/gemm_bench.py --lib tools/attn_lab/liblab_$v.so --rounds 7 --iters 10 \
    --out $OUT/$v.json > $OUT/$v.log 2>&1
rc=$?; echo "== $v"; grep -v amdgpu.ids $OUT/$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/fp16_flag_rate.py --out $OUT/fp16_flag_rate.json > $OUT/fp16_flag_rate.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/fp16_flag_rate.log; exit $rc
