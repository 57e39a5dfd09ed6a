#!/bin/bash
# GEMM v8 lab kernels vs tuned hipBLASLt on the 70k encoder shapes (each in its own process, interleaved
# against hipBLASLt inside it).  Usage: bash tools/gpu_gemm8.sh <tag> <lib names...>
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
timeout -k 10 300 python tools/gemm_bench.py --lib tools/attn_lab/liblab_$v.so --rounds 7 --iters 10 \
    --out $OUT/$v.json > $OUT/$v.log 2>&1
rc=$?; echo "== $v"; grep -v amdgpu.ids $OUT/$v.log; [ $rc -eq 0 ] || exit $rc
done
