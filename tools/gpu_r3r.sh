#!/bin/bash
# GEMM v9 lab (two workgroups per CU) vs the product GEMMs: correctness diff + interleaved timing.
set -o pipefail
TAG=${1:-r03_r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/ffn_bench.py --lab tools/attn_lab/liblab_gemm9.so --out $OUT/ffn_v9_bf16.json > $OUT/ffn_v9_bf16.log 2>&1
rc=$?; echo "v9 bf16 rc=$rc"; cat $OUT/ffn_v9_bf16.log | grep -v amdgpu.ids | tail -60; exit $rc
