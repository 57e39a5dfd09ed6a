#!/bin/bash
# v8 GEMM variants vs hipBLASLt; fp16 / bf16 flag-rate and fixup cost.
set -o pipefail
OUT=gpurun_out/r03_d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_gemm8.sh r03_d gemm8 gemm8np || exit $?
for f in fp16 bf16; do
timeout -k 10 300 python tools/fp16_flag_rate.py --fmt $f --out $OUT/flag_rate_$f.json > $OUT/flag_rate_$f.log 2>&1
rc=$?; echo "== $f"; grep -v amdgpu.ids $OUT/flag_rate_$f.log; [ $rc -eq 0 ] || exit $rc
done
