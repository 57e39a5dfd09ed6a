#!/bin/bash
# Round-6 A/B of the fc1 GELU epilogue variants (tools/attn_lab builds of the product sources): the isolated
# GEMM entry points (tools/gemm_ab.py) and the whole eager forward (tools/forward_ab.py), same process.
# LIBS: comma list, first = reference.  bash tools/gpu_r6_ab_gelu.sh <tag>
TAG=${1:-r06_gelu}
LIBS=${LIBS:-tools/attn_lab/liblab_head.so,prod,tools/attn_lab/liblab_geluES.so}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python tools/gemm_ab.py --libs $LIBS --only fc1_gelu,fc1_gelu_ln,out_resid --rounds 9 --out gpurun_out/$TAG/gemm_ab.json > gpurun_out/$TAG/gemm_ab.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/$TAG/gemm_ab.log | tail -16
timeout -k 10 700 python tools/forward_ab.py --libs $LIBS --rounds 7 --out gpurun_out/$TAG/forward_ab.json > gpurun_out/$TAG/forward_ab.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/$TAG/forward_ab.log | tail -5
