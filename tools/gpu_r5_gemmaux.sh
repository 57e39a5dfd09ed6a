#!/bin/bash
# GEMM K-tile DMA cache-policy A/B (lab builds with -DGP_GEMM_AUX_A=2 / -DGP_GEMM_AUX_W=2, non-temporal A or W
# loads) against the product in one process.  bash tools/gpu_r5_gemmaux.sh <tag>
set -o pipefail
TAG=${1:-r05_gaux}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/forward_ab.py --libs prod,tools/attn_lab/liblab_ant.so,tools/attn_lab/liblab_wnt.so --rounds 7 > $OUT/forward_ab.json 2> $OUT/forward_ab.err
rc=$?; echo "forward_ab rc=$rc"; tail -c 1500 $OUT/forward_ab.json; exit $rc
