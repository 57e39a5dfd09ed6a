#!/bin/bash
# r02_s6 A/B: idle-wave skip (product, GP_ATTN_SKIP_IDLE=1) vs without (lab build)
set -o pipefail
OUT=gpurun_out/s6d; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/attn_ab.py --libs prod,tools/attn_lab/liblab_noskip.so --rounds 9 --out $OUT/ab_skip.json > $OUT/ab_skip.log 2>&1
rc=$?; tail -4 $OUT/ab_skip.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -v --timeout 300 --timeout-method thread -k "hip_graph or fp16" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; exit $rc
