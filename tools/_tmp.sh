cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r01_pp1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "window" > gpurun_out/r01_pp1/k.log 2>&1; rc=$?; echo "kern rc=$rc"; tail -3 gpurun_out/r01_pp1/k.log; [ $rc -eq 0 ] || exit 1; \
timeout -k 10 200 python tools/attn_bench.py --iters 12 --impls 2p@2,2p@514,2p@1538,2p@1026,2p@2,2p@1538 > gpurun_out/r01_pp1/ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r01_pp1/ab.log
