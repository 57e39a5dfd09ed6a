cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r01_pp1 && \
GP_ATTN_VAR=1538 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "prescaled and not impl" > gpurun_out/r01_pp1/k1538.log 2>&1; echo "k1538 rc=$?"; tail -2 gpurun_out/r01_pp1/k1538.log
