set -o pipefail; mkdir -p gpurun_out/s6b; cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "seam or attention" > gpurun_out/s6b/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/s6b/pytest.log; exit $rc
