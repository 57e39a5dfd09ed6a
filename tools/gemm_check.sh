# Lab GEMM vs hipBLASLt on the encoder's shapes (tools/gemm_bench.py); usage: bash tools/gemm_check.sh TAG
set -o pipefail
TAG=${1:-gemm}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/gemm_bench.py --out gpurun_out/$TAG/gemm.json > gpurun_out/$TAG/gemm.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/gemm.log; exit $rc
