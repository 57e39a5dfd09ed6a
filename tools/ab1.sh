# Interleaved attention A/B of lab builds against the product (tools/attn_ab.py); usage: bash tools/ab1.sh TAG LIBS [BRANCHES]
set -o pipefail
TAG=$1; LIBS=$2; BR=${3:-all}
mkdir -p gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python tools/attn_ab.py --libs $LIBS --branches $BR --rounds 7 --out gpurun_out/$TAG/ab.json > gpurun_out/$TAG/ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/ab.log; exit $rc
