#!/bin/bash
# Round 4: the default 70k bench (HIP-graph replay) with the residual epilogues (product) and without
# (GIGAPATH_RESID_FUSED=0: round 3's residual_layernorm sequence), interleaved twice on one box
set -o pipefail
TAG=${1:-r04_n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/fused_$rep.json 2> $OUT/fused_$rep.err
  rc=$?; echo "fused $rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
  GIGAPATH_RESID_FUSED=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/unfused_$rep.json 2> $OUT/unfused_$rep.err
  rc=$?; echo "unfused $rep rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r04_n*/*.json")):
    d = json.loads(open(f).read().strip().split("\n")[-1])
    print(f.split("/")[-1], d["ms_per_step"], {k: v for k, v in d["kernel_ms_per_step"].items()})
PY
