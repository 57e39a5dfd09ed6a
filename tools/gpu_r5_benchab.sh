#!/bin/bash
# Round-5 bench A/B of a host-path environment switch: bash tools/gpu_r5_benchab.sh <tag> <VAR> [rounds]
# alternates python bench.py (HIP-graph replay, 20 steps) with VAR unset and VAR=0, one process per run.
set -o pipefail
TAG=$1; VAR=$2; N=${3:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 $N); do
  timeout -k 10 240 python bench.py --steps 20 --no-cpu-baseline --no-c4-ref > $OUT/on_$i.json 2> $OUT/on_$i.err || exit $?
  timeout -k 10 240 env $VAR=0 python bench.py --steps 20 --no-cpu-baseline --no-c4-ref > $OUT/off_$i.json 2> $OUT/off_$i.err || exit $?
  python -c "import json; a=json.load(open('$OUT/on_$i.json')); b=json.load(open('$OUT/off_$i.json')); print('round $i on', a['ms_per_step'], 'off', b['ms_per_step'])"
done
