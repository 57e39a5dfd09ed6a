#!/bin/bash
# The three single-GPU benches of the final tree (70k C3, 256k, C5 packed).  bash tools/gpu_r5_bench3.sh <tag>
set -o pipefail
TAG=${1:-r05_final3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/b70.err || exit $?
timeout -k 10 300 python bench.py --tiles 256000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_256k.json 2> $OUT/b256.err || exit $?
timeout -k 10 300 python bench.py --mode mixed --steps 3 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bc5.err || exit $?
for f in bench_70k bench_256k bench_c5; do
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split(chr(10))[-1]); print(sys.argv[1], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])" $OUT/$f.json
done
