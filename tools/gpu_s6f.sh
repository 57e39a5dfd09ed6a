#!/bin/bash
# r02_s6: re-tune the 70k GEMM shapes with a 1 GB rotating buffer (cold operands), then A/B the forward
OUT=gpurun_out/s6f; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u tools/tune_gemms.py --tiles 70000 --rotating-mb 1024 --fresh --out $OUT/tuned_rot.csv > $OUT/tune.log 2>&1
rc=$?; tail -3 $OUT/tune.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/base_$i.json 2>/dev/null || exit 1
  GIGAPATH_TUNED_GEMMS_FILE=$OUT/tuned_rot.csv timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/rot_$i.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('$OUT/base_$i.json')); b=json.load(open('$OUT/rot_$i.json')); print('base', a['ms_per_step'], a['kernel_ms_per_step']); print('rot ', b['ms_per_step'], b['kernel_ms_per_step'])"
done
