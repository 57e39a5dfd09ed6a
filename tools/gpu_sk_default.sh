#!/bin/bash
# which kernels hipBLASLt's default (heuristic) solution runs for the 70k bias GEMMs, and the forward A/B
OUT=gpurun_out/skdef; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GIGAPATH_TUNED_GEMMS_FILE=tools/tuned_default_bias.csv timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "
import csv,glob
f=glob.glob('$OUT/prof/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'Cijk' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:150])
"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/base_$i.json 2>/dev/null || exit 1
  GIGAPATH_TUNED_GEMMS_FILE=tools/tuned_default_bias.csv timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/def_$i.json 2>/dev/null || exit 1
  python -c "import json; a=json.load(open('$OUT/base_$i.json')); b=json.load(open('$OUT/def_$i.json')); print('tuned', a['ms_per_step'], {k: v for k, v in a['kernel_ms_per_step'].items() if 'gemm' in k}); print('dflt ', b['ms_per_step'], {k: v for k, v in b['kernel_ms_per_step'].items() if 'gemm' in k})"
done
