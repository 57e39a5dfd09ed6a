#!/bin/bash
# bf16 GELU by table in gp_ffn_fc1_gelu: the GEMM tests (bit-exact h vs torch's GELU of the kernel's own
# pre-activation, every bf16 value), fused FFN A/B against the previous build (lab library), 70k bench.
set -o pipefail
TAG=${1:-r03_u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
rc=$?; echo "pytest gemm rc=$rc"; tail -3 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ffn_bench.py --lab tools/attn_lab/liblab_gemm_head.so --out $OUT/ffn_lut_vs_head.json > $OUT/ffn_bench.log 2>&1
rc=$?; echo "ffn_bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/ffn_bench.log; exit $rc; }
python -c "import json;d=json.load(open('$OUT/ffn_lut_vs_head.json'));print(d['ffn'], {k:v for k,v in d['parts'].items() if 'fc1' in k}, d.get('lab_vs_product_ffn_rel_diff'))"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_70k.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_70k.json'));print(d['ms_per_step'], d.get('kernel_ms_per_step'), d['value'])"
