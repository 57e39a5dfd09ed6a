#!/bin/bash
# Full-line epilogue stores (DPP row_ror:8): GEMM tests, probe against the half-line build and an
# nt-for-every-width build, FFN A/B, 70k bench.
set -o pipefail
TAG=${1:-r03_aa}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gemm.log 2>&1
rc=$?; echo "pytest gemm rc=$rc"; tail -2 $OUT/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_overhead_probe.py --lab tools/attn_lab/liblab_gemm_halfline.so --lab tools/attn_lab/liblab_gemm_nt768.so --out $OUT/gemm_probe.json > $OUT/gemm_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids $OUT/gemm_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ffn_bench.py --lab tools/attn_lab/liblab_gemm_halfline.so --out $OUT/ffn_vs_halfline.json > $OUT/ffn_bench.log 2>&1
rc=$?; echo "ffn_bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/ffn_bench.log; exit $rc; }
python -c "import json;d=json.load(open('$OUT/ffn_vs_halfline.json'));print(d['ffn'], d['parts'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_70k.json 2> $OUT/bench_70k.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_70k.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench_70k.json'));print(d['ms_per_step'], d.get('kernel_ms_per_step'))"
