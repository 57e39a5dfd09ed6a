#!/bin/bash
# Round 4: the default bench command (70k, CPU baseline on every usable core) timed end
# to end, with the box's CPU facts recorded.
set -o pipefail
TAG=${1:-r04_f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > $OUT/cpu_facts.txt 2>&1
cat $OUT/cpu_facts.txt
start=$(date +%s)
timeout -k 10 900 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?; end=$(date +%s); echo "bench default rc=$rc wall=$((end-start))s"; tail -c 1500 $OUT/bench_default.json; [ $rc -eq 0 ] || exit $rc
# residual x cache-policy lab builds (GP_GEMM_XSTORE_AUX / GP_GEMM_XLOAD_AUX) against the product build
timeout -k 10 400 python tools/forward_ab.py --libs prod,tools/attn_lab/liblab_xnt.so,tools/attn_lab/liblab_xntld.so --rounds 5 --out $OUT/forward_ab_xnt.json > $OUT/forward_ab_xnt.log 2>&1
rc=$?; echo "forward ab xnt rc=$rc"; grep forward_ms $OUT/forward_ab_xnt.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/epi_cost.py --out $OUT/epi_cost.json > $OUT/epi_cost.log 2>&1
rc=$?; echo "epi cost rc=$rc"; cat $OUT/epi_cost.log | grep -v amdgpu.ids; exit $rc
