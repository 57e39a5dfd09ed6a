#!/bin/bash
# Map TunableOp's hipBLASLt solution ids to kernel names (stream-K or not) and time every candidate of
# the 70k-tile GEMM shapes (TunableOp verbose log), so a non-stream-K tuning can be chosen per shape.
OUT=gpurun_out/skmap; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/hipblaslt_algos 618384 618464 618465 618466 618467 618611 618612 618613 618614 > $OUT/names_csv.txt 2>&1 || exit $?
cat $OUT/names_csv.txt | cut -c1-160
PYTORCH_TUNABLEOP_VERBOSE=3 timeout -k 10 600 python -u tools/tune_gemms.py --sp-tiles 70000 --sp-worlds 1 --fresh --out $OUT/tuned_fresh.csv > $OUT/tune_verbose.log 2>&1
rc=$?; tail -2 $OUT/tune_verbose.log; [ $rc -eq 0 ] || exit $rc
grep -o "Gemm_Hipblaslt_[0-9]*" $OUT/tune_verbose.log | sort -u | sed s/Gemm_Hipblaslt_// > $OUT/cand_ids.txt
wc -l $OUT/cand_ids.txt
timeout -k 10 120 ./tools/hipblaslt_algos $(cat $OUT/cand_ids.txt | head -4000) > $OUT/names_cand.txt 2>&1
rc=$?; grep -c STREAMK $OUT/names_cand.txt; grep -c dataparallel $OUT/names_cand.txt; exit $rc
