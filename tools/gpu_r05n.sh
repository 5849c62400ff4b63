#!/bin/bash
# Round 5, call n: SQ counters per kNN kernel, balanced (FBR_KNN_BAL=1) vs per-lane flat walk.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
CMD="bench.py --batch 256 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in 1 0; do
  FBR_KNN_BAL=$v timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/bal$v -o pmc --output-format csv -- python3 $CMD > $OUT/bal$v.log 2>&1 || { tail $OUT/bal$v.log; exit 3; }
  python3 tools/pmc_by_kernel.py $(find $OUT/bal$v -name "*counter_collection.csv" | head -1) k_gn_knn > $OUT/bal$v.txt || exit 4
  echo "== bal=$v"; cat $OUT/bal$v.txt
done
