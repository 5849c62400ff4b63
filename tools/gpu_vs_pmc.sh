#!/bin/bash
# VoxelGrid + registration parity tests, a default bench line, then the voxel_scan WRITE_SIZE /
# FETCH_SIZE PMC passes.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_vs.sh $1 || exit 21
CMD="bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 $CMD > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 $CMD > $OUT/bench_write.log 2>&1 || exit 13
python3 tools/hbm_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") C2 1024 $OUT/hbm_traffic.json > $OUT/hbm.txt || exit 14
cat $OUT/hbm.txt
