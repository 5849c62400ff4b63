#!/bin/bash
# Round profile: the default bench line (with CPU baseline), a rocprofv3 --kernel-trace --stats pass
# of the same command, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) -> profiles/hbm_traffic.json
# and a final bench line that picks the traffic up.  usage: tools/profile_round.sh rNN
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
CMD="bench.py --steps 10 --warmup 3 --latency 0 --ingest 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $CMD --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 $CMD --no-cpu-baseline > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 $CMD --no-cpu-baseline > $OUT/bench_write.log 2>&1 || exit 13
python3 tools/hbm_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") C2 ${BATCH:-1024} $OUT/hbm_traffic.json || exit 14
cp $OUT/hbm_traffic.json profiles/hbm_traffic.json
timeout -k 10 600 python3 bench.py > $OUT/bench_final.log 2>&1 || exit 15
python3 tools/roofline_check.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/bench_trace.log > $OUT/roofline_check.txt 2>&1 || exit 16
find $OUT -name "*stats.csv" -o -name "*.json" | head
