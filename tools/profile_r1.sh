#!/bin/bash
# rocprofv3 kernel-trace/stats pass, then separate PMC passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_r1
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_write.log 2>&1 || exit 13
find $OUT -name "*.csv" | head -20
