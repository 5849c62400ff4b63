#!/bin/bash
# Round 5, call f: kernel concurrency of the C2 B=1024 step (kernel trace, tools/concurrency.py).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 11; }
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 tools/concurrency.py $f 4 > $OUT/concurrency.txt 2>&1; cat $OUT/concurrency.txt
