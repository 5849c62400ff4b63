#!/bin/bash
# Kernel trace of the pose-chained single-scan chain (latency line), summarised per scan.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat.json 2> $OUT/lat.err || exit 31
python3 tools/trace_gaps.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) > $OUT/lat_gaps.txt || exit 32
cat $OUT/lat_gaps.txt
