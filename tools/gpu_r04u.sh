#!/bin/bash
# kernel trace of the pose-chained single-scan chain at HEAD: per-scan timeline and gaps
set -o pipefail
OUT=gpurun_out/r04u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat.json 2> $OUT/lat.err || exit 31
python3 tools/trace_gaps.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) > $OUT/lat_gaps.txt || exit 32
python3 tools/scan_timeline.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) 20 > $OUT/scan_timeline.txt || exit 33
cat $OUT/scan_timeline.txt; head -5 $OUT/lat_gaps.txt
