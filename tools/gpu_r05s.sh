#!/bin/bash
# Round 5, call s: single-scan timeline at HEAD (C2, kernel trace of the latency probe).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/lat -o lat --output-format csv -- python3 tools/latency_probe.py 40 > $OUT/probe.log 2>&1 || { tail $OUT/probe.log; exit 3; }
python3 tools/scan_timeline.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) 30 > $OUT/timeline.txt || exit 4
cat $OUT/timeline.txt; tail -1 $OUT/probe.log
