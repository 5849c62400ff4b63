#!/bin/bash
# The -m gpu suite, smoke(), a default bench line, and a kernel trace of the single-scan chain.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 21; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 22
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 23
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat.json 2> $OUT/lat.err || exit 31
python3 tools/trace_gaps.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) > $OUT/lat_gaps.txt || exit 32
cat $OUT/smoke.log $OUT/lat_gaps.txt
