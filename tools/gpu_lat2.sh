#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/solver_bench > $OUT/solver_bench.txt 2>&1 || exit 30
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "stream or process_scan" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat.json 2> $OUT/lat.err || exit 31
python3 tools/trace_gaps.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) > $OUT/lat_gaps.txt || exit 32
timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat_noprof.json 2>> $OUT/lat.err || exit 33
cat $OUT/solver_bench.txt $OUT/lat_noprof.json; tail -1 $OUT/pytest.log; head -3 $OUT/lat_gaps.txt
