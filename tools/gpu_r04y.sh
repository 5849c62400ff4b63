#!/bin/bash
# single-scan path: guess copy + CropBox on a side stream forked at call start, no err fill:
# single-scan parity tests, latency lines, kernel trace of the chain
set -o pipefail
OUT=gpurun_out/r04y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "process_scan or stream or msg or features or register or split_voxel or capacity" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
for k in 1 2; do
  timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat.json 2>> $OUT/lat.err || exit 22
  echo "lat $(python3 -c "import json; l=json.loads(open('$OUT/lat.json').read().strip().splitlines()[-1]); print(l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['launches_per_scan'], l['host_ms_per_scan'], l.get('chain_max_abs_pose_diff_vs_oracle'))")" | tee -a $OUT/lat_summary.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat_trace.json 2> $OUT/lat_trace.err || exit 31
python3 tools/scan_timeline.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) 20 > $OUT/scan_timeline.txt || exit 33
cat $OUT/scan_timeline.txt
