#!/bin/bash
# split VoxelGrid for few-segment calls: parity tests, latency line with / without it, kernel
# trace of the pose-chained single-scan chain (per-scan timeline)
set -o pipefail
OUT=gpurun_out/r04u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "split_voxel or voxel_grid_inplace or voxel_grid_large" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
for e in "FBR_VG_SPLIT=4" "FBR_VG_SPLIT=1" "FBR_VG_SPLIT=8"; do
  env $e timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat_$e.json 2>> $OUT/lat.err || exit 22
  echo "$e $(python3 -c "import json; l=json.loads(open('$OUT/lat_$e.json').read().strip().splitlines()[-1]); print(l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['host_ms_per_scan'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/lat -o lat -- python3 tools/latency_probe.py 40 C2 > $OUT/lat_trace.json 2> $OUT/lat_trace.err || exit 31
python3 tools/scan_timeline.py $(find $OUT/lat -name "*kernel_trace.csv" | head -1) 20 > $OUT/scan_timeline.txt || exit 33
cat $OUT/scan_timeline.txt
