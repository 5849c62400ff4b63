#!/bin/bash
# Round 5, call u: single-scan GN grids sized from the previous scan's work items -- stream tests,
# then latency A/B against the previous build (libfbr_hip_prev.so), interleaved, 3 repeats.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_mirror.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stream or process_scan or mirror or register" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_prev.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], l['host_ms_per_scan'])"
done; done
