#!/bin/bash
# Round 5, call u: latency at HEAD against the build of 2bf1c20 (before the stream-mode window) -- tests,
# then latency A/B against the previous build (libfbr_hip_r05h.so), interleaved, 3 repeats.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05v
mkdir -p $OUT
true
true
for rep in 1 2 3; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_r05h.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], l['host_ms_per_scan'])"
done; done
