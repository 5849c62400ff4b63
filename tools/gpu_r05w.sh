#!/bin/bash
# Round 5, call w: single-scan latency knob sweep (C2, latency probe, interleaved, 2 repeats) and
# HEAD against the build of 2bf1c20 (libfbr_hip_r05h.so).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05w
mkdir -p $OUT
for rep in 1 2; do
  for v in default r05h FBR_VG_SPLIT=8 FBR_VG_SPLIT=2 FBR_GN_FUSED=1 FBR_GN_LAG=3 FBR_FEAT_WAVES=2 FBR_KNN_LPQ=1; do
    E=""; L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so
    if [ $v = r05h ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_r05h.so; elif [ $v != default ]; then E="$v"; fi
    env $E FBR_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
    python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], 'mean', l['ms_per_scan_mean'])"
  done
done
