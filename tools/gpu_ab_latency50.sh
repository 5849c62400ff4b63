#!/bin/bash
# Latency A/B at the driver's chain length (50 pose-chained C2 scans): the in-tree library (new)
# against libfbr_hip_prev.so (prev, the round-5 library), interleaved.  usage: tools/gpu_ab_latency50.sh TAG [reps]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; REPS=${2:-3}
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
for rep in $(seq 1 $REPS); do for v in new prev; do
  L=$PKG/libfbr_hip.so; [ $v = prev ] && L=$PKG/libfbr_hip_prev.so
  FBR_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 50 > $OUT/lat_${v}_$rep.json 2>$OUT/lat_${v}_$rep.err || { tail $OUT/lat_${v}_$rep.err; exit 16; }
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('LAT $v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], 'max', l.get('ms_per_scan_max'), l.get('result_waits'), l.get('slowest'))"
done; done
