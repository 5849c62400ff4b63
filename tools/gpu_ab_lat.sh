#!/bin/bash
# Single-scan latency of the in-tree library (new) against libfbr_hip_prev.so (prev), interleaved.
# usage: tools/gpu_ab_lat.sh TAG [reps]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; REPS=${2:-2}; mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
for rep in $(seq 1 $REPS); do for v in new prev; do
  L=$PKG/libfbr_hip.so; [ $v = prev ] && L=$PKG/libfbr_hip_prev.so
  FBR_LIB=$L timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --latency 50 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1]); l=d['latency']
print('latency $v rep $rep', l.get('ms_per_scan_p50'), l.get('ms_per_scan_p99'), l.get('ms_per_scan_max'))"
done; done
