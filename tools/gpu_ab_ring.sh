#!/bin/bash
# A/B of the in-tree library (new) against libfbr_hip_prev.so (prev) on the per-ring filter: the
# VoxelGrid / ring / exact-order GPU tests, then interleaved C2 B = 1024 lines in the default and in
# the exact (--exact-voxel-order 1) order, and a 50-scan latency line each.
# usage: tools/gpu_ab_ring.sh TAG [reps]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; REPS=${2:-2}
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "voxel or ring or exact or order" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in $(seq 1 $REPS); do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 50 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/d_${v}_$rep.json 2>/dev/null || exit 17
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --exact-voxel-order 1 > $OUT/x_${v}_$rep.json 2>/dev/null || exit 18
  python3 -c "
import json
d=json.loads(open('$OUT/d_${v}_$rep.json').read().strip().splitlines()[-1]); x=json.loads(open('$OUT/x_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep default', d['value'], d['kernel_ms_per_step']['voxel_ring'], 'lat p50', d['latency']['ms_per_scan_p50'], '| exact', x['value'], x['kernel_ms_per_step']['voxel_ring'])"
done; done
