#!/bin/bash
# Round 5, call af: per-ring surf filter occupancy -- pass A keeps only x, y, z in registers (80 ->
# 72 VGPRs, 7 workgroups per CU; new) and the same forced to 64 VGPRs (vrq8, 44 B of spills),
# against the previous build (prev = 9392d15): ring-filter / VoxelGrid / registration tests, then
# interleaved B = 1024 lines and C3 B = 256.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05af
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { case $1 in prev) echo $PKG/libfbr_hip_prev.so;; new) echo $PKG/libfbr_hip.so;; *) echo $PKG/libfbr_hip_$1.so;; esac; }
SEL="ring or voxel or regist or batch or c3"
for v in new vrq8; do
  FBR_LIB=$(lib $v) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest_$v.txt 2>&1 || { tail -40 $OUT/pytest_$v.txt; exit 10; }
  echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
for rep in 1 2 3; do for v in new prev vrq8; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'voxel_ring', k['voxel_ring'], 'features', k['features'])"
done; done
for v in new prev vrq8; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], 'voxel_ring', k['voxel_ring'])"
done
