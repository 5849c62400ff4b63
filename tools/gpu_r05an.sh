#!/bin/bash
# Round 5, call an: the per-ring filter's bitonic run sort with f64 min / max exchanges (key_min /
# key_max; also removes the KQ = 8 kernel's spills: 64 VGPRs, no scratch) (new) vs prev = b8a59b2:
# ring-filter / VoxelGrid tests, interleaved C2 B = 1024 and C3 B = 256.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05an
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "ring or voxel or regist or batch" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'voxel_ring', k['voxel_ring'])"
done; done
for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], 'voxel_ring', k['voxel_ring'])"
done
