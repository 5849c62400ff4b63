#!/bin/bash
# Round 5, call z: tie segments partition in LDS, stale-slot walks visit only candidates -- feature
# tests (ties, stream, golden), features stamps (B = 4), latency and throughput A/B against the
# previous build (libfbr_hip_prev.so).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05z
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_mirror.py tests/test_oracle_pinning.py -m gpu -x -v --timeout 600 --timeout-method thread -k "features or tie or stream or golden or process_scan or batch or sort" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_stamps.so timeout -k 10 300 python3 tools/feat_stamps.py 4 > $OUT/feat_stamps_b4.txt 2>&1 || { cat $OUT/feat_stamps_b4.txt; exit 3; }
tail -12 $OUT/feat_stamps_b4.txt
for rep in 1 2 3; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_prev.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('$v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'])"
done; done
for rep in 1 2; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_prev.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v rep $rep', d['value'], 'features', k['features'])"
done; done
