#!/bin/bash
# Round 5, call h: projection tests (rowcount change), features phase stamps in the batch mode
# (B = 64: one wave per ring), interleaved A/B of the rowcount change, latency line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_deskew.py tests/test_cpp_mirror.py -m gpu -x -v --timeout 300 --timeout-method thread -k "projection or deskew or mirror or batch_matches or stream" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 10; }
tail -2 $OUT/pytest.txt
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_diag.so timeout -k 10 300 python3 tools/feat_stamps.py 64 > $OUT/feat_stamps.txt 2>&1; cat $OUT/feat_stamps.txt
Q="--steps 10 --warmup 2 --latency 50 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_prev.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 300 python3 bench.py $Q > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('AB $v rep $rep', d['value'], 'extract', k['extract'], 'lat', d['latency']['ms_per_scan_p50'])"
done; done
