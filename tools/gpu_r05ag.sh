#!/bin/bash
# Round 5, call ag: occupancy of the residual (124 VGPRs, 4 waves per SIMD) and of the batch
# feature kernel (128, 4): res5 / res6 = k_gn_residual held to 5 / 6 waves (96 / 80 VGPRs, 72 /
# 128 B spills), feat5 / feat6 = k_features<.., 1> at 5 / 6 (112 / 192 B spills); prev = the
# default build (c74a1a5).  Parity tests per variant, then interleaved B = 1024 lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ag
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { case $1 in prev) echo $PKG/libfbr_hip_prev.so;; *) echo $PKG/libfbr_hip_$1.so;; esac; }
for v in res5 res6; do
  FBR_LIB=$(lib $v) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "regist or batch or c3 or c5" > $OUT/pytest_$v.txt 2>&1 || { tail -40 $OUT/pytest_$v.txt; exit 10; }
  echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
for v in feat5 feat6; do
  FBR_LIB=$(lib $v) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "feature or tie or golden or batch or stream" > $OUT/pytest_$v.txt 2>&1 || { tail -40 $OUT/pytest_$v.txt; exit 11; }
  echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
for rep in 1 2 3; do for v in prev res5 res6 feat5 feat6; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'gn_residual', k['gn_residual'], 'features', k['features'])"
done; done
