#!/bin/bash
# Round 5, call g: batch conflict masks only for the corner candidates + surf window (k_features):
# equivalence + feature / registration tests, interleaved A/B against the previous build.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py tests/test_keyframes.py tests/test_deskew.py -m gpu -x -v --timeout 600 --timeout-method thread -k "surf_walk_window or registration or batch or c3 or c5 or c4_full or golden or stream or features or ring_filter or deskew or keyframe" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 10; }
tail -2 $OUT/pytest.txt
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2 3; do for v in new prev; do
  if [ $v = prev ]; then L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_prev.so; else L=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip.so; fi
  FBR_LIB=$L timeout -k 10 300 python3 bench.py $Q > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('AB $v rep $rep', d['value'], 'features', k['features'])"
done; done
