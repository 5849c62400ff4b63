#!/bin/bash
# Round 5, call ap: projection loop unrolled 4 / 8 (pu4 / pu8: more point loads in flight, 50
# VGPRs) and the iteration-0 per-row kNN kernel held to 7 / 8 waves per SIMD (kw7 / kw8: 72 / 64
# VGPRs, 44 / 76 B of spills) vs prev = bad372a: parity subsets, interleaved C2 B = 1024.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ap
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { case $1 in prev) echo $PKG/libfbr_hip_prev.so;; *) echo $PKG/libfbr_hip_$1.so;; esac; }
for v in pu8 kw8; do
  FBR_LIB=$(lib $v) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "projection or regist or batch" > $OUT/pytest_$v.txt 2>&1 || { tail -40 $OUT/pytest_$v.txt; exit 10; }
  echo "$v: $(tail -1 $OUT/pytest_$v.txt)"
done
for rep in 1 2 3; do for v in prev pu4 pu8 kw7 kw8; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'project', k['project'], 'gn_knn', k['gn_knn'])"
done; done
