#!/bin/bash
# Round 5, call ak: kNN insertion as independent v_min_f64(k[t], v_max_f64(k[t-1], x)) per slot
# (depth 2; new) and the same with the 0.5 m-cell kernels (R = 2: C3, C5) keeping the select form
# (r2sel), against prev = 2c629ff (selects everywhere): GPU suite on new, kNN parity subset on
# r2sel, interleaved C2 B = 1024, C3 B = 256, C5 B = 16.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ak
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { case $1 in prev) echo $PKG/libfbr_hip_prev.so;; new) echo $PKG/libfbr_hip.so;; *) echo $PKG/libfbr_hip_$1.so;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -1 $OUT/pytest_gpu.txt
FBR_LIB=$(lib r2sel) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "regist or c3 or c5 or knn or tile" > $OUT/pytest_r2sel.txt 2>&1 || { tail -40 $OUT/pytest_r2sel.txt; exit 11; }
echo "r2sel: $(tail -1 $OUT/pytest_r2sel.txt)"
for rep in 1 2 3; do for v in new prev r2sel; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'gn_knn', k['gn_knn'])"
done; done
for rep in 1 2; do for v in new prev r2sel; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}_$rep.json 2>/dev/null || exit 18
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c5_${v}_$rep.json 2>/dev/null || exit 19
  python3 -c "
import json
for c in ('c3', 'c5'):
    d=json.loads(open('$OUT/'+c+'_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
    print(c.upper(), '$v rep $rep', d['value'], 'gn_knn', k['gn_knn'])"
done; done
