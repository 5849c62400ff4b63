#!/bin/bash
# Round 5, call al: the kNN point distance computed unconditionally and the crop-box test as a
# conditional overwrite (the compiler had sunk the distance under a branch on the test's result)
# (new) vs prev = 4f9a687: kNN parity subset, interleaved C2 B = 1024, C3, C5, latency.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05al
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 300 --timeout-method thread -k "regist or c3 or c5 or knn or tile or process_scan or crop" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'gn_knn', k['gn_knn'])"
done; done
for rep in 1 2; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}_$rep.json 2>/dev/null || exit 18
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c5_${v}_$rep.json 2>/dev/null || exit 19
  FBR_LIB=$(lib $v) timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json
for c in ('c3', 'c5'):
    d=json.loads(open('$OUT/'+c+'_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
    print(c.upper(), '$v rep $rep', d['value'], 'gn_knn', k['gn_knn'])
l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1]); print('LAT $v rep $rep', l['ms_per_scan_p50'], l['ms_per_scan_p99'])"
done; done
