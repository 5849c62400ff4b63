#!/bin/bash
# Throughput A/B of the in-tree library (new) against libfbr_hip_prev.so (prev), after a GPU test
# subset: interleaved C2 B = 1024 lines, then C3 B = 256 and C5 B = 16 once each.
# usage: tools/gpu_ab_tput.sh TAG "pytest -k expression" [reps] [kernel families to print, comma-separated]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; SEL=$2; REPS=${3:-3}; KF=${4:-gn_knn}
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in $(seq 1 $REPS); do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], {f: k[f] for f in '$KF'.split(',')})"
done; done
for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c5_${v}.json 2>/dev/null || exit 19
  python3 -c "
import json
for c in ('c3', 'c5'):
    d=json.loads(open('$OUT/'+c+'_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
    print(c.upper(), '$v', d['value'], {f: k[f] for f in '$KF'.split(',')})"
done
