#!/bin/bash
# Round 5, call aj: kNN insertion as a v_min_f64 / v_max_f64 bubble over the keys read as doubles
# (new) against the 64-bit compare + select form (prev = 2c629ff) -- full GPU suite (incl. the new
# direct-results equivalence test), kNN stats-free SQ pass of both, interleaved B = 1024, C3, C5.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05aj
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -1 $OUT/pytest_gpu.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'gn_knn', k['gn_knn'], 'gn_residual', k['gn_residual'])"
done; done
for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c5_${v}.json 2>/dev/null || exit 19
  python3 -c "
import json
for c in ('c3', 'c5'):
    d=json.loads(open('$OUT/'+c+'_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
    print(c.upper(), '$v', d['value'], 'gn_knn', k['gn_knn'])"
done
CMD="bench.py --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in new prev; do
  FBR_LIB=$(lib $v) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_$v -o bench --output-format csv -- python3 $CMD > $OUT/sq_$v.log 2>&1 || { tail $OUT/sq_$v.log; exit 20; }
  python3 tools/pmc_by_kernel.py $(find $OUT/sq_$v -name "*counter_collection.csv" | head -1) k_gn_knn > $OUT/sq_$v.txt 2>&1 || true
  echo "== SQ $v"; cat $OUT/sq_$v.txt
done
