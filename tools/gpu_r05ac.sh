#!/bin/bash
# Round 5, call ac: flat kNN queue with the rows' cell_start loads issued together (rows2: all 9; rows2nb3: 3 at a time; exact x extent kept)
# the flat queue's cell_start loads issued together (rows2: all 9 rows; rows2nb3: 3 at a time) --
# registration tests (C2 / C3 / C4 / C5 parity) on new and rows2nb3, the interleaved B = 1024 line
# against the previous build (prev), C3 B = 256 once each, and an SQ pass of each for gn_knn.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ac
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { case $1 in prev) echo $PKG/libfbr_hip_prev.so;; new) echo $PKG/libfbr_hip.so;; *) echo $PKG/libfbr_hip_$1.so;; esac; }
SEL="regist or c3 or c5 or c4 or knn or tile or process_scan"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 600 --timeout-method thread -k "$SEL" > $OUT/pytest_new.txt 2>&1 || { tail -40 $OUT/pytest_new.txt; exit 10; }
tail -1 $OUT/pytest_new.txt
FBR_LIB=$(lib rows2) timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 600 --timeout-method thread -k "$SEL" > $OUT/pytest_rows2.txt 2>&1 || { tail -40 $OUT/pytest_rows2.txt; exit 11; }
tail -1 $OUT/pytest_rows2.txt
for rep in 1 2 3; do for v in new prev rows2 rows2nb3; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v rep $rep', d['value'], 'gn_knn', k['gn_knn'], 'gn_residual', k['gn_residual'])"
done; done
for v in new prev rows2nb3; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], 'gn_knn', k['gn_knn'])"
done
CMD="bench.py --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in new prev rows2 rows2nb3; do
  FBR_LIB=$(lib $v) timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_$v -o bench --output-format csv -- python3 $CMD > $OUT/sq_$v.log 2>&1 || { tail $OUT/sq_$v.log; exit 19; }
  python3 tools/pmc_by_kernel.py $(find $OUT/sq_$v -name "*counter_collection.csv" | head -1) k_gn_knn > $OUT/sq_$v.txt 2>&1 || true
  echo "== SQ $v"; cat $OUT/sq_$v.txt
done
# single-scan timeline at HEAD (kernels + copies of one pose-chained C2 scan)
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/lat_trace -o lat --output-format csv -- python3 tools/latency_probe.py 40 > $OUT/lat_trace.log 2>&1 || { tail $OUT/lat_trace.log; exit 20; }
tail -1 $OUT/lat_trace.log
KT=$(find $OUT/lat_trace -name "*kernel_trace.csv" | head -1)
python3 tools/scan_timeline.py $KT 20 > $OUT/lat_timeline_20.txt; python3 tools/scan_timeline.py $KT 30 > $OUT/lat_timeline_30.txt
cat $OUT/lat_timeline_20.txt
