#!/bin/bash
# Round 5, call ah: row counts from k_project's first claims (k_rowsum reads ~57 per-chunk counts
# per row instead of k_rowcount's pass over the 1800-cell owner row) -- full GPU suite, then
# interleaved B = 1024 lines and single-scan latency against the previous build (prev = 62b421d).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ah
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -1 $OUT/pytest_gpu.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'project', k['project'], 'extract', k['extract'])"
done; done
for rep in 1 2; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('LAT $v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'])"
done; done
