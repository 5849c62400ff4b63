#!/bin/bash
# Round 5, call ao: the features' sorted-path bitonic sort with f64 min / max exchanges (new) vs
# prev = 15b6a11: feature tests (ties, stale slot, golden, stream, batch), interleaved C2 B = 1024,
# C3 B = 256 and single-scan latency (ring 0's stale-slot segment takes the sorted path).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ao
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_mirror.py tests/test_oracle_pinning.py tests/test_deskew.py -m gpu -x -v --timeout 600 --timeout-method thread -k "feature or tie or stream or golden or process_scan or batch or sort or deskew or c3" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  FBR_LIB=$(lib $v) timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('B1024 $v rep $rep', d['value'], 'features', k['features'], 'LAT', l['ms_per_scan_p50'], l['ms_per_scan_p99'])"
done; done
for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_${v}.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], 'features', k['features'])"
done
