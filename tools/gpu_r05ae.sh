#!/bin/bash
# Round 5, call ae: flag waits query the stream only after 2 ms (hipStreamQuery's marker cost
# ~5.7 us before every launch enqueued after a wait) -- GN / batch / stream tests, latency and
# B = 1024 throughput A/B against the previous build (libfbr_hip_prev.so = 4bf9326), interleaved,
# and the new single-scan timeline.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ae
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py tests/test_cpp_mirror.py tests/test_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('LAT $v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], 'mean', l['ms_per_scan_mean'])"
done; done
for rep in 1 2 3; do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('B1024 $v rep $rep', d['value'], 'gn_knn', k['gn_knn'], 'gn_solve', k['gn_solve'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/lat_trace -o lat --output-format csv -- python3 tools/latency_probe.py 40 > $OUT/lat_trace.log 2>&1 || { tail $OUT/lat_trace.log; exit 20; }
KT=$(find $OUT/lat_trace -name "*kernel_trace.csv" | head -1)
python3 tools/scan_timeline.py $KT 20 > $OUT/lat_timeline_20.txt; python3 tools/scan_timeline.py $KT 30 > $OUT/lat_timeline_30.txt
cat $OUT/lat_timeline_20.txt
