#!/bin/bash
# Latency A/B of the in-tree library (new) against libfbr_hip_prev.so (prev), with a GPU test
# subset first.  usage: tools/gpu_ab_latency.sh TAG "pytest -k expression" [reps]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; SEL=$2; REPS=${3:-3}
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
lib() { if [ $1 = prev ]; then echo $PKG/libfbr_hip_prev.so; else echo $PKG/libfbr_hip.so; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
for rep in $(seq 1 $REPS); do for v in new prev; do
  FBR_LIB=$(lib $v) timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])
print('LAT $v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/lat_trace -o lat --output-format csv -- python3 tools/latency_probe.py 40 > $OUT/lat_trace.log 2>&1 || { tail $OUT/lat_trace.log; exit 20; }
python3 tools/scan_timeline.py $(find $OUT/lat_trace -name "*kernel_trace.csv" | head -1) 20 > $OUT/lat_timeline_20.txt && cat $OUT/lat_timeline_20.txt
