#!/bin/bash
# Round 5, call ad: single-scan direct results (the ending k_gn_solve packs the result into
# host-mapped memory; no finalize / pack launch, copy or stream sync) -- GPU suite, latency A/B
# against FBR_DIRECT=0 (interleaved), the single-scan timeline, one default bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ad
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -1 $OUT/pytest_gpu.txt
for rep in 1 2 3; do for v in 1 0; do
  FBR_DIRECT=$v timeout -k 10 120 python3 tools/latency_probe.py 100 > $OUT/lat_d${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; l=json.loads(open('$OUT/lat_d${v}_$rep.json').read().strip().splitlines()[-1])
print('direct=$v rep $rep p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], 'mean', l['ms_per_scan_mean'], l['host_ms_per_scan'])"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/lat_trace -o lat --output-format csv -- python3 tools/latency_probe.py 40 > $OUT/lat_trace.log 2>&1 || { tail $OUT/lat_trace.log; exit 20; }
KT=$(find $OUT/lat_trace -name "*kernel_trace.csv" | head -1)
python3 tools/scan_timeline.py $KT 20 > $OUT/lat_timeline_20.txt; python3 tools/scan_timeline.py $KT 30 > $OUT/lat_timeline_30.txt
cat $OUT/lat_timeline_20.txt
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 23
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], 'latency', d['latency']['ms_per_scan_p50'], d['latency']['ms_per_scan_p99'], 'chain', d['latency'].get('chain_max_abs_pose_diff_vs_oracle'))"
