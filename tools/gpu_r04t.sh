#!/bin/bash
# latency line (copy-worker spin 5 ms, cached worker device) and the default bench line
set -o pipefail
OUT=gpurun_out/r04t
mkdir -p $OUT
timeout -k 10 600 python3 bench.py --steps 10 --warmup 3 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/bench_lat.json 2> $OUT/err || exit 21
python3 -c "
import json; d=json.loads(open('$OUT/bench_lat.json').read().strip().splitlines()[-1]); l=d['latency']
print(d['value'], l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['ms_per_scan_mean'], l['host_ms_per_scan'])"
