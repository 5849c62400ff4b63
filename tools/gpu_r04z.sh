#!/bin/bash
# single-scan upload with 8 host copy participants and 256 KB chunks: latency lines
set -o pipefail
OUT=gpurun_out/r04z
mkdir -p $OUT
for k in 1 2 3; do
  timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat.json 2>> $OUT/lat.err || exit 22
  echo "lat $(python3 -c "import json; l=json.loads(open('$OUT/lat.json').read().strip().splitlines()[-1]); print(l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['host_ms_per_scan'])")" | tee -a $OUT/lat_summary.txt
done
