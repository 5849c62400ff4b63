#!/bin/bash
# single-scan latency under GN knobs (fused kNN + residual, matrix-core partials, kNN lanes per query)
set -o pipefail
OUT=gpurun_out/r04w
mkdir -p $OUT
for e in "FBR_X=0" "FBR_GN_FUSED=1" "FBR_RES_MFMA=1" "FBR_GN_FUSED=1 FBR_RES_MFMA=1" "FBR_KNN_LPQ=1" "FBR_X=0"; do
  env $e timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat.json 2>> $OUT/lat.err || exit 22
  echo "lat [$e] $(python3 -c "import json; l=json.loads(open('$OUT/lat.json').read().strip().splitlines()[-1]); print(l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['launches_per_scan'], l['host_ms_per_scan'])")" | tee -a $OUT/lat_summary.txt
done
