#!/bin/bash
# single-scan ring filter (512-thread kernel for small launches), adaptive copy spin: ring-filter and
# split-VoxelGrid parity tests, latency lines, the default batch line
set -o pipefail
OUT=gpurun_out/r04v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave_ring_filter or split_voxel or features or process_scan or stream" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
for e in "FBR_GN_LAG=0" "FBR_GN_LAG=2" "FBR_GN_LAG=0" "FBR_GN_LAG=2"; do
  env $e timeout -k 10 300 python3 tools/latency_probe.py 50 C2 > $OUT/lat.json 2>> $OUT/lat.err || exit 22
  echo "lat $e $(python3 -c "import json; l=json.loads(open('$OUT/lat.json').read().strip().splitlines()[-1]); print(l['ms_per_scan_p50'], l['ms_per_scan_p99'], l['launches_per_scan'], l['host_ms_per_scan'])")" | tee -a $OUT/lat_summary.txt
done
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/bench.json 2> $OUT/bench.err || exit 23
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
