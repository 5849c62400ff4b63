#!/bin/bash
# Round 5, call r: stream-mode surf window (single scans) + batch label buffer without clearing + GN
# grid 16384 -- feature / stream / batch tests, then latency and throughput A/B against the whole
# walk (FBR_FEAT_SURF_WINDOW=0; it also turns the batch window off).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05r
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py tests/test_cpp_mirror.py -m gpu -x -v --timeout 600 --timeout-method thread -k "surf_walk or stream or features or batch or golden or c4 or mirror or process_scan" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -2 $OUT/pytest.txt
Q="--steps 10 --warmup 2 --latency 100 --ingest 0 --exact-line 0 --no-cpu-baseline"
for rep in 1 2; do for v in 1 0; do
  FBR_FEAT_SURF_WINDOW=$v timeout -k 10 300 python3 bench.py $Q > $OUT/ab_w${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_w${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; l=d['latency']
print('window=$v rep $rep', d['value'], 'features', k['features'], 'gn_knn', k['gn_knn'], 'lat p50', l['ms_per_scan_p50'], 'p99', l['ms_per_scan_p99'], 'chain', l['chain_max_abs_pose_diff_vs_oracle'])"
done; done
