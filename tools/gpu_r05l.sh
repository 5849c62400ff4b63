#!/bin/bash
# Round 5, call l: the balanced flat kNN walk -- GPU suite (default: balanced), then an interleaved
# A/B against the per-lane flat walk (FBR_KNN_BAL=0) on C2 B = 1024 and C3 B = 256.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05l
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -2 $OUT/pytest.txt
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
for rep in 1 2; do for v in 1 0; do
  FBR_KNN_BAL=$v timeout -k 10 300 python3 bench.py $Q > $OUT/ab_bal${v}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_bal${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('AB bal=$v rep $rep', d['value'], 'gn_knn', k['gn_knn'], 'res', k['gn_residual'])"
done; done
for v in 1 0; do
  FBR_KNN_BAL=$v timeout -k 10 300 python3 bench.py --config C3 --batch 256 $Q > $OUT/c3_bal${v}.json 2>/dev/null || exit 17
  python3 -c "
import json; d=json.loads(open('$OUT/c3_bal${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 bal=$v', d['value'], 'gn_knn', k['gn_knn'])"
done
