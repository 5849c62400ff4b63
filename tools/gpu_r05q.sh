#!/bin/bash
# Round 5, call q: knob re-sweep at HEAD (C2 B = 1024, interleaved, 2 repeats).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
for rep in 1 2; do
  for v in default FBR_RES_MFMA=1 FBR_GN_GRID=16384 FBR_GN_TAIL=4 FBR_GN_TAIL=16 FBR_COMPACT_CELLS=512 FBR_GN_LAG=3; do
    if [ $v = default ]; then E=""; else E="$v"; fi
    env $E timeout -k 10 300 python3 bench.py $Q > $OUT/ab_${v}_$rep.json 2>/dev/null || exit 16
    python3 -c "
import json; d=json.loads(open('$OUT/ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v rep $rep', d['value'], 'gn_knn', k['gn_knn'], 'res', k['gn_residual'], 'extract', k['extract'])"
  done
done
