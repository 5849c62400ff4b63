#!/bin/bash
# Ingest A/B: batch/ingest GPU tests, then interleaved ingest lines (fbr_process_batch from host
# memory, 3 x 1024 C2 jobs) for each environment variant.
# usage: tools/gpu_ingest_ab.sh TAG REPS "ENV=V ..." "ENV=V ..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "batch or ingest or process" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
B="bench.py --steps 3 --warmup 1 --latency 0 --ingest 3 --exact-line 0 --no-cpu-baseline --profile off"
for r in $(seq 1 $REPS); do v=0; for E in "$@"; do
  v=$((v + 1)); N=v${v}_$r
  env $E timeout -k 10 300 python3 $B > $OUT/$N.json 2> $OUT/$N.err || { tail $OUT/$N.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/$N.json').read().strip().splitlines()[-1]); i=d['ingest']
print('$N [$E]', i['value'], i['h2d_GBps'], i['poses_equal_resident'], 'batch', d['value'])"
done; done
