#!/bin/bash
# Interleaved C2 B = 1024 lines of the default against environment variants (knob defaults re-checked
# at HEAD; BENCH_ARGS adds bench.py flags, e.g. "--config C3 --batch 256").
# usage: tools/gpu_knob_sweep.sh TAG REPS "ENV=V ..." ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; REPS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline ${BENCH_ARGS}"
for r in $(seq 1 $REPS); do v=0; for E in "" "$@"; do
  N=v${v}_$r; v=$((v + 1))
  env $E timeout -k 10 300 python3 $B > $OUT/$N.json 2> $OUT/$N.err || { tail $OUT/$N.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/$N.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$N [${E:-default}]', d['value'], {a: round(b,3) for a,b in k.items() if b > 0.3})"
done; done
