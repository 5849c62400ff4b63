#!/bin/bash
# Three-way A/B of environment settings inside one library: a pytest subset, then interleaved C2
# B = 1024 lines (default, ENV_B, ENV_C), then C3 B = 256 once each.
# usage: tools/gpu_ab_env3.sh TAG "pytest -k expr" "ENV_B=..." "ENV_C=..." [reps]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; SEL=$2; ENVB=$3; ENVC=$4; REPS=${5:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
  tail -1 $OUT/pytest.txt
fi
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
envof() { case $1 in a) echo "FBR_AB=a";; b) echo "$ENVB";; c) echo "$ENVC";; esac; }
for r in $(seq 1 $REPS); do for v in a b c; do
  env $(envof $v) timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v $r', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items() if a.startswith('gn')})"
done; done
for v in a b c; do
  env $(envof $v) timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_$v.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], {a: round(b,3) for a,b in k.items() if a.startswith('gn')})"
done
