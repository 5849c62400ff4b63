#!/bin/bash
# A/B of an environment setting inside one library: a pytest subset, then interleaved C2 B = 1024
# lines (default vs ENV, latency line included), then C3 B = 256 once each.
# usage: tools/gpu_ab_env_light.sh TAG "pytest -k expr" "ENV=VALUE ..." [reps]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; SEL=$2; ENVB=$3; REPS=${4:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
  tail -1 $OUT/pytest.txt
fi
B="bench.py --steps 10 --warmup 2 --latency 20 --ingest 0 --exact-line 0 --no-cpu-baseline"
for r in $(seq 1 $REPS); do for v in a b; do
  E="FBR_AB=a"; [ $v = b ] && E="$ENVB"
  env $E timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; l=d.get('latency') or {}
print('$v $r', d['value'], d['ms_per_step'], 'lat', l.get('ms_per_scan_p50'), {a: round(b,3) for a,b in k.items() if b > 0.01})"
done; done
for v in a b; do
  E="FBR_AB=a"; [ $v = b ] && E="$ENVB"
  env $E timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_$v.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_$v.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 $v', d['value'], {a: round(b,3) for a,b in k.items() if a in ('project','extract')})"
done
