#!/bin/bash
# A/B of the 16-B batch scan records (default) against the 24-B scans (FBR_PACKED_SCANS=0): the
# packed-record parity tests, then interleaved C2 B = 1024 lines with the ingest line, C3 B = 256.
# usage: tools/gpu_ab_packed.sh TAG [reps]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; REPS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "packed or batch_matches or feature_masks or deskew" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
B="bench.py --steps 10 --warmup 2 --latency 0 --exact-line 0 --no-cpu-baseline"
for r in $(seq 1 $REPS); do for v in a b; do
  P=1; [ $v = b ] && P=0
  FBR_PACKED_SCANS=$P timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('packed=$P rep $r', d['value'], d['ms_per_step'], 'ingest', d.get('ingest', {}).get('value'), {a: round(b,3) for a,b in k.items() if b > 0.01})"
done; done
for P in 1 0; do
  FBR_PACKED_SCANS=$P timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/c3_$P.json 2>/dev/null || exit 18
  python3 -c "
import json; d=json.loads(open('$OUT/c3_$P.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('C3 packed=$P', d['value'], {a: round(b,3) for a,b in k.items() if a in ('project','extract')})"
done
