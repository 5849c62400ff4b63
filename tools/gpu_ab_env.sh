#!/bin/bash
# A/B of an environment setting inside one library: a pytest subset, then interleaved C2 B=1024
# lines (default vs ENV), then one SQ VALU pass of each (every kernel alone).
# usage: tools/gpu_ab_env.sh TAG "pytest -k expr" "ENV=VALUE ..." [reps]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; SEL=$2; ENVB=$3; REPS=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$SEL" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
  tail -1 $OUT/pytest.txt
fi
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
for r in $(seq 1 $REPS); do for v in a b; do
  E=""; [ $v = b ] && E="$ENVB"
  env $E timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v $r', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items() if b > 0.01})"
done; done
CMD="bench.py --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in a b; do
  E=""; [ $v = b ] && E="$ENVB"
  env $E timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_$v -o bench --output-format csv -- python3 $CMD > $OUT/sq_$v.log 2>&1 || { tail $OUT/sq_$v.log; exit 11; }
  python3 tools/valu_pmc.py $(find $OUT/sq_$v -name "*counter_collection.csv" | head -1) C2 1024 $OUT/valu_$v.json > $OUT/valu_$v.txt || exit 12
  echo "== $v $( [ $v = b ] && echo $ENVB )"; head -4 $OUT/valu_$v.txt
done
