#!/bin/bash
# fit list (k_gn_fit): GPU suite, interleaved A/B against FBR_FIT_LIST=0, kernel stats of both
set -o pipefail
OUT=gpurun_out/r04ac
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -3 $OUT/pytest.log
run() {  # name, env
  local name=$1 e=$2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run fl1a "FBR_FIT_LIST=1"
run fl0a "FBR_FIT_LIST=0"
run fl1b "FBR_FIT_LIST=1"
run fl0b "FBR_FIT_LIST=0"
run fl1c "FBR_FIT_LIST=1"
run fl0c "FBR_FIT_LIST=0"
export TMPDIR=/tmp
FBR_FIT_LIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 5 --warmup 2 > $OUT/p1.log 2>&1 || exit 23
FBR_FIT_LIST=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof0 -o run -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 5 --warmup 2 > $OUT/p0.log 2>&1 || exit 24
for d in prof1 prof0; do f=$(find $OUT/$d -name '*kernel_stats.csv' | head -1); echo "== $d"; grep -E 'k_gn_(knn|fit|residual|solve)' "$f" | cut -c1-160; done
