#!/bin/bash
# iteration-0 flat queue seeded by the query's own row (FBR_KNN_FLAT0=1): the GPU suite with it on,
# interleaved A/B against the default, sequential kernel stats of both
set -o pipefail
OUT=gpurun_out/r04aj
mkdir -p $OUT
FBR_KNN_FLAT0=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -2 $OUT/pytest.log
run() {  # name, env
  local name=$1 e=$2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run f0_a "FBR_KNN_FLAT0=1"
run def_a "FBR_KNN_FLAT0=0"
run f0_b "FBR_KNN_FLAT0=1"
run def_b "FBR_KNN_FLAT0=0"
run f0_c "FBR_KNN_FLAT0=1"
run def_c "FBR_KNN_FLAT0=0"
export TMPDIR=/tmp
for v in 1 0; do
  FBR_KNN_FLAT0=$v FBR_NSUB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 4 --warmup 1 > $OUT/p_$v.log 2>&1 || exit 23
done
