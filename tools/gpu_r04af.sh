#!/bin/bash
# counted flat walk at HEAD: GPU suite, then iteration-0 flat queue (FBR_KNN_FLAT0=1) and the
# 0.5 m flat queue on C3 (FBR_KNN_FLAT_R2=1) against defaults, interleaved
set -o pipefail
OUT=gpurun_out/r04af
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -2 $OUT/pytest.log
run() {  # name, env, extra args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e $*] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run def_a "FBR_X=0"
run f0_a "FBR_KNN_FLAT0=1"
run def_b "FBR_X=0"
run f0_b "FBR_KNN_FLAT0=1"
run c3_def "FBR_X=0" --config C3 --batch 256
run c3_r2 "FBR_KNN_FLAT_R2=1" --config C3 --batch 256
run c3_def2 "FBR_X=0" --config C3 --batch 256
run c3_r2b "FBR_KNN_FLAT_R2=1" --config C3 --batch 256
