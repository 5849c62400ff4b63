#!/bin/bash
# batch-size / sub-batch sweep with three launch slots (throughput line only)
set -o pipefail
OUT=gpurun_out/r04aa
mkdir -p $OUT
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run b1024 "FBR_X=0" --batch 1024 --steps 10 --warmup 3
run b1536 "FBR_X=0" --batch 1536 --steps 8 --warmup 3
run b2048 "FBR_X=0" --batch 2048 --steps 6 --warmup 3
run b1024_nsub2 "FBR_NSUB=2" --batch 1024 --steps 10 --warmup 3
run b768 "FBR_X=0" --batch 768 --steps 12 --warmup 3
run b1024b "FBR_X=0" --batch 1024 --steps 10 --warmup 3
