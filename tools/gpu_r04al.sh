#!/bin/bash
# knob sweep at the counted walk: GN enqueue lag against interleaved defaults
set -o pipefail
OUT=gpurun_out/r04al
mkdir -p $OUT
run() {  # name, env
  local name=$1 e=$2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run def1 "FBR_X=0"
run lag1 "FBR_GN_LAG=1"
run lag3 "FBR_GN_LAG=3"
run def2 "FBR_X=0"
run lag4 "FBR_GN_LAG=4"
run lag1b "FBR_GN_LAG=1"
run def3 "FBR_X=0"
