#!/bin/bash
# knob sweep at HEAD (three launch slots, B = 1024): each knob against interleaved defaults
set -o pipefail
OUT=gpurun_out/r04ab
mkdir -p $OUT
run() {  # name, env
  local name=$1 e=$2
  env $e timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run def1 "FBR_X=0"
run cc512 "FBR_COMPACT_CELLS=512"
run cc2048 "FBR_COMPACT_CELLS=2048"
run def2 "FBR_X=0"
run vr0 "FBR_VR_WAVE=0"
run grid4k "FBR_GN_GRID=4096"
run tail4 "FBR_GN_TAIL=4"
run def3 "FBR_X=0"
run tail16 "FBR_GN_TAIL=16"
run grid16k "FBR_GN_GRID=16384"
run def4 "FBR_X=0"
