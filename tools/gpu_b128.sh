#!/bin/bash
# Sub-batch count / GN knobs at B = 128 (the C4 per-GPU share).  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
B="timeout -k 10 300 python3 bench.py --batch 128 --steps 20 --warmup 5 --latency 0 --ingest 0 --no-cpu-baseline --profile off"
for v in "FBR_NSUB=3" "FBR_NSUB=2" "FBR_NSUB=4" "FBR_NSUB=3 FBR_GN_TAIL=4" "FBR_NSUB=3 FBR_GN_TAIL=0" "FBR_NSUB=4 FBR_GN_TAIL=4" "FBR_NSUB=3"; do
  env $v $B > $OUT/b128_$(echo $v | tr ' =' '__').json 2>>$OUT/err || exit 21
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/b128_$(echo $v | tr ' =' '__').json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
done
