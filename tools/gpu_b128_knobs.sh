#!/bin/bash
# Feature-wave and kNN-lane knobs at B = 128, then the B = 1024 rate with the same flags.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
B="timeout -k 10 300 python3 bench.py --batch 128 --steps 20 --warmup 5 --latency 0 --ingest 0 --no-cpu-baseline --profile off"
for v in "FBR_NSUB=3" "FBR_FEAT_WAVES=2" "FBR_FEAT_WAVES=4" "FBR_KNN_LPQ=8" "FBR_FEAT_WAVES=2 FBR_GN_TAIL=4" "FBR_NSUB=3"; do
  env $v $B > $OUT/b128_$(echo $v | tr ' =' '__').json 2>>$OUT/err || exit 21
  echo "$v $(python3 -c "import json,sys; d=json.loads(open('$OUT/b128_$(echo $v | tr ' =' '__').json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
done
timeout -k 10 300 python3 bench.py --batch 1024 --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline --profile off > $OUT/b1024.json 2>>$OUT/err || exit 22
echo "B1024 $(python3 -c "import json; d=json.loads(open('$OUT/b1024.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
