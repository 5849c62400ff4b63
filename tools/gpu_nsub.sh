#!/bin/bash
# sub-batch count x batch size with pipelined launches.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
for B in 128 256 512 1024; do
  for N in 1 2 3; do
    st=$((20 * 128 / B + 5)); [ $st -lt 10 ] && st=10
    run b${B}_n${N} "FBR_NSUB=$N FBR_VR_WAVE=0" --batch $B --steps $st --warmup 3
  done
done
run b1024_n1_vr1 "FBR_NSUB=1 FBR_VR_WAVE=1" --batch 1024 --steps 10 --warmup 3
run b128_n1_vr1 "FBR_NSUB=1 FBR_VR_WAVE=1" --batch 128 --steps 25 --warmup 3
run b2048_n1 "FBR_NSUB=1 FBR_VR_WAVE=0" --batch 2048 --steps 10 --warmup 3
run b2048_n2 "FBR_NSUB=2 FBR_VR_WAVE=0" --batch 2048 --steps 10 --warmup 3
