#!/bin/bash
# Hardware-queue / sub-batch-stream sweep (GPU_MAX_HW_QUEUES x FBR_NSUB) at B = 128 and B = 1024,
# plus the C3 / C5 lines.  usage: tools/gpu_hwq.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 "$@" > $OUT/$name.json 2>>$OUT/err || exit 21
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
B128="--batch 128 --steps 20 --warmup 5 --profile off"
B1024="--batch 1024 --steps 10 --warmup 3 --profile off"
run b128_q4_n3 "GPU_MAX_HW_QUEUES=4 FBR_NSUB=3" $B128
run b128_q8_n3 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=3" $B128
run b128_q8_n4 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=4" $B128
run b128_q8_n6 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=6" $B128
run b128_q8_n8 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=8" $B128
run b1024_q4_n3 "GPU_MAX_HW_QUEUES=4 FBR_NSUB=3" $B1024
run b1024_q8_n4 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=4" $B1024
run b1024_q8_n6 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=6" $B1024
run b1024_q8_n8 "GPU_MAX_HW_QUEUES=8 FBR_NSUB=8" $B1024
run c3_b256 "FBR_NSUB=3" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c5_b16 "FBR_NSUB=3" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
