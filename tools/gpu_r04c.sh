#!/bin/bash
# pipelined batch launches: GPU suite subset + B = 128 / 1024 lines with and without FBR_PIPE
set -o pipefail
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_c4.py tests/test_distributed.py tests/test_gpu_parity.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 21; }
tail -3 $OUT/pytest.txt
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
B128="--batch 128 --steps 20 --warmup 5 --profile off"
B1024="--batch 1024 --steps 10 --warmup 3 --profile off"
run b128_pipe0 "FBR_PIPE=0" $B128
run b128_pipe1 "FBR_PIPE=1" $B128
run b128_pipe1_n2 "FBR_PIPE=1 FBR_NSUB=2" $B128
run b128_pipe1_q8 "FBR_PIPE=1 GPU_MAX_HW_QUEUES=8" $B128
run b1024_pipe0 "FBR_PIPE=0" $B1024
run b1024_pipe1 "FBR_PIPE=1" $B1024
run b1024_pipe1_n2 "FBR_PIPE=1 FBR_NSUB=2" $B1024
run b1024_pipe1_q8 "FBR_PIPE=1 GPU_MAX_HW_QUEUES=8" $B1024
run b128_pipe1_prof "FBR_PIPE=1" --batch 128 --steps 20 --warmup 5 --profile all
