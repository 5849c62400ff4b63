#!/bin/bash
# pipelined launches + wave-per-ring surf filter: parity subset, then B = 128 / 1024 lines
set -o pipefail
OUT=gpurun_out/r04d
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
run b128_pipe0_vr0 "FBR_PIPE=0 FBR_VR_WAVE=0" $B128
run b128_pipe1_vr0 "FBR_PIPE=1 FBR_VR_WAVE=0" $B128
run b128_pipe1 "FBR_PIPE=1" $B128
run b128_pipe1_n2 "FBR_PIPE=1 FBR_NSUB=2" $B128
run b128_pipe1_q8 "FBR_PIPE=1 GPU_MAX_HW_QUEUES=8" $B128
run b1024_pipe0_vr0 "FBR_PIPE=0 FBR_VR_WAVE=0" $B1024
run b1024_pipe0 "FBR_PIPE=0" $B1024
run b1024_pipe1 "FBR_PIPE=1" $B1024
run b1024_pipe1_n2 "FBR_PIPE=1 FBR_NSUB=2" $B1024
run b1024_pipe1_q8 "FBR_PIPE=1 GPU_MAX_HW_QUEUES=8" $B1024
run seq_b256_vr0 "FBR_NSUB=1 FBR_PIPE=0 FBR_VR_WAVE=0" --batch 256 --steps 5 --warmup 2 --profile all
run seq_b256_vr1 "FBR_NSUB=1 FBR_PIPE=0" --batch 256 --steps 5 --warmup 2 --profile all
run b1024_prof "" --batch 1024 --steps 10 --warmup 3 --profile all
python3 - $OUT <<'PY' | tee -a $OUT/summary.txt
import json, sys
out = sys.argv[1]
for f in ("seq_b256_vr0", "seq_b256_vr1", "b1024_prof"):
    d = json.loads(open(f"{out}/{f}.json").read().strip().splitlines()[-1])
    ks = d["roofline"]["kernels"]
    print(f, d["value"], " ".join(f"{k}={v['avg_launch_us']:.0f}us/{v['ms_per_step']:.2f}ms" for k, v in ks.items()))
PY
