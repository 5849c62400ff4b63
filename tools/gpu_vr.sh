#!/bin/bash
# wave-per-ring surf filter A/B: parity (wave vs workgroup kernel, features vs oracle), then the
# sequential per-kernel line and the overlapped B = 1024 line for FBR_VR_WAVE = 0 / 1.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "wave_ring or features" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  python3 - $OUT/$name.json "$name [$e]" <<'PY' | tee -a $OUT/summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d["roofline"]["kernels"]
print(sys.argv[2], d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_launch_us']:.0f}us/{v['ms_per_step']:.2f}ms" for k, v in ks.items()))
PY
}
run seq_vr0 "FBR_NSUB=1 FBR_PIPE=0 FBR_VR_WAVE=0" --batch 256 --steps 5 --warmup 2 --profile all
run seq_vr1 "FBR_NSUB=1 FBR_PIPE=0 FBR_VR_WAVE=1" --batch 256 --steps 5 --warmup 2 --profile all
run b1024_vr0 "FBR_VR_WAVE=0" --batch 1024 --steps 10 --warmup 3 --profile all
run b1024_vr1 "FBR_VR_WAVE=1" --batch 1024 --steps 10 --warmup 3 --profile all
run b128_vr0 "FBR_VR_WAVE=0" --batch 128 --steps 20 --warmup 5 --profile off
run b128_vr1 "FBR_VR_WAVE=1" --batch 128 --steps 20 --warmup 5 --profile off
run b128_vr0_n1 "FBR_VR_WAVE=0 FBR_NSUB=1" --batch 128 --steps 20 --warmup 5 --profile off
