#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
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
run seq "FBR_NSUB=1 FBR_PIPE=0" --batch 256 --steps 5 --warmup 2 --profile all
run b1024 "" --batch 1024 --steps 10 --warmup 3 --profile all
run b1024_noprof "" --batch 1024 --steps 10 --warmup 3 --profile off
run b128_noprof "" --batch 128 --steps 40 --warmup 5 --profile off
