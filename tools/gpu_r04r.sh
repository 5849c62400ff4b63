#!/bin/bash
# query-binned block tiles (k_knn_tile.hip): counters and batch time on C5 / C3, parity tests, C5 / C3 bench lines
set -o pipefail
OUT=gpurun_out/r04r
mkdir -p $OUT
p() {  # "ENV=.. ..." CONFIG B
  env FBR_KNN_TILE_STATS=1 $1 timeout -k 10 300 python3 tools/tile_probe.py $2 $3 | tee -a $OUT/probe.txt || exit 31
}
p "FBR_KNN_TILE=0" C5 4
p "FBR_KNN_TILE=1" C5 4
p "FBR_KNN_TILE=0" C5 16
p "FBR_KNN_TILE=1" C5 16
p "FBR_KNN_TILE=0" C3 64
p "FBR_KNN_TILE=1" C3 64
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "knn_tile or c5_dense or c3_ouster" > $OUT/pytest_tile.txt 2>&1; rc=$?; tail -3 $OUT/pytest_tile.txt
[ $rc -le 1 ] || exit 32
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  python3 - $OUT/$name.json "$name [$e]" <<'PY' | tee -a $OUT/summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d.get("roofline", {}).get("kernels", {})
print(sys.argv[2], round(d["value"], 1), d["ms_per_step"], " ".join(f"{k}={v['ms_per_step']:.3f}" for k, v in ks.items()))
PY
}
run c5_tile "FBR_KNN_TILE=1" --config C5 --batch 16 --steps 3 --warmup 1 --profile off
run c5_notile "FBR_KNN_TILE=0" --config C5 --batch 16 --steps 3 --warmup 1 --profile off
run c5_tile_prof "FBR_KNN_TILE=1" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
