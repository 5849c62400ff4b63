#!/bin/bash
# wave-tile kNN (k_knn_tile.hip): its parity tests first, then the whole GPU suite, then C5 / C3
# lines with the tiles on and off, then the default C2 bench line
set -o pipefail
OUT=gpurun_out/r04p
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "knn_tile or c5_dense" > $OUT/pytest_tile.txt 2>&1; rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -40 $OUT/pytest_tile.txt; exit 21; }
tail -2 $OUT/pytest_tile.txt
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
run c5_tile "FBR_KNN_TILE=1" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
run c5_notile "FBR_KNN_TILE=0" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
run c3_tile "FBR_KNN_TILE=1" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c3_notile "FBR_KNN_TILE=0" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c3_tile025r2 "FBR_KNN_TILE_CELL=0.25 FBR_KNN_TILE_REACH=2" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c3_tile025r1 "FBR_KNN_TILE_CELL=0.25 FBR_KNN_TILE_REACH=1" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c5_tile0125r2 "FBR_KNN_TILE_REACH=2" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
[ $rc -eq 0 ] || { tail -30 $OUT/pytest_tile.txt; exit 25; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 23; }
tail -2 $OUT/pytest.txt
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $OUT/bench.json 2>$OUT/bench.err || { tail -20 $OUT/bench.err; exit 24; }
tail -c 400 $OUT/bench.json
