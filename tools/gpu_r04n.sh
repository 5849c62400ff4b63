#!/bin/bash
# MFMA normal-equation partials: GPU parity suite, A/B against the butterfly (FBR_RES_MFMA=0),
# pipeline depth, round-2 bisect builds present in ablib/
set -o pipefail
OUT=gpurun_out/r04n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
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
run b1024_mfma "FBR_RES_MFMA=1" --batch 1024 --steps 10 --warmup 3 --profile all
run b1024_bfly "FBR_RES_MFMA=0" --batch 1024 --steps 10 --warmup 3 --profile all
run b1024_mfma_off "FBR_RES_MFMA=1" --batch 1024 --steps 10 --warmup 3 --profile off
run b1024_bfly_off "FBR_RES_MFMA=0" --batch 1024 --steps 10 --warmup 3 --profile off
run b1024_mfma_off2 "FBR_RES_MFMA=1" --batch 1024 --steps 10 --warmup 3 --profile off
for B in 128 256; do
  st=$((20 * 128 / B + 5))
  run b${B}_p2 "FBR_PIPE=2" --batch $B --steps $st --warmup 3 --profile off
  run b${B}_p3 "FBR_PIPE=3" --batch $B --steps $st --warmup 3 --profile off
done
run b1024_p3 "FBR_PIPE=3" --batch 1024 --steps 10 --warmup 3 --profile off
run c5_cell05 "FBR_RES_MFMA=1" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
run c5_cell025 "FBR_KNN_CELL=0.25" --config C5 --batch 16 --steps 3 --warmup 1 --profile all
run c3_cell05 "FBR_RES_MFMA=1" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
run c3_cell025 "FBR_KNN_CELL=0.25" --config C3 --batch 256 --steps 5 --warmup 2 --profile all
tags=""  # ablib builds travel only when .gpurunignore lets them
for t in r02mid r02pretile; do [ -f ablib/$t/feature_base_pointcloud_registration_amd/libfbr_hip.so ] && tags="$tags $t"; done
[ -n "$tags" ] && bash tools/gpu_bisect.sh r04n_bisect $tags
