#!/bin/bash
# pipeline depth (FBR_PIPE 2 / 3) at B = 128 / 256 / 1024, C4 tests, and the round-2 bisect builds
set -o pipefail
OUT=gpurun_out/r04m
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_c4.py tests/test_distributed.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$e] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
for B in 128 256 1024; do
  st=$((20 * 128 / B + 5)); [ $st -lt 10 ] && st=10
  run b${B}_p2 "FBR_PIPE=2" --batch $B --steps $st --warmup 3
  run b${B}_p3 "FBR_PIPE=3" --batch $B --steps $st --warmup 3
done
run b1024_p2b "FBR_PIPE=2" --batch 1024 --steps 10 --warmup 3
run b1024_p3b "FBR_PIPE=3" --batch 1024 --steps 10 --warmup 3
tags=""
for t in r02mid r02pregrid r02grid r02pretile; do [ -f ablib/$t/feature_base_pointcloud_registration_amd/libfbr_hip.so ] && tags="$tags $t"; done
[ -n "$tags" ] && bash tools/gpu_bisect.sh r04m_bisect $tags
