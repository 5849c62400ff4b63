#!/bin/bash
# per-ring surf filter with the candidates staged in LDS for the centroid pass (libfbr_hip_vrl.so,
# -DFBR_VR_LDS_PTS): GPU suite on that build, interleaved A/B, kernel stats + FETCH_SIZE of both
set -o pipefail
OUT=gpurun_out/r04ai
mkdir -p $OUT
L=feature_base_pointcloud_registration_amd
FBR_LIB=$PWD/$L/libfbr_hip_vrl.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -2 $OUT/pytest.log
run() {  # name, lib
  local name=$1 lib=$2
  FBR_LIB=$PWD/$L/$lib timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$lib] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run vrl_a libfbr_hip_vrl.so
run def_a libfbr_hip.so
run vrl_b libfbr_hip_vrl.so
run def_b libfbr_hip.so
run vrl_c libfbr_hip_vrl.so
run def_c libfbr_hip.so
export TMPDIR=/tmp
for v in vrl def; do
  lib=libfbr_hip.so; [ $v = vrl ] && lib=libfbr_hip_vrl.so
  FBR_LIB=$PWD/$L/$lib FBR_NSUB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 4 --warmup 1 > $OUT/p_$v.log 2>&1 || exit 23
  FBR_LIB=$PWD/$L/$lib timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$v -o run --output-format csv -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 4 --warmup 1 > $OUT/f_$v.log 2>&1 || exit 24
done
