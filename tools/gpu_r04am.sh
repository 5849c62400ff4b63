#!/bin/bash
# flat kNN walk with a branch-free row advance (libfbr_hip_rs.so, -DFBR_KNN_ROW_SEL) against the default build,
# build first, on the CPU: cd feature_base_pointcloud_registration_amd && python3 -c "import build; build.build_hip(defines=('FBR_KNN_ROW_SEL',), name='libfbr_hip_rs.so')"
# interleaved, B = 1024; then kernel stats of both
set -o pipefail
OUT=gpurun_out/r04am
mkdir -p $OUT
L=feature_base_pointcloud_registration_amd
run() {  # name, lib
  local name=$1 lib=$2
  FBR_LIB=$PWD/$L/$lib timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 10 --warmup 3 > $OUT/$name.json 2>>$OUT/err || exit 22
  echo "$name [$lib] $(python3 -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
}
run rs_a libfbr_hip_rs.so
run def_a libfbr_hip.so
run rs_b libfbr_hip_rs.so
run def_b libfbr_hip.so
run rs_c libfbr_hip_rs.so
run def_c libfbr_hip.so
export TMPDIR=/tmp
for v in rs def; do
  lib=libfbr_hip.so; [ $v = rs ] && lib=libfbr_hip_rs.so
  FBR_LIB=$PWD/$L/$lib FBR_NSUB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 --profile off --steps 4 --warmup 1 > $OUT/p_$v.log 2>&1 || exit 23
done
