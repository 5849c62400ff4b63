#!/bin/bash
# Exact-order iteration: selftests + VoxelGrid check, then sequential / overlapped bench lines with
# and without the exact order.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_voxel_order.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_vo.log 2>&1 || { tail -20 $OUT/pytest_vo.log; exit 21; }
SIZES=3000,16000,18432,18433,40000 timeout -k 10 200 python3 -u tools/vg_exact_check.py > $OUT/vg.log 2>&1 || exit 22
cat $OUT/vg.log
B="timeout -k 10 400 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --steps 10 --warmup 3"
FBR_NSUB=1 $B --batch 256 > $OUT/seq_exact.json 2>>$OUT/err || exit 24
FBR_VG_EXACT=0 FBR_NSUB=1 $B --batch 256 > $OUT/seq_noexact.json 2>>$OUT/err || exit 25
$B > $OUT/bench_exact.json 2>>$OUT/err || exit 26
