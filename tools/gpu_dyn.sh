#!/bin/bash
# Dynamic-row kNN check: parity tests (dyn vs unrolled, C3, C5), then C5 / C3 bench lines for
# cell-size variants and the unrolled baseline.  usage: tools/gpu_dyn.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dynamic_row or sparse_grid or c3_ or c5_ or registration_matches_oracle_c2" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -3 $OUT/pytest.log
B="timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline"
FBR_KNN_DYN=0 $B --config C5 --batch 16 > $OUT/c5_unrolled.json 2>>$OUT/err || exit 22
$B --config C5 --batch 16 > $OUT/c5_dyn.json 2>>$OUT/err || exit 23
FBR_KNN_CELL=0.25 $B --config C5 --batch 16 > $OUT/c5_dyn_025.json 2>>$OUT/err || exit 24
FBR_KNN_CELL=0.25 FBR_KNN_CELL_X=0.0625 $B --config C5 --batch 16 > $OUT/c5_dyn_025_0625.json 2>>$OUT/err || exit 25
FBR_KNN_CELL=0.125 FBR_KNN_CELL_X=0.0625 $B --config C5 --batch 16 > $OUT/c5_dyn_0125_0625.json 2>>$OUT/err || exit 26
FBR_KNN_DYN=0 $B --config C3 --batch 256 > $OUT/c3_unrolled.json 2>>$OUT/err || exit 27
$B --config C3 --batch 256 > $OUT/c3_dyn.json 2>>$OUT/err || exit 28
FBR_KNN_CELL=0.25 $B --config C3 --batch 256 > $OUT/c3_dyn_025.json 2>>$OUT/err || exit 29
echo ok
