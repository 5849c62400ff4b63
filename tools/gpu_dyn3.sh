#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
export FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_diag.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dynamic_row or sparse_grid or c3_ or c5_ or registration_matches_oracle_c2 or batch_" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
tail -2 $OUT/pytest.log
FBR_KNN_DYN=0 CFG=C5 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5.txt 2>&1 || exit 31
FBR_KNN_DYN=0 CFG=C5 ITERS=1 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5_it0.txt 2>&1 || exit 32
CFG=C2 timeout -k 10 300 python3 tools/knn_stats.py 256 1/0.25 > $OUT/knn_c2.txt 2>&1 || exit 33
B="timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline"
FBR_KNN_DYN=0 $B --config C5 --batch 16 > $OUT/c5_u05.json 2>>$OUT/err || exit 23
FBR_KNN_DYN=0 FBR_KNN_CELL=0.25 $B --config C5 --batch 16 > $OUT/c5_u025.json 2>>$OUT/err || exit 24
FBR_KNN_DYN=0 $B --config C3 --batch 256 > $OUT/c3_u05.json 2>>$OUT/err || exit 25
FBR_KNN_DYN=0 FBR_KNN_CELL=0.25 $B --config C3 --batch 256 > $OUT/c3_u025.json 2>>$OUT/err || exit 26
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/c2.json 2>>$OUT/err || exit 27
