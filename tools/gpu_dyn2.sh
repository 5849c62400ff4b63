#!/bin/bash
# Dynamic-row kNN iteration: kNN stats (diag build) and bench lines, C5 / C3, dyn vs unrolled.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
export FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_diag.so
for D in 1 0; do
FBR_KNN_DYN=$D CFG=C5 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5_dyn$D.txt 2>&1 || exit 31
FBR_KNN_DYN=$D CFG=C5 ITERS=1 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5_it0_dyn$D.txt 2>&1 || exit 32
FBR_KNN_DYN=$D CFG=C3 timeout -k 10 300 python3 tools/knn_stats.py 64 0.5/0.125 > $OUT/knn_c3_dyn$D.txt 2>&1 || exit 33
done
B="timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline"
$B --config C5 --batch 16 > $OUT/c5_dyn.json 2>>$OUT/err || exit 23
FBR_KNN_CELL=0.25 $B --config C5 --batch 16 > $OUT/c5_dyn_025.json 2>>$OUT/err || exit 24
$B --config C3 --batch 256 > $OUT/c3_dyn.json 2>>$OUT/err || exit 28
grep -h "cell" $OUT/knn_*.txt
