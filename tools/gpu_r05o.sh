#!/bin/bash
# Round 5, call o: kNN statistics of the per-lane flat walk (points per flat query, lane efficiency).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
export FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_kstats.so FBR_KNN_BAL=0
timeout -k 10 200 python3 tools/knn_stats.py 256 default > $OUT/knn_stats.txt 2>&1 || { cat $OUT/knn_stats.txt; exit 3; }
cat $OUT/knn_stats.txt
