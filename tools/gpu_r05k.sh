#!/bin/bash
# Round 5, call k: kNN work statistics at the default cells (C2 B = 256, C3 B = 64, C5 B = 4):
# points within the warm-start cut per flat query (sizing a filter-then-insert walk).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
export FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_kstats.so
timeout -k 10 200 python3 tools/knn_stats.py 256 default > $OUT/knn_stats.txt 2>&1 || { cat $OUT/knn_stats.txt; exit 3; }
CFG=C3 timeout -k 10 200 python3 tools/knn_stats.py 64 default >> $OUT/knn_stats.txt 2>&1 || { cat $OUT/knn_stats.txt; exit 4; }
CFG=C5 timeout -k 10 300 python3 tools/knn_stats.py 4 default >> $OUT/knn_stats.txt 2>&1 || { cat $OUT/knn_stats.txt; exit 5; }
cat $OUT/knn_stats.txt
