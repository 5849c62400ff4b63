#!/bin/bash
# kNN per-query statistics (diagnostic build) for C5 and C2 at several cell sizes, all iterations
# and iteration 0 alone.  usage: tools/gpu_knnstats.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_diag.so
CFG=C5 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5.txt 2>&1 || exit 31
CFG=C5 ITERS=1 timeout -k 10 300 python3 tools/knn_stats.py 16 0.5/0.125 0.25/0.125 > $OUT/knn_c5_it0.txt 2>&1 || exit 32
CFG=C2 timeout -k 10 300 python3 tools/knn_stats.py 256 1/0.25 > $OUT/knn_c2.txt 2>&1 || exit 33
CFG=C3 timeout -k 10 300 python3 tools/knn_stats.py 64 0.5/0.125 0.25/0.125 > $OUT/knn_c3.txt 2>&1 || exit 34
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/bench_c2.json 2>$OUT/bench.err || exit 35
cat $OUT/knn_*.txt
