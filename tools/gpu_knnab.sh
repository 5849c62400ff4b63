#!/bin/bash
# kNN variant bench lines: C2 default, C5 / C3 with the unrolled search.  usage: tools/gpu_knnab.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B="timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline"
$B --config C5 --batch 16 > $OUT/c5_u05.json 2>>$OUT/err || exit 23
FBR_KNN_CELL=0.25 $B --config C5 --batch 16 > $OUT/c5_u025.json 2>>$OUT/err || exit 24
$B --config C3 --batch 256 > $OUT/c3_u05.json 2>>$OUT/err || exit 25
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/c2.json 2>>$OUT/err || exit 27
