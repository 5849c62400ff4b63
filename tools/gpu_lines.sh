#!/bin/bash
# Bench lines: B = 128 (the C4 per-GPU share), sequential B = 256, default B = 1024.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
B="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --no-cpu-baseline"
$B --batch 128 > $OUT/b128.json 2>>$OUT/err || exit 21
FBR_NSUB=1 $B --batch 256 > $OUT/seq256.json 2>>$OUT/err || exit 22
$B > $OUT/b1024.json 2>>$OUT/err || exit 23
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python3 bench.py --batch 128 --steps 4 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline --profile off > $OUT/b128_trace.json 2>>$OUT/err || exit 24
