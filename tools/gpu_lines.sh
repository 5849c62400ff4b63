#!/bin/bash
# Extra bench lines for profiles/: the C4 per-GPU share (B = 128), C3 and C5, and SQ issue counters
# (sequential sub-batches, so every dispatch runs alone) for the VALU-issue fraction.
# usage: tools/gpu_lines.sh TAG
set -o pipefail
TAG=${1:-lines}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --batch 128 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_b128.json 2> $OUT/err.log || exit 31
timeout -k 10 600 python3 bench.py --config C3 --batch 256 --steps 10 --warmup 3 --cpu-sample 8 > $OUT/c3_b256.json 2>> $OUT/err.log || exit 32
timeout -k 10 600 python3 bench.py --config C5 --batch 16 --steps 5 --warmup 2 --cpu-sample 2 > $OUT/c5_b16.json 2>> $OUT/err.log || exit 33
SQ="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
FBR_NSUB=1 timeout -k 10 300 rocprofv3 --pmc $SQ -d $OUT/sq_c2 -o sq --output-format csv -- python3 bench.py --batch 256 --steps 3 --warmup 1 --no-cpu-baseline --profile off > $OUT/sq_c2.log 2>&1 || exit 34
FBR_NSUB=1 timeout -k 10 300 rocprofv3 --pmc $SQ -d $OUT/sq_c5 -o sq --output-format csv -- python3 bench.py --config C5 --batch 8 --steps 2 --warmup 1 --no-cpu-baseline --profile off > $OUT/sq_c5.log 2>&1 || exit 35
FBR_NSUB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/seq_c2 -o seq --output-format csv -- python3 bench.py --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/seq_c2.json 2> $OUT/seq_c2.err || exit 36
ls -R $OUT | head -40
