#!/bin/bash
# Kernel trace of B = 128 bench steps (3 sub-batches), summarised by tools/step_timeline.py.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o tr -- python3 bench.py --batch 128 --steps 12 --warmup 4 --latency 0 --ingest 0 --no-cpu-baseline --profile off > $OUT/b128.json 2> $OUT/b128.err || exit 31
F=$(find $OUT/tr -name "*kernel_trace.csv" | head -1)
python3 tools/step_timeline.py $F 3 6 > $OUT/timeline.txt || exit 32
cat $OUT/timeline.txt
