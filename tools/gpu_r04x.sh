#!/bin/bash
# ingest line (host scans -> HBM -> poses) by packing-thread count
set -o pipefail
OUT=gpurun_out/r04x
mkdir -p $OUT
for e in "FBR_STAGE_THREADS=8" "FBR_STAGE_THREADS=16" "FBR_STAGE_THREADS=12" "FBR_STAGE_THREADS=8" "FBR_STAGE_THREADS=16"; do
  env $e timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --latency 0 --ingest 2 --exact-line 0 --no-cpu-baseline --profile off > $OUT/b.json 2>> $OUT/err || exit 22
  echo "[$e] $(python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); g=d['ingest']; print(g['value'], g['h2d_GBps'], g['poses_equal_resident'])")" | tee -a $OUT/summary.txt
done
# C3: flat row queue for the 0.5 m cells (FBR_KNN_FLAT_R2)
for e in "FBR_KNN_FLAT_R2=0" "FBR_KNN_FLAT_R2=1" "FBR_KNN_FLAT_R2=0" "FBR_KNN_FLAT_R2=1"; do
  env $e timeout -k 10 400 python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/c3.json 2>> $OUT/err || exit 23
  echo "C3 [$e] $(python3 -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
done
env FBR_KNN_FLAT_R2=1 timeout -k 10 400 python3 bench.py --config C5 --batch 16 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/c5.json 2>> $OUT/err || exit 24
echo "C5 [FBR_KNN_FLAT_R2=1] $(python3 -c "import json; d=json.loads(open('$OUT/c5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")" | tee -a $OUT/summary.txt
