#!/bin/bash
# Overlapped-only A/B of environment settings (default bench workload, no side lines), interleaved.
# usage: tools/ab_over.sh TAG "ENV=.." "ENV=.." ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
i=0
for E in "$@"; do
  i=$((i+1))
  n=$(echo "v${i}_$E" | tr ' =.' '_-p')
  env $E timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency 0 --ingest 0 > gpurun_out/abo_${TAG}_${n}.log 2>&1 || exit 32
done
python3 tools/ab_summary.py gpurun_out/abo_${TAG}_*.log
