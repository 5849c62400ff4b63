#!/bin/bash
# A/B of environment settings on the bench workload (sequential per-kernel line + overlapped line).
# usage: tools/ab_env.sh TAG "ENV=.. ENV2=.." "ENV=.." ...   (an empty string = defaults)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
i=0
for E in "$@"; do
  i=$((i+1))
  n=$(echo "v${i}_$E" | tr ' =.' '_-p')
  env $E FBR_NSUB=1 timeout -k 10 200 python3 bench.py --batch ${BATCH:-256} --steps 4 --warmup 1 --no-cpu-baseline --latency 0 --ingest 0 --profile all > gpurun_out/abe_${TAG}_${n}_seq.log 2>&1 || exit 31
  env $E timeout -k 10 200 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --latency 0 --ingest 0 > gpurun_out/abe_${TAG}_${n}.log 2>&1 || exit 32
done
python3 tools/ab_summary.py gpurun_out/abe_${TAG}_*.log
