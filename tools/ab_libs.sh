#!/bin/bash
# A/B of diagnostic library builds on the bench workload: for each FBR_LIB variant, one sequential
# (FBR_NSUB=1, per-kernel times) and one default (overlapped) bench line.  usage: tools/ab_libs.sh TAG lib...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for L in "$@"; do
  n=$(basename $L .so)
  FBR_LIB=$PWD/$L FBR_NSUB=1 timeout -k 10 200 python3 bench.py --batch ${BATCH:-256} --steps 4 --warmup 1 --no-cpu-baseline --profile all > gpurun_out/ab_${TAG}_${n}_seq.log 2>&1 || exit 31
  FBR_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/ab_${TAG}_${n}.log 2>&1 || exit 32
done
python3 tools/ab_summary.py gpurun_out/ab_${TAG}_*.log
