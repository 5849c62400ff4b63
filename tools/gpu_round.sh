#!/bin/bash
# One GPU call: the -m gpu suite, the round profile (bench under rocprofv3 stats + PMC passes +
# final bench line), then a per-GPU batch-size sweep.  usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || exit 21
bash tools/profile_round.sh $TAG || exit 22
for B in 512 768; do
  timeout -k 10 300 python3 bench.py --batch $B --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_b${B}_$TAG.log 2>&1 || exit 23
done
tail -n 3 gpurun_out/pytest_gpu_$TAG.log
