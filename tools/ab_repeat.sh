#!/bin/bash
# Interleaved repeats of the default bench line under environment variants (run-to-run noise is
# about +-2 %, so single A/B pairs decide nothing).  usage: tools/ab_repeat.sh TAG REPS "ENV=.." ...
set -o pipefail
TAG=$1; REPS=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $REPS); do
  i=0
  for E in "$@"; do
    i=$((i+1))
    env $E timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abr_${TAG}_v${i}_r${r}.log 2>&1 || exit 41
    echo "v$i [$E] r$r $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/abr_${TAG}_v${i}_r${r}.log)"
  done
done
