#!/bin/bash
# C3 (B = 256) A/B of the default library and one FBR_LIB variant, interleaved.  usage: TAG LIB
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
B="python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 300 $B > $OUT/def_$r.json 2>>$OUT/err || exit 21
  FBR_LIB=$PWD/$2 timeout -k 10 300 $B > $OUT/var_$r.json 2>>$OUT/err || exit 22
done
for f in $OUT/def_*.json $OUT/var_*.json; do
  echo "$f $(python3 -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], round(d['kernel_ms_per_step']['features'],3), d['parity_vs_ref']['n_sel_equal'])")" | tee -a $OUT/summary.txt
done
