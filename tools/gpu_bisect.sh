#!/bin/bash
# C3 / C5 lines of older commits' builds (ablib/<tag>, git archive + in-tree build) next to HEAD.
# usage: tools/gpu_bisect.sh OUTTAG tag...
set -o pipefail
OUT=$PWD/gpurun_out/$1; shift
mkdir -p $OUT
summ() {
  python3 - "$1" "$2" <<'PY' | tee -a $OUT/summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d["roofline"]["kernels"]
print(sys.argv[2], round(d["value"], 1), d["ms_per_step"], " ".join(f"{k}={v['ms_per_step']:.2f}" for k, v in ks.items()))
PY
}
one() {  # dir tag env
  local dir=$1 tag=$2 e=$3
  (cd $dir && env $e timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline --profile all > $OUT/c3_$tag.json 2>>$OUT/err) || exit 21
  summ $OUT/c3_$tag.json "C3 $tag"
  (cd $dir && env $e timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 3 --warmup 1 --latency 0 --ingest 0 --no-cpu-baseline --profile all > $OUT/c5_$tag.json 2>>$OUT/err) || exit 22
  summ $OUT/c5_$tag.json "C5 $tag"
}
for t in "$@"; do one ablib/$t $t ""; done
one . head_nopipe "FBR_PIPE=0 FBR_NSUB=3"
one . head ""
