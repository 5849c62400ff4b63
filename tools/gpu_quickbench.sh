#!/bin/bash
# Quick iteration call: a pytest selection (-m gpu), the default bench line, a sequential per-kernel
# line (FBR_NSUB=1, B = 256), and optional FETCH_SIZE / WRITE_SIZE passes (PMC=1).
# usage: tools/gpu_quickbench.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-quick}
SEL=${2:-tests/test_gpu_parity.py}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$SEL" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 21; }
  tail -2 $OUT/pytest.log
fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 22
FBR_NSUB=1 timeout -k 10 300 python3 bench.py --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/seq.json 2>> $OUT/bench.err || exit 23
if [ "${PMC:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o b --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile off > $OUT/fetch.log 2>&1 || exit 24
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o b --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile off > $OUT/write.log 2>&1 || exit 25
  python3 tools/hbm_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") C2 1024 $OUT/hbm_traffic.json || exit 26
fi
python3 - "$OUT" <<'EOF'
import json, sys
out = sys.argv[1]
for f in ("bench.json", "seq.json"):
    d = json.load(open(f"{out}/{f}"))
    ks = d["roofline"]["kernels"]
    print(f, d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_launch_us']:.0f}us/{v['frac']:.3f}" for k, v in ks.items()))
EOF
