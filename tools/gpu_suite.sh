#!/bin/bash
# The -m gpu suite, smoke(), and a default bench line.  usage: tools/gpu_suite.sh TAG [extra bench args]
set -o pipefail
OUT=gpurun_out/$1
shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 21; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 22
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err || exit 23
timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/bench_c5.json 2>> $OUT/bench.err || exit 24
cat $OUT/smoke.log
