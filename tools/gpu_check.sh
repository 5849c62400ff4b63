#!/bin/bash
# One GPU call: the -m gpu suite, the default bench line, a --profile off line (timing overhead
# check), and a rocprofv3 --kernel-trace --stats pass of the default bench command; then the
# roofline cross-check.  usage: tools/gpu_check.sh TAG [pytest selection]
set -o pipefail
TAG=${1:-chk}
SEL=${2:-tests}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 21; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 22
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --profile off --no-cpu-baseline > $OUT/bench_noprof.json 2>> $OUT/bench.err || exit 23
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || exit 24
STATS=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
python3 tools/roofline_check.py $STATS $OUT/bench_trace.json > $OUT/roofline_check.txt || exit 25
cat $OUT/roofline_check.txt
