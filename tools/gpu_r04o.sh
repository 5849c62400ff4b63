#!/bin/bash
# three launch slots by default: the whole GPU suite, then the default bench line
set -o pipefail
OUT=gpurun_out/r04o
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
timeout -k 10 400 python3 bench.py --steps 10 --warmup 3 > $OUT/bench.json 2>$OUT/bench.err || { tail -20 $OUT/bench.err; exit 22; }
tail -c 600 $OUT/bench.json
