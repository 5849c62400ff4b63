#!/bin/bash
# VoxelGrid + registration parity tests, then a default bench line.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "voxel or registration or batch or exact or smoke or golden" > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 21; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 23
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['kernel_ms_per_step'])"
