#!/bin/bash
# Exact-order (std::sort emulation) check: the voxel-order selftests and the exact-mode tests, then
# the exact_voxel_order = 1 main line at B = 1024 (per-kernel times) and the default line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06x}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "voxel_order or exact or voxel_grid" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
summ() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items() if b > 0.01})"; }
timeout -k 10 300 python3 $B --exact-voxel-order 1 > $OUT/exact.json 2> $OUT/exact.err || { tail $OUT/exact.err; exit 14; }
summ $OUT/exact.json "exact B1024"
timeout -k 10 300 python3 $B > $OUT/def.json 2> $OUT/def.err || { tail $OUT/def.err; exit 15; }
summ $OUT/def.json "default B1024"
