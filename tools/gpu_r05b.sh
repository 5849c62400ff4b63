#!/bin/bash
# Round 5, call b: the round-3 leader-sort replay (selftest variant 5) on its own, then the GPU suite
# (ADVICE fixes, per-context exact mode / pipeline depth) and a default bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05b
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_voxel_order.py -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_voxel_order.txt 2>&1
echo "voxel_order rc=$?"; grep -E "PASS|FAIL|Error|assert" $OUT/pytest_voxel_order.txt | head -30
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "not inplace-leader-r03" > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -3 $OUT/pytest_gpu.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 11; }
cat $OUT/smoke.txt
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 12; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('BENCH', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['frac'], r.get('hbm_frac'), d.get('latency',{}).get('ms_per_scan_p50'), d.get('exact_voxel_order'))"
