#!/bin/bash
# round-end rehearsal at HEAD: whole GPU suite, smoke(), the default bench line
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 10; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 11; }
tail -1 $OUT/smoke.txt
timeout -k 10 900 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 12; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
r=d['roofline']; print('BENCH', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['frac'], r.get('hbm_frac'))
print('latency', d['latency']['ms_per_scan_p50'], d['latency']['ms_per_scan_p99'], 'ingest', d['ingest']['value'], 'exact', d['exact_voxel_order']['value'], 'cpu', d['cpu_baseline']['value'], 'parity', d['parity_vs_ref'])"
