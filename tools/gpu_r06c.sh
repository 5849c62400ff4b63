#!/bin/bash
# Round-6 check: full GPU suite + smoke, then the default bench line (latency + ingest, no CPU
# baseline) twice.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06c; mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 9; }
cat $OUT/smoke.txt
for r in 1 2; do
timeout -k 10 400 python3 bench.py --no-cpu-baseline --exact-line 0 --latency 100 > $OUT/bench_$r.json 2> $OUT/bench_$r.err || { tail $OUT/bench_$r.err; exit 11; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('bench', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items()})
print('latency', d['latency']); print('ingest', d['ingest']['value']); r=d['roofline']; print('roof', r['kernel'], r['bound'], r['frac'], r['hbm_frac'])"
done
