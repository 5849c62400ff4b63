#!/bin/bash
# Round 5, call c: the round-3 mis-sort replay in the product kernels (the exact round-3 leader form
# inlined / outlined), the native RCCL tests, the GPU suite at HEAD (padded LDS pitches in
# k_project / k_compact) and the SQ decomposition of project / extract, bench.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -k "not inplace-leader-r03" > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 10; }
tail -3 $OUT/pytest_gpu.txt
CMD="bench.py --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d $OUT/sqa -o bench --output-format csv -- python3 $CMD > $OUT/sqa.log 2>&1 || { tail $OUT/sqa.log; exit 13; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/sqb -o bench --output-format csv -- python3 $CMD > $OUT/sqb.log 2>&1 || { tail $OUT/sqb.log; exit 14; }
python3 tools/sq_decomp.py $(find $OUT/sqa -name "*counter_collection.csv") $(find $OUT/sqb -name "*counter_collection.csv") $OUT/sq_decomp.json --config C2 --batch 1024 > $OUT/sq_decomp.txt 2>&1; cat $OUT/sq_decomp.txt
timeout -s KILL 300 rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE -d $OUT/mem -o bench --output-format csv -- python3 $CMD > $OUT/mem.log 2>&1 || { tail $OUT/mem.log; exit 15; }
python3 tools/mem_pmc.py $(find $OUT/mem -name "*counter_collection.csv") $OUT/mem_pmc.json > $OUT/mem_pmc.txt 2>&1; cat $OUT/mem_pmc.txt
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2; do for lpq in 1 8; do
  FBR_KNN_LPQ=$lpq timeout -k 10 300 python3 bench.py $Q > $OUT/ab_lpq${lpq}_$rep.json 2>/dev/null || exit 16
  python3 -c "import json; d=json.loads(open('$OUT/ab_lpq${lpq}_$rep.json').read().strip().splitlines()[-1]); print('LPQ $lpq rep $rep', d['value'])"
done; done
# C3 B=256: the round-2 build 69dd8f7 (21.5k then) against HEAD, interleaved on this box
for rep in 1 2; do
  (cd abwt/r02_69dd8f7 && timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --profile off) > $OUT/c3_69dd8f7_$rep.json 2>/dev/null || exit 17
  timeout -k 10 300 python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/c3_head_$rep.json 2>/dev/null || exit 18
  python3 -c "
import json
for t in ('69dd8f7', 'head'):
    d=json.loads(open('$OUT/c3_'+t+'_$rep.json').read().strip().splitlines()[-1]); print('C3', t, 'rep $rep', d['value'], d['ms_per_step'])"
done
timeout -k 10 900 python3 bench.py --exact-line 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 12; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('BENCH', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['frac'], d['kernel_ms_per_step'])"
