#!/bin/bash
# Round-5 profile at HEAD: GPU suite + smoke; the bench workload (C2, B = 1024) under rocprofv3 PMC
# passes, each alone (FETCH_SIZE, WRITE_SIZE -> hbm_traffic.json; SQ VALU -> valu_pmc.json; the two
# SQ wait / instruction-mix passes -> sq_decomp.json; the memory pipeline -> mem_pmc.json); the same
# workload under a kernel trace + stats (its bench line prices against the fresh PMC files), the
# roofline cross-check and the concurrency profile; the C5 SQ pass and C5 / C3 lines; the default
# bench line last.  usage: tools/gpu_profile_r05.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r05}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 10; }
  tail -2 $OUT/pytest_gpu.txt
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 9; }
  cat $OUT/smoke.txt
fi
CMD="bench.py --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
pmc() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $OUT/$name -o bench --output-format csv -- python3 $CMD --profile off > $OUT/bench_$name.log 2>&1 || { tail $OUT/bench_$name.log; return 1; }
  echo "$name done"
}
pmc fetch FETCH_SIZE || exit 12
pmc write WRITE_SIZE || exit 13
pmc sq SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 14
pmc sqa SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 15
pmc sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 16
pmc mem TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE || exit 17
csv() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/hbm_traffic.py $(csv fetch) $(csv write) C2 1024 $OUT/hbm_traffic.json > $OUT/hbm_traffic.txt || exit 18
python3 tools/valu_pmc.py $(csv sq) C2 1024 $OUT/valu_pmc.json > $OUT/valu_pmc.txt || exit 19
python3 tools/sq_decomp.py $(csv sqa) $(csv sqb) $OUT/sq_decomp.json --config C2 --batch 1024 > $OUT/sq_decomp.txt || exit 20
python3 tools/mem_pmc.py $(csv mem) $OUT/mem_pmc.json > $OUT/mem_pmc.txt || exit 21
cp $OUT/hbm_traffic.json profiles/hbm_traffic.json
cp $OUT/valu_pmc.json profiles/valu_pmc.json
cp $OUT/sq_decomp.json profiles/sq_decomp.json
cat $OUT/hbm_traffic.txt $OUT/valu_pmc.txt $OUT/sq_decomp.txt $OUT/mem_pmc.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $CMD > $OUT/bench_trace.log 2>&1 || exit 22
echo trace done
python3 tools/roofline_check.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/bench_trace.log --trace $(find $OUT/trace -name "*kernel_trace.csv" | head -1) > $OUT/roofline_check.txt 2>&1 || exit 23
python3 tools/concurrency.py $(find $OUT/trace -name "*kernel_trace.csv" | head -1) 6 > $OUT/concurrency.txt 2>&1 || exit 24
cat $OUT/roofline_check.txt $OUT/concurrency.txt
C5="bench.py --config C5 --batch 16 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_c5 -o bench --output-format csv -- python3 $C5 --profile off > $OUT/bench_sq_c5.log 2>&1 || exit 25
python3 tools/valu_pmc.py $(find $OUT/sq_c5 -name "*counter_collection.csv") C5 16 $OUT/valu_pmc_c5.json > $OUT/valu_pmc_c5.txt || exit 26
cp $OUT/valu_pmc_c5.json profiles/valu_pmc_c5.json
timeout -k 10 400 python3 $C5 --valu-json profiles/valu_pmc_c5.json > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 27
timeout -k 10 400 python3 bench.py --config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 28
timeout -k 10 900 python3 bench.py > $OUT/bench_final.json 2> $OUT/bench_final.err || exit 29
python3 -c "
import json; d=json.loads(open('$OUT/bench_final.json').read().strip().splitlines()[-1])
r=d['roofline']; print('FINAL', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['frac'], r.get('hbm_frac'), r.get('valu_frac'), r.get('traffic'))
print('latency', d.get('latency',{}).get('ms_per_scan_p50'), 'ingest', d.get('ingest',{}).get('value'), 'exact', d.get('exact_voxel_order',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))
for f in ('bench_c5.json', 'bench_c3.json'):
    e=json.loads(open('$OUT/'+f).read().strip().splitlines()[-1]); r=e['roofline']
    print(f, e['value'], e['ms_per_step'], r['bound'], r['kernel'], r.get('valu_frac'), r.get('hbm_frac'))"
