#!/bin/bash
# Round-4 profile: GPU suite; the bench workload under rocprofv3 PMC passes, each alone (FETCH_SIZE,
# WRITE_SIZE, an SQ/GRBM pass) -> profiles/hbm_traffic.json + profiles/valu_pmc.json; the same
# workload under a kernel trace + stats (its bench line prices against the fresh PMC files) and the
# roofline cross-check; the C5 SQ pass and C5 line (profiles/valu_pmc_c5.json); the default bench line.
# usage: tools/gpu_profile_r04.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r04}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 10; }
  tail -2 $OUT/pytest_gpu.txt
fi
CMD="bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o bench --output-format csv -- python3 $CMD --profile off > $OUT/bench_fetch.log 2>&1 || exit 12
echo fetch done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o bench --output-format csv -- python3 $CMD --profile off > $OUT/bench_write.log 2>&1 || exit 13
echo write done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq -o bench --output-format csv -- python3 $CMD --profile off > $OUT/bench_sq.log 2>&1 || exit 14
echo sq done
python3 tools/hbm_traffic.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") C2 1024 $OUT/hbm_traffic.json > $OUT/hbm_traffic.txt || exit 15
python3 tools/valu_pmc.py $(find $OUT/sq -name "*counter_collection.csv") C2 1024 $OUT/valu_pmc.json > $OUT/valu_pmc.txt || exit 16
cp $OUT/hbm_traffic.json profiles/hbm_traffic.json
cp $OUT/valu_pmc.json profiles/valu_pmc.json
cat $OUT/hbm_traffic.txt $OUT/valu_pmc.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 $CMD > $OUT/bench_trace.log 2>&1 || exit 11
echo trace done
python3 tools/roofline_check.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/bench_trace.log > $OUT/roofline_check.txt 2>&1 || exit 18
cat $OUT/roofline_check.txt
C5="bench.py --config C5 --batch 16 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_c5 -o bench --output-format csv -- python3 $C5 --profile off > $OUT/bench_sq_c5.log 2>&1 || exit 19
python3 tools/valu_pmc.py $(find $OUT/sq_c5 -name "*counter_collection.csv") C5 16 $OUT/valu_pmc_c5.json > $OUT/valu_pmc_c5.txt || exit 20
cp $OUT/valu_pmc_c5.json profiles/valu_pmc_c5.json
cat $OUT/valu_pmc_c5.txt
timeout -k 10 400 python3 $C5 --valu-json profiles/valu_pmc_c5.json > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 21
timeout -k 10 400 python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 22
timeout -k 10 900 python3 bench.py > $OUT/bench_final.log 2> $OUT/bench_final.err || exit 17
python3 -c "
import json; d=json.loads(open('$OUT/bench_final.log').read().strip().splitlines()[-1])
r=d['roofline']; print('FINAL', d['value'], d['ms_per_step'], r['bound'], r['kernel'], r['frac'], r.get('hbm_frac'), r.get('valu_frac'), r.get('traffic'))
print('latency', d.get('latency',{}).get('ms_per_scan_p50'), 'ingest', d.get('ingest',{}).get('value'), 'exact', d.get('exact_voxel_order',{}).get('value'), 'cpu', d.get('cpu_baseline',{}).get('value'))
for f in ('bench_c5.json', 'bench_c3.json'):
    e=json.loads(open('$OUT/'+f).read().strip().splitlines()[-1]); r=e['roofline']
    print(f, e['value'], e['ms_per_step'], r['bound'], r['kernel'], r.get('valu_frac'), r.get('hbm_frac'))"
