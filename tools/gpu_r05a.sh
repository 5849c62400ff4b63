#!/bin/bash
# Round 5, call a: VALU roof calibration (probe sweep + its SQ pass), the SQ wait / instruction-mix
# decomposition passes of the C2 B=1024 workload, and a default bench line on this box.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 120 python3 tools/valu_calib.py run $OUT/valu_calib.json > $OUT/valu_calib.txt 2>&1 || { cat $OUT/valu_calib.txt; exit 10; }
cat $OUT/valu_calib.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/calib_sq -o calib --output-format csv -- python3 tools/valu_calib.py run > $OUT/calib_sq.log 2>&1 || { tail $OUT/calib_sq.log; exit 11; }
python3 tools/valu_calib.py pmc $(find $OUT/calib_sq -name "*counter_collection.csv") $OUT/valu_calib.json $OUT/valu_calib_pmc.json || exit 12
CMD="bench.py --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d $OUT/sqa -o bench --output-format csv -- python3 $CMD > $OUT/sqa.log 2>&1 || { tail $OUT/sqa.log; exit 13; }
echo pass A done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/sqb -o bench --output-format csv -- python3 $CMD > $OUT/sqb.log 2>&1 || { tail $OUT/sqb.log; exit 14; }
echo pass B done
python3 tools/sq_decomp.py $(find $OUT/sqa -name "*counter_collection.csv") $(find $OUT/sqb -name "*counter_collection.csv") $OUT/sq_decomp.json --calib $OUT/valu_calib_pmc.json > $OUT/sq_decomp.txt 2>&1; cat $OUT/sq_decomp.txt
timeout -k 10 600 python3 bench.py --exact-line 0 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 15; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('BENCH', d['value'], d['ms_per_step'], r['kernel'], r['frac'], d.get('latency',{}).get('ms_per_scan_p50'))"
