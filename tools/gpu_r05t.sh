#!/bin/bash
# Round 5, call t: SQ counters per kernel of the single-scan chain (latency probe, C2).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/a -o a --output-format csv -- python3 tools/latency_probe.py 20 > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 3; }
python3 tools/pmc_by_kernel.py $(find $OUT/a -name "*counter_collection.csv" | head -1) > $OUT/a.txt || exit 4
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F64 SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/b -o b --output-format csv -- python3 tools/latency_probe.py 20 > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 5; }
python3 tools/pmc_by_kernel.py $(find $OUT/b -name "*counter_collection.csv" | head -1) > $OUT/b.txt || exit 6
cat $OUT/a.txt $OUT/b.txt
