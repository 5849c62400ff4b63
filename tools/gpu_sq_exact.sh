#!/bin/bash
# SQ decomposition (two PMC passes, every dispatch alone) of the exact_voxel_order = 1 workload at
# B = 256, to see what the std::sort emulation's kernels wait on.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06sqx}; mkdir -p $OUT
CMD="bench.py --batch 256 --steps 2 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off --exact-voxel-order 1"
pmc() { local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $OUT/$name -o bench --output-format csv -- python3 $CMD > $OUT/bench_$name.log 2>&1 || { tail $OUT/bench_$name.log; return 1; }; }
pmc sqa SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 15
pmc sqb SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE || exit 16
csv() { find $OUT/$1 -name "*counter_collection.csv" | head -1; }
python3 tools/sq_decomp.py $(csv sqa) $(csv sqb) $OUT/sq_decomp.json --config C2 --batch 256 > $OUT/sq_decomp.txt || exit 20
cat $OUT/sq_decomp.txt
