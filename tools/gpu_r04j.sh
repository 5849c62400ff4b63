#!/bin/bash
# (1) the ballot-leader in-place sort inside the product kernel (diagnostic build), (2) SQ VALU
# counters of the two per-ring surf filters (FBR_VR_WAVE=0 / 1), sequential B = 256.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
bash tools/gpu_leader.sh r04j
CMD="bench.py --batch 256 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in 0 1; do
  FBR_VR_WAVE=$v FBR_NSUB=1 FBR_PIPE=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_vr$v -o b --output-format csv -- python3 $CMD > $OUT/sq_vr$v.log 2>&1 || exit 31
  python3 tools/valu_pmc.py $(find $OUT/sq_vr$v -name "*counter_collection.csv") C2 256 $OUT/valu_vr$v.json | tee $OUT/valu_vr$v.txt
done
