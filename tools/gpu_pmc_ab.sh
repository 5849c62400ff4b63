#!/bin/bash
# PMC A/B of the in-tree library (new) against libfbr_hip_prev.so (prev) on the bench workload
# (C2, B = 1024): the SQ instruction-mix pass and the memory-pipeline pass, each alone, then the
# per-kernel sums of a kernel family (tools/pmc_family.py).  usage: tools/gpu_pmc_ab.sh TAG [family]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; KF=${2:-k_gn_knn}
mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
CMD="bench.py --steps 4 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in new prev; do
  if [ $v = prev ]; then export FBR_LIB=$PKG/libfbr_hip_prev.so; else export FBR_LIB=$PKG/libfbr_hip.so; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/sq_$v -o bench --output-format csv -- python3 $CMD > $OUT/sq_$v.log 2>&1 || { tail $OUT/sq_$v.log; exit 11; }
  timeout -s KILL 300 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ GRBM_GUI_ACTIVE -d $OUT/mem_$v -o bench --output-format csv -- python3 $CMD > $OUT/mem_$v.log 2>&1 || { tail $OUT/mem_$v.log; exit 12; }
  python3 tools/pmc_family.py "$KF" $OUT/sq_$v/bench_counter_collection.csv $OUT/mem_$v/bench_counter_collection.csv | sed "s/^/$v /"
done
