#!/bin/bash
# Registration / crop GPU tests, then an SQ VALU pass of the new and the round-5 library (every
# kernel alone: per-launch VALU instructions and durations), then interleaved C2 B=1024 lines.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06b; mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "registration or crop or batch or c4 or golden or stream" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
CMD="bench.py --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for v in new prev; do
  L=$PKG/libfbr_hip.so; [ $v = prev ] && L=$PKG/libfbr_hip_prev.so
  FBR_LIB=$L timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_$v -o bench --output-format csv -- python3 $CMD > $OUT/sq_$v.log 2>&1 || { tail $OUT/sq_$v.log; exit 11; }
  python3 tools/valu_pmc.py $(find $OUT/sq_$v -name "*counter_collection.csv" | head -1) C2 1024 $OUT/valu_$v.json > $OUT/valu_$v.txt || exit 12
  echo "== $v"; cat $OUT/valu_$v.txt
done
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
for r in 1 2; do for v in new prev; do
  L=$PKG/libfbr_hip.so; [ $v = prev ] && L=$PKG/libfbr_hip_prev.so
  FBR_LIB=$L timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v $r', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items()})"
done; done
