#!/bin/bash
# Two quick probes: (1) ingest rate vs packing threads (FBR_STAGE_THREADS 8 / 16 / 24); (2) the
# projection's global first-wins merge atomics replaced by plain stores (diagnostic timing build
# libfbr_hip_projstore.so: an upper bound of what an exclusive-column merge could save).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06m}; mkdir -p $OUT
PKG=$PWD/feature_base_pointcloud_registration_amd
for t in 8 16 24; do
  FBR_STAGE_THREADS=$t timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --latency 0 --ingest 3 --exact-line 0 --no-cpu-baseline --profile off > $OUT/ing_$t.json 2> $OUT/ing_$t.err || { tail $OUT/ing_$t.err; exit 11; }
  python3 -c "
import json; d=json.loads(open('$OUT/ing_$t.json').read().strip().splitlines()[-1]); i=d['ingest']
print('threads $t ingest', i['value'], i['h2d_GBps'], i['poses_equal_resident'])"
done
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
for r in 1 2; do for v in def store; do
  L=$PKG/libfbr_hip.so; [ $v = store ] && L=$PKG/libfbr_hip_projstore.so
  FBR_LIB=$L timeout -k 10 300 python3 $B > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 13; }
  python3 -c "
import json; d=json.loads(open('$OUT/${v}_$r.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$v $r', d['value'], d['ms_per_step'], 'project', k['project'], 'extract', k['extract'])"
done; done
