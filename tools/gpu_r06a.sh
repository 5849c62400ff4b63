#!/bin/bash
# Round-6 first look: the GPU suite, then the default C2 B=1024 line (x2) interleaved with
# FBR_GN_FUSED=1 (x2) and the round-5 library (prev), then the exact_voxel_order=1 main line at
# B=1024 with its per-kernel times.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
summ() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items()})"; }
PKG=$PWD/feature_base_pointcloud_registration_amd
for r in 1 2; do
  timeout -k 10 300 python3 $B > $OUT/def_$r.json 2> $OUT/def_$r.err || { tail $OUT/def_$r.err; exit 11; }
  summ $OUT/def_$r.json "default $r"
  FBR_GN_FUSED=1 timeout -k 10 300 python3 $B > $OUT/fused_$r.json 2> $OUT/fused_$r.err || { tail $OUT/fused_$r.err; exit 12; }
  summ $OUT/fused_$r.json "fused $r"
  FBR_LIB=$PKG/libfbr_hip_prev.so timeout -k 10 300 python3 $B > $OUT/prev_$r.json 2> $OUT/prev_$r.err || { tail $OUT/prev_$r.err; exit 13; }
  summ $OUT/prev_$r.json "prev(r05) $r"
done
timeout -k 10 300 python3 $B --exact-voxel-order 1 > $OUT/exact.json 2> $OUT/exact.err || { tail $OUT/exact.err; exit 14; }
summ $OUT/exact.json "exact B1024"
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 100 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/lat.json 2> $OUT/lat.err || { tail $OUT/lat.err; exit 15; }
python3 -c "
import json; d=json.loads(open('$OUT/lat.json').read().strip().splitlines()[-1]); print('latency', d['value'], d['latency'])"
