#!/bin/bash
# Round-6 first look: default C2 B=1024 line (x2) interleaved with FBR_GN_FUSED=1 (x2), then the
# exact_voxel_order=1 main line at B=1024 with its per-kernel times.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06a; mkdir -p $OUT
B="bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline"
summ() { python3 -c "
import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('$2', d['value'], d['ms_per_step'], {a: round(b,3) for a,b in k.items()})"; }
for r in 1 2; do
  timeout -k 10 300 python3 $B > $OUT/def_$r.json 2> $OUT/def_$r.err || { tail $OUT/def_$r.err; exit 11; }
  summ $OUT/def_$r.json "default $r"
  FBR_GN_FUSED=1 timeout -k 10 300 python3 $B > $OUT/fused_$r.json 2> $OUT/fused_$r.err || { tail $OUT/fused_$r.err; exit 12; }
  summ $OUT/fused_$r.json "fused $r"
done
timeout -k 10 300 python3 $B --exact-voxel-order 1 > $OUT/exact.json 2> $OUT/exact.err || { tail $OUT/exact.err; exit 13; }
summ $OUT/exact.json "exact B1024"
