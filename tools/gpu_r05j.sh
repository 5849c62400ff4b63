#!/bin/bash
# Round 5, call j: features phase stamps in the batch mode (B = 64: one wave per ring), and the
# per-kernel breakdown of the default bench at HEAD.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_stamps.so timeout -k 10 300 python3 tools/feat_stamps.py 64 > $OUT/feat_stamps.txt 2>&1 || { cat $OUT/feat_stamps.txt; exit 3; }
cat $OUT/feat_stamps.txt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 4
python3 -c "
import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['kernel_ms_per_step'])"
