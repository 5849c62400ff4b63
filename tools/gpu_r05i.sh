#!/bin/bash
# Round 5, call i: features phase stamps in the batch mode (B = 64: one wave per ring).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p $OUT
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_stamps.so timeout -k 10 300 python3 tools/feat_stamps.py 64 > $OUT/feat_stamps.txt 2>&1; cat $OUT/feat_stamps.txt
