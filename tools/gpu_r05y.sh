#!/bin/bash
# Round 5, call x: VoxelGrid split 8 by default -- VoxelGrid / stream tests; features phase stamps of
# a one-job launch (four waves per ring, the single-scan shape).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
true
true
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_stamps.so timeout -k 10 300 python3 tools/feat_stamps.py 4 > $OUT/feat_stamps_b1.txt 2>&1 || { cat $OUT/feat_stamps_b1.txt; exit 3; }
cat $OUT/feat_stamps_b1.txt
