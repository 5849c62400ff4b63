#!/bin/bash
# Round 5, call x: VoxelGrid split 8 by default -- VoxelGrid / stream tests; features phase stamps of
# a one-job launch (four waves per ring, the single-scan shape).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05x
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_voxel_order.py -m gpu -x -v --timeout 300 --timeout-method thread -k "voxel or split or stream or process_scan" > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 10; }
tail -1 $OUT/pytest.txt
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_stamps.so timeout -k 10 300 python3 tools/feat_stamps.py 1 > $OUT/feat_stamps_b1.txt 2>&1 || { cat $OUT/feat_stamps_b1.txt; exit 3; }
cat $OUT/feat_stamps_b1.txt
