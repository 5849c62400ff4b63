#!/bin/bash
# The ballot-leader in-place radix sort inside the product kernel (diagnostic build with
# -DFBR_VG_IP_LEADER, ablib/leader/libfbr_hip.so): the VoxelGrid parity tests and the bench's
# parity block against the default build.  usage: tools/gpu_leader.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
FBR_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_leader.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_voxel_order.py -m gpu -v --timeout 600 --timeout-method thread -k "voxel or registration_matches or batch or exact" > $OUT/pytest_leader.txt 2>&1
echo "leader pytest rc=$?"; tail -5 $OUT/pytest_leader.txt
