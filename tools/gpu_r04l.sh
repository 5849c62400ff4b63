#!/bin/bash
# C3 / C5 regression bisect (round-2 end .. round-3 builds vs HEAD) + k_features phase stamps
set -o pipefail
FBR_DIAG_LIB=$PWD/feature_base_pointcloud_registration_amd/libfbr_hip_diag.so timeout -k 10 300 python3 tools/feat_stamps.py 256 > gpurun_out/r04l_feat_stamps.txt 2>&1 || echo "stamps failed"
cat gpurun_out/r04l_feat_stamps.txt | head -20
bash tools/gpu_bisect.sh r04l r02end r03a r03b r03c
