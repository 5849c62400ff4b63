#!/bin/bash
# wave-tile kNN counters and batch time per capacity / cell / reach / cluster rounds on C5 and C3
set -o pipefail
OUT=gpurun_out/r04q
mkdir -p $OUT
p() {  # "ENV=.. ..." CONFIG B
  env FBR_KNN_TILE_STATS=1 $1 timeout -k 10 300 python3 tools/tile_probe.py $2 $3 | tee -a $OUT/probe.txt || exit 31
}
p "FBR_KNN_TILE=0" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0 FBR_KNN_TILE_ROUNDS=1 FBR_KNN_TILE_SPAN=64" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=1" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0 FBR_KNN_TILE_SPAN=2 FBR_KNN_TILE_ROUNDS=8" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=1 FBR_KNN_TILE_REACH=2" C5 4
p "FBR_KNN_TILE=0" C3 32
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=1 FBR_KNN_TILE_CELL=0.25 FBR_KNN_TILE_REACH=2" C3 32
