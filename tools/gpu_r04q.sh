#!/bin/bash
# wave-tile kNN (queued fallback) counters and batch time on C5 and C3, then the tile parity test
set -o pipefail
OUT=gpurun_out/r04q
mkdir -p $OUT
p() {  # "ENV=.. ..." CONFIG B
  env FBR_KNN_TILE_STATS=1 $1 timeout -k 10 300 python3 tools/tile_probe.py $2 $3 | tee -a $OUT/probe.txt || exit 31
}
p "FBR_KNN_TILE=0" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0 FBR_KNN_TILE_REACH=2" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=1 FBR_KNN_TILE_REACH=2" C5 4
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=0 FBR_KNN_TILE_ROUNDS=1 FBR_KNN_TILE_SPAN=64" C5 4
p "FBR_KNN_TILE=0" C3 32
p "FBR_KNN_TILE=1 FBR_KNN_TILE_CAP=1 FBR_KNN_TILE_CELL=0.25 FBR_KNN_TILE_REACH=2" C3 32
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "knn_tile" > $OUT/pytest_tile.txt 2>&1; tail -3 $OUT/pytest_tile.txt
