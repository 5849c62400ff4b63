#!/bin/bash
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
for cfg in "128 3" "128 1" "128 6" "256 3" "1024 3"; do
  set -- $cfg
  FBR_NSUB=$2 timeout -k 10 200 python3 tools/batch_host.py $1 20 >> $OUT/host.txt 2>>$OUT/err || exit 21
  echo "nsub=$2 $(tail -1 $OUT/host.txt)"
done
timeout -k 10 900 python -u -m pytest tests/test_c4.py -m gpu -x -v --timeout 900 --timeout-method thread --durations=0 > $OUT/pytest_c4.txt 2>&1 || { tail -40 $OUT/pytest_c4.txt; exit 22; }
tail -8 $OUT/pytest_c4.txt
