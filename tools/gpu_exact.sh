#!/bin/bash
# -m gpu suite, then bench lines with the exact VoxelGrid order (default, with the CPU parity
# block) and without it (FBR_VG_EXACT=0), sequential and overlapped.  usage: TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 21; }
tail -2 $OUT/pytest_gpu.log
B="timeout -k 10 400 python3 bench.py --latency 0 --ingest 0"
$B --steps 10 --warmup 3 > $OUT/bench_exact.json 2>>$OUT/err || exit 22
FBR_VG_EXACT=0 $B --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_noexact.json 2>>$OUT/err || exit 23
FBR_NSUB=1 $B --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/seq_exact.json 2>>$OUT/err || exit 24
FBR_VG_EXACT=0 FBR_NSUB=1 $B --batch 256 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/seq_noexact.json 2>>$OUT/err || exit 25
