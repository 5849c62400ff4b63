set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 21; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 22
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit 23
for T in 1 0; do
FBR_KNN_TILE=$T timeout -k 10 300 python3 bench.py --config C5 --batch 16 --steps 5 --warmup 2 --latency 0 --ingest 0 --no-cpu-baseline > $OUT/bench_c5_tile$T.json 2>> $OUT/bench.err || exit 24
done
echo done
