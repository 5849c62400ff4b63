#!/bin/bash
# Round 5, call d: iteration-0 kNN through the flat queue with a seeded bound (FBR_KNN_SEED0=1):
# parity (registration tests with the knob on), interleaved C2 / C3 A/B, and a per-kernel trace of
# C3 B=256 for the round-2 build 69dd8f7 and HEAD (where C3 lost its ~2 %).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p $OUT
FBR_KNN_SEED0=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 600 --timeout-method thread -k "registration or batch or c3 or c5 or c4_full or golden or stream" > $OUT/pytest_seed0.txt 2>&1 || { tail -30 $OUT/pytest_seed0.txt; exit 10; }
tail -2 $OUT/pytest_seed0.txt
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2 3; do for s0 in 0 1; do
  FBR_KNN_SEED0=$s0 timeout -k 10 300 python3 bench.py $Q > $OUT/ab_seed${s0}_$rep.json 2>/dev/null || exit 16
  FBR_KNN_SEED0=$s0 timeout -k 10 300 python3 bench.py $Q --config C3 --batch 256 --steps 5 > $OUT/ab_c3_seed${s0}_$rep.json 2>/dev/null || exit 17
  python3 -c "
import json
for f in ('ab_seed${s0}_$rep', 'ab_c3_seed${s0}_$rep'):
    d=json.loads(open('$OUT/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['value'], d['kernel_ms_per_step']['gn_knn'])"
done; done
export TMPDIR=/tmp
(cd abwt/r02_69dd8f7 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../../$OUT/tr_old -o c3 --output-format csv -- python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --no-cpu-baseline --profile off > ../../$OUT/tr_old.log 2>&1) || exit 18
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/tr_head -o c3 --output-format csv -- python3 bench.py --config C3 --batch 256 --steps 5 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off > $OUT/tr_head.log 2>&1 || exit 19
for t in old head; do echo "== $t"; f=$(find $OUT/tr_$t -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]: print(f\"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} {r['Name'][:90]}\")"; done
# single-scan latency knobs (host scan in, pose out; 100 pose-chained C2 scans each), interleaved
L="--steps 1 --warmup 1 --batch 16 --latency 100 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2; do for v in base large fused seed0; do
  case $v in base) E="";; large) E="FBR_VG_LARGE_MIN=2048";; fused) E="FBR_GN_FUSED=1";; seed0) E="FBR_KNN_SEED0=1";; esac
  env $E timeout -k 10 300 python3 bench.py $L > $OUT/lat_${v}_$rep.json 2>/dev/null || exit 20
  python3 -c "import json; d=json.loads(open('$OUT/lat_${v}_$rep.json').read().strip().splitlines()[-1])['latency']; print('LAT $v rep $rep', d['ms_per_scan_p50'], d['ms_per_scan_p99'], d['chain_max_abs_pose_diff_vs_oracle'] if 'chain_max_abs_pose_diff_vs_oracle' in d else '')"
done; done
