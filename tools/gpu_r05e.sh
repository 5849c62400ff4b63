#!/bin/bash
# Round 5, call e: batch surf walk resolved within reach of each segment's end (default) against the
# whole walk (FBR_FEAT_SURF_WINDOW=0): equivalence test + registration tests, interleaved C2 A/B;
# C3 B=256 scheduling sweep (sub-batches, pipeline depth, GN tail).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_c4.py -m gpu -x -v --timeout 600 --timeout-method thread -k "surf_walk_window or registration or batch or c3 or c5 or c4_full or golden or stream or features" > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 10; }
tail -2 $OUT/pytest.txt
Q="--steps 10 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2 3; do for sw in 1 0; do
  FBR_FEAT_SURF_WINDOW=$sw timeout -k 10 300 python3 bench.py $Q > $OUT/ab_sw${sw}_$rep.json 2>/dev/null || exit 16
  python3 -c "
import json; d=json.loads(open('$OUT/ab_sw${sw}_$rep.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']
print('SW $sw rep $rep', d['value'], 'features', k['features'], 'gn_knn', k['gn_knn'])"
done; done
C3="--config C3 --batch 256 --steps 6 --warmup 2 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
for rep in 1 2; do for v in base nsub2 d2 tail0 d2nsub2; do
  case $v in base) E=""; A="";; nsub2) E="FBR_NSUB=2"; A="";; d2) E=""; A="--pipeline-depth 2";; tail0) E="FBR_GN_TAIL=0"; A="";; d2nsub2) E="FBR_NSUB=2"; A="--pipeline-depth 2";; esac
  env $E timeout -k 10 300 python3 bench.py $C3 $A > $OUT/c3_${v}_$rep.json 2>/dev/null || exit 17
  python3 -c "import json; d=json.loads(open('$OUT/c3_${v}_$rep.json').read().strip().splitlines()[-1]); print('C3 $v rep $rep', d['value'])"
done; done
