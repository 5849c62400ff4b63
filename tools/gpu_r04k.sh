#!/bin/bash
# four-wave ring filter + branch-free fdlibm atanf / multiplied column rounding: parity, then the
# sequential per-kernel line, SQ counts and the overlapped line for FBR_VR_WAVE = 0 / 2
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 21; }
tail -2 $OUT/pytest.txt
run() {  # name, env, bench args
  local name=$1 e=$2; shift 2
  env $e timeout -k 10 300 python3 bench.py --latency 0 --ingest 0 --no-cpu-baseline --exact-line 0 "$@" > $OUT/$name.json 2>>$OUT/err || exit 22
  python3 - $OUT/$name.json "$name [$e]" <<'PY' | tee -a $OUT/summary.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = d["roofline"]["kernels"]
print(sys.argv[2], d["value"], d["ms_per_step"], " ".join(f"{k}={v['avg_launch_us']:.0f}us/{v['ms_per_step']:.2f}ms" for k, v in ks.items()))
PY
}
run seq_vr0 "FBR_NSUB=1 FBR_PIPE=0 FBR_VR_WAVE=0" --batch 256 --steps 5 --warmup 2 --profile all
run seq_vr2 "FBR_NSUB=1 FBR_PIPE=0 FBR_VR_WAVE=2" --batch 256 --steps 5 --warmup 2 --profile all
run b1024_vr0 "FBR_VR_WAVE=0" --batch 1024 --steps 10 --warmup 3 --profile off
run b1024_vr2 "FBR_VR_WAVE=2" --batch 1024 --steps 10 --warmup 3 --profile off
run b1024_vr0b "FBR_VR_WAVE=0" --batch 1024 --steps 10 --warmup 3 --profile off
run b1024_vr2b "FBR_VR_WAVE=2" --batch 1024 --steps 10 --warmup 3 --profile off
CMD="bench.py --batch 256 --steps 3 --warmup 1 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline --profile off"
FBR_VR_WAVE=2 FBR_NSUB=1 FBR_PIPE=0 timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/sq_vr2 -o b --output-format csv -- python3 $CMD > $OUT/sq_vr2.log 2>&1 || exit 31
python3 tools/valu_pmc.py $(find $OUT/sq_vr2 -name "*counter_collection.csv") C2 256 $OUT/valu_vr2.json | tee $OUT/valu_vr2.txt
