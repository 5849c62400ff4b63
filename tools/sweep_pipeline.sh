set -o pipefail
mkdir -p gpurun_out/r05as
for r in 1 2; do
  for v in "d3" "d4" "d2" "nsub2" "b2048"; do
    case $v in d3) A="";E="FBR_X=0";; d4) A="--pipeline-depth 4";E="FBR_X=0";; d2) A="--pipeline-depth 2";E="FBR_X=0";; nsub2) A="";E="FBR_NSUB=2";; b2048) A="--batch 2048";E="FBR_X=0";; esac
    env $E timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --latency 0 --ingest 0 --exact-line 0 --no-cpu-baseline $A > gpurun_out/r05as/${v}_$r.json 2>/dev/null || exit 3
    python3 -c "import json; d=json.loads(open('gpurun_out/r05as/${v}_$r.json').read().strip().splitlines()[-1]); print('$v r$r', d['value'], d['ms_per_step'])"
  done
done
