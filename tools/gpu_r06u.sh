set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06u
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "full_masks or ragged" > gpurun_out/r06u/pytest.txt 2>&1 || { tail -40 gpurun_out/r06u/pytest.txt; exit 10; }
tail -1 gpurun_out/r06u/pytest.txt
timeout -k 10 600 python3 bench.py > gpurun_out/r06u/bench.json 2> gpurun_out/r06u/bench.err || { tail gpurun_out/r06u/bench.err; exit 11; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06u/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step']); print('masks', d.get('feature_masks')); print('ingest', d['ingest']['value'], d['ingest']['h2d_GBps']); print('lat', d['latency']['ms_per_scan_p50'], d['latency']['ms_per_scan_p99']); print('parity', d['parity_vs_ref']); print('exact', {k: d['exact_voxel_order'].get(k) for k in ('value','pose_bit_equal')})"
