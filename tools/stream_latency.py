"""Stream-mode latency: one scan at a time through fbr_process_scan (the reference's operating mode,
cloudHandler -> registration per scan), per-scan wall time and per-kernel device time, with the
CPU oracle's process_scan beside it.  usage: stream_latency.py [config] [scans]"""
import json
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
import pyoracle as O  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
P = synth.config_params(cfg)
H, W = P.n_scan, P.horizon_scan
cm, sm = synth.config_map(cfg)
traj = synth.trajectory(11, n + 3)
scans = [synth.scan(g, H, W, seed=300 + k) for k, g in enumerate(traj)]
kernels = ["project", "extract", "features", "voxel_ring", "concat", "voxel_scan", "gn_init", "crop", "gn_knn",
           "gn_residual", "gn_solve", "gn_finalize"]
with api.Context(P) as ctx:
    ctx.set_map(cm, sm)
    pose = np.asarray(traj[0], np.float32)
    for k in range(3):  # warm-up
        pose, _ = ctx.process_scan(scans[k], 0.2 * k, pose)
    ctx.set_profiling(True)
    times = []
    for k in range(3, n + 3):
        t0 = time.perf_counter()
        pose, st = ctx.process_scan(scans[k], 0.2 * k, pose)
        times.append(time.perf_counter() - t0)
    ks = {name: round(ctx.kernel_time(name)[0] / n, 4) for name in kernels}
m = O.Map(P, cm, sm)
s = O.Stream(P)
po = np.asarray(traj[0], np.float32)
t0 = time.perf_counter()
for k in range(min(n + 3, 8)):
    po, _ = s.process_scan(m, scans[k], 0.2 * k, po, n_threads=P.number_of_cores)
cpu = (time.perf_counter() - t0) / min(n + 3, 8)
print(json.dumps({"config": cfg, "scans": n, "gpu_ms_per_scan_median": round(1e3 * float(np.median(times)), 3),
                  "gpu_ms_per_scan_p90": round(1e3 * float(np.percentile(times, 90)), 3),
                  "kernel_ms_per_scan": ks, "cpu_oracle_ms_per_scan_4threads": round(1e3 * cpu, 2)}))
