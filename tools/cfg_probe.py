"""Diagnostic: one job of a config through the device path and the CPU oracle (sizes, times,
pose difference).  usage: cfg_probe.py CONFIG [jobs] [oracle_threads]"""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
import pyoracle as O  # noqa: E402

cfg = sys.argv[1]
nj = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 16
P = synth.config_params(cfg, max_batch=nj)
t = time.time()
cm, sm = synth.config_map(cfg)
jobs = synth.make_jobs(cfg, nj, base_seed=5000)
print(f"{cfg}: map raw {len(cm)}+{len(sm)}, scans {[len(j[0]) for j in jobs]}, gen {time.time() - t:.1f}s", flush=True)
with api.Context(P) as ctx:
    t = time.time()
    ctx.set_map(cm, sm)
    gc, gs = ctx.get_map()
    print(f"set_map {time.time() - t:.1f}s, DS map {len(gc)}+{len(gs)}", flush=True)
    ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
    ctx.batch_launch(); ctx.batch_wait()
    ctx.set_profiling(True)
    t = time.time()
    ctx.batch_launch(); ctx.batch_wait()
    dt = time.time() - t
    poses, st = ctx.batch_results()
    ks = {k: round(ctx.kernel_time(k)[0], 3) for k in ["project", "extract", "features", "voxel_ring", "concat",
                                                        "voxel_scan", "gn_knn", "gn_residual", "gn_solve"]}
    print(f"device batch {dt * 1e3:.1f} ms: {ks}", flush=True)
    for k in ["n_points", "n_corner", "n_surf", "n_corner_ds", "n_surf_ds", "n_corner_map", "n_surf_map", "iterations", "status"]:
        print(f"  {k}: {st[k].tolist()}")
if "--no-oracle" not in sys.argv:
    t = time.time()
    m = O.Map(P, cm, sm)
    print(f"oracle map {time.time() - t:.1f}s", flush=True)
    for j, (pts, guess, gt) in enumerate(jobs):
        t = time.time()
        po, so = O.Stream(P).process_scan(m, pts, 0.0, guess, n_threads=nth)
        d = np.abs(poses[j].astype(np.float64) - po)
        print(f"job {j}: oracle {time.time() - t:.1f}s iters {so['iterations']} vs {st['iterations'][j]}, "
              f"|dpose| {d.max():.2e}, |pose-gt| {np.abs(po[3:] - gt[3:]).max():.3f}", flush=True)
