"""Measurement of the LIO-SAM keyframe local-map path: per scan,
extractSurroundingKeyFrames on the device (selection on the host, transform + VoxelGrid + grid
build on the device) followed by a single-scan registration against the local map; the oracle's
restatement of the same two steps timed beside it.  usage: kf_bench.py [n_keyframes] [reps]"""
import json
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import KEYPOSE, default_params, keyframe_params  # noqa: E402
import pyoracle as O  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 40
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
H, W = 64, 1800
P = default_params(H, W)
traj = synth.trajectory(3, nk + 1, step=1.0)
poses = np.zeros(nk, KEYPOSE)
corners, surfs = [], []
for k in range(nk):
    f = O.Stream(P).features(synth.scan(traj[k], H, W, seed=200 + k))
    corners.append(O.voxel_grid(f["corner"], P.mapping_corner_leaf_size))
    surfs.append(O.voxel_grid(f["surf"], P.mapping_surf_leaf_size))
    g = traj[k]
    poses[k] = (g[3], g[4], g[5], k, g[0], g[1], g[2], 0.0, 1.0 * k)
kp = keyframe_params()
stamp = float(poses["time"][-1]) + 0.5
f = O.Stream(P).features(synth.scan(traj[nk], H, W, seed=999))
guess = np.asarray(traj[nk], np.float32)
with api.Context(P) as ctx:
    for k in range(nk):
        ctx.keyframes_add(poses[k], corners[k], surfs[k])
    ctx.extract_surrounding_keyframes(stamp, kp)
    ctx.register(f["corner"], f["surf"], guess)
    t0 = time.perf_counter()
    for _ in range(reps):
        nc, ns, nf = ctx.extract_surrounding_keyframes(stamp, kp)
    t_ext = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        pg, sg = ctx.register(f["corner"], f["surf"], guess)
    t_reg = (time.perf_counter() - t0) / reps
t0 = time.perf_counter()
oc, os_, onf = O.kf_extract(P, poses, corners, surfs, kp, stamp)
o_ext = time.perf_counter() - t0
t0 = time.perf_counter()
po, so, _ = O.Map(P, oc, os_, raw=True).register(f["corner"], f["surf"], guess)
o_reg = time.perf_counter() - t0
print(json.dumps({"keyframes": nk, "frames_extracted": nf, "local_map": [nc, ns],
                  "device_extract_ms": round(t_ext * 1e3, 3), "device_register_ms": round(t_reg * 1e3, 3),
                  "oracle_extract_ms": round(o_ext * 1e3, 3), "oracle_register_ms_4threads": round(o_reg * 1e3, 3),
                  "pose_max_abs_diff": float(np.abs(pg.astype(np.float64) - po).max()),
                  "iterations": [int(sg["iterations"]), int(so["iterations"])]}))
