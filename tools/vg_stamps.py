#!/usr/bin/env python3
"""Diagnostic: phase times of k_voxel_grid_ip's first workgroup (the surf mapping-DS cloud) in the
single-scan chain, from a FBR_VG_STAMPS build (s_memtime ticks: grid set-up, keys, sort, emit)."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import build  # noqa: E402

diag = os.environ.get("FBR_DIAG_LIB") or build.build_hip(defines=("FBR_VG_STAMPS",), name="libfbr_hip_vgst.so")
os.environ["FBR_LIB"] = diag
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402

P = synth.config_params("C2", max_batch=1)
cm, sm = synth.config_map("C2")
traj = synth.trajectory(7, 24)
H, W = synth.CONFIGS["C2"][:2]
L = api.lib()
L.fbr_diag_vg_stamps.argtypes = [ctypes.c_void_p]
rows = []
with api.Context(P) as c:
    c.set_map(cm, sm)
    _, pose = synth.job(7)
    for k, p in enumerate(traj):
        pose, st = c.process_scan(synth.scan(p, H, W, seed=500 + k), 0.2 * k, pose)
        t = np.zeros(8, np.uint64)
        L.fbr_diag_vg_stamps(t.ctypes.data)
        if k >= 4:
            rows.append(np.diff(t[:5].astype(np.int64)))
d = np.median(np.array(rows), axis=0)
print("k_voxel_grid_ip workgroup 0 (surf cloud), median s_memtime ticks per phase:",
      dict(zip(["minmax+grid", "keys", "sort", "emit"], d.tolist())), "total", int(d.sum()))
