#!/usr/bin/env python3
"""Order-dependence probe: run the GPU parity tests that precede test_registration_golden_fixture
one at a time in one process and, after each, the golden registration (pose error printed), to find
which earlier call leaves state that changes a later context's registration.

usage: order_probe.py
"""
import os
import sys
import traceback

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import test_gpu_parity as T  # noqa: E402
from feature_base_pointcloud_registration_amd import api  # noqa: E402


def golden():
    d = np.load(os.path.join(T.G, "reg_small.npz"))
    P = T.default_params(16, 900)
    with api.Context(P) as ctx:
        ctx.set_map(d["corner_map"], d["surf_map"])
        pose, st, trace = ctx.register(d["corner"], d["surf"], d["guess"], trace=True)
    err = np.abs(np.asarray(pose, np.float64)[3:] - d["pose"][3:]).max()
    terr = np.abs(trace - d["trace"]).max(axis=1)
    first_bad = int(np.argmax(terr > 1e-4)) if (terr > 1e-4).any() else -1
    return err, st["iterations"], st["n_sel"], first_bad


steps = [
    ("start", None),
    ("device_math", T.test_device_math_is_bit_exact),
    ("sincosf", T.test_device_sincosf_matches_glibc),
    ("eigen6", T.test_degeneracy_eigen6_wave_matches_single_lane_and_oracle),
    ("proj C1-1", lambda: T.test_projection_bit_exact("C1", 1)),
    ("proj C2-3", lambda: T.test_projection_bit_exact("C2", 3)),
    ("proj C3-5", lambda: T.test_projection_bit_exact("C3", 5)),
    ("proj edge", T.test_projection_edge_cases),
    ("feat golden", T.test_features_golden_fixture_stream_mode),
    ("feat C1", lambda: T.test_features_bit_exact_stream("C1")),
    ("feat C2", lambda: T.test_features_bit_exact_stream("C2")),
    ("feat C3", lambda: T.test_features_bit_exact_stream("C3")),
    ("feat ties", T.test_features_with_curvature_ties),
    ("voxel golden", T.test_voxel_grid_golden_and_oracle),
]
for name, fn in steps:
    if fn is not None:
        try:
            fn()
        except Exception:
            traceback.print_exc()
            print(f"{name}: test raised", flush=True)
    for rep in range(2):
        err, iters, nsel, fb = golden()
        print(f"after {name:14s} rep {rep}: pose err {err:.3e} iterations {iters} n_sel {nsel} first bad trace row {fb}",
              flush=True)
