#!/usr/bin/env python3
"""Diagnostic: device fbr_voxel_grid vs the oracle (std::sort order) on random clouds of several
sizes (each VoxelGrid kernel path); prints voxel counts and bit-equality per size."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "oracle"))
import pyoracle as O  # noqa: E402
from feature_base_pointcloud_registration_amd import api  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import POINT_XYZI, default_params  # noqa: E402

rng = np.random.default_rng(21)
with api.Context(default_params(16, 900)) as ctx:
    for n in [int(x) for x in os.environ.get("SIZES", "3000,6000,18432,18433,30000,40000").split(",")]:
        pts = np.zeros(n, POINT_XYZI)
        pts["x"], pts["y"] = rng.uniform(-30, 30, n), rng.uniform(-30, 30, n)
        pts["z"] = rng.normal(0, 0.4, n) + (rng.random(n) < 0.3) * rng.uniform(0, 6, n)
        pts["intensity"] = rng.uniform(0, 255, n)
        g, o = ctx.voxel_grid(pts, 0.4), O.voxel_grid(pts, 0.4)
        eq = len(g) == len(o) and g.tobytes() == o.tobytes()
        print(f"n={n} device={len(g)} oracle={len(o)} bit_equal={eq}", flush=True)
