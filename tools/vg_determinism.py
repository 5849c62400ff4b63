#!/usr/bin/env python3
"""Determinism probe for the device VoxelGrid paths (fbr_voxel_grid / fbr_set_map): the same cloud
filtered repeatedly, in one context and in fresh ones, must give bit-identical outputs.

usage: vg_determinism.py [REPS]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import default_params  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
corner, surf = synth.prior_map(seed=11)
P = default_params(16, 1800)


def digest(a):
    return (len(a), hash(np.ascontiguousarray(a).view(np.uint8).tobytes()))


for label, cloud, leaf in (("surf", surf, 0.4), ("corner", corner, 0.2)):
    seen = {}
    with api.Context(P) as ctx:
        for r in range(reps):
            seen.setdefault(digest(ctx.voxel_grid(cloud, leaf)), []).append(f"same-ctx {r}")
    for r in range(reps // 2):
        with api.Context(P) as ctx:
            seen.setdefault(digest(ctx.voxel_grid(cloud, leaf)), []).append(f"new-ctx {r}")
    print(f"voxel_grid {label} ({len(cloud)} pts): {len(seen)} distinct outputs:",
          {k[0]: len(v) for k, v in seen.items()}, flush=True)

seen = {}
for r in range(reps // 2):
    with api.Context(P) as a:
        a.set_map(corner, surf)
        c, s = a.get_map()
        seen.setdefault((digest(c), digest(s)), []).append(r)
print(f"set_map: {len(seen)} distinct outputs:", {(k[0][0], k[1][0]): len(v) for k, v in seen.items()}, flush=True)
