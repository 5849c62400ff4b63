#!/usr/bin/env python3
"""CPU model: how many Gauss-Newton kNN searches (iteration >= 1) could be skipped as provably
unchanged.  A query that moved by delta since the previous iteration keeps its 5 nearest
neighbours, in the same order, if the previous distances d1 < ... < d6 (d6: the 6th neighbour)
have every consecutive gap above 2 * delta (no point can cross another) and d5 + delta < 1 (the
correspondence gate).  For C2 jobs, the oracle's per-iteration poses, the mapping-DS queries, and
delta = the exact displacement of each query (a bound on the device would be larger).
usage: knn_skip_model.py [jobs]
"""
import os
import sys

import numpy as np
from scipy.spatial import cKDTree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle as O  # noqa: E402
from feature_base_pointcloud_registration_amd import synth  # noqa: E402


def xform(pose, q):
    T = O.affine_from_pose(np.asarray(pose, np.float32)).astype(np.float64)
    return q @ T[:3, :3].T + T[:3, 3]


def main():
    nj = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    P = synth.config_params("C2")
    cmap, smap = synth.config_map("C2")
    omap = O.Map(P, cmap, smap)
    mc, ms = omap.arrays()
    trees = {"corner": cKDTree(np.stack([mc["x"], mc["y"], mc["z"]], 1).astype(np.float64)),
             "surf": cKDTree(np.stack([ms["x"], ms["y"], ms["z"]], 1).astype(np.float64))}
    per_it = {}
    for pts, guess, _ in synth.make_jobs("C2", nj, base_seed=1000):
        f = O.Stream(P).features(pts)
        _, st, trace = omap.register(f["corner"], f["surf"], guess)
        poses = [np.asarray(guess, np.float32)] + [trace[i] for i in range(len(trace) - 1)]
        for name, cloud, leaf in (("corner", f["corner"], P.mapping_corner_leaf_size),
                                  ("surf", f["surf"], P.mapping_surf_leaf_size)):
            ds = O.voxel_grid(cloud, leaf)
            q = np.stack([ds["x"], ds["y"], ds["z"]], 1).astype(np.float64)
            for i in range(1, len(poses)):
                xp, xc = xform(poses[i - 1], q), xform(poses[i], q)
                delta = np.linalg.norm(xc - xp, axis=1)
                d, _ = trees[name].query(xp, k=6)
                gaps = np.diff(d, axis=1).min(axis=1)
                skip = (gaps > 2 * delta + 1e-6) & (d[:, 4] + delta < 1.0)
                a = per_it.setdefault(i, [0, 0, []])
                a[0] += int(skip.sum())
                a[1] += len(q)
                a[2].append(np.median(delta))
    for i, (s, n, md) in sorted(per_it.items()):
        print(f"iteration {i}: skippable {s / n:.3f} of {n} queries (median displacement {np.median(md) * 1000:.2f} mm)")


if __name__ == "__main__":
    main()
