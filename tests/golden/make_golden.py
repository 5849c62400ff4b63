#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the CPU oracle (oracle/fbr_oracle.cpp).

The reference (/root/reference) ships no tests, fixtures or golden vectors and cannot be built in
this image, so these fixtures are produced by the oracle's restatement of the
reference path; they freeze its outputs (regression pinning) and give the GPU tests committed
expected values.  Inputs are stored alongside the outputs so the fixtures do not depend on the
synthetic generator.

Fixtures:
  vlp16_w900.npz  one 16x900 scan (seed 1) -> cloud_info projection fields, feature label mask,
                  corner / surface clouds; a second scan (seed 2) for stream-mode state carry-over
  reg_small.npz   a small prior map (~30k pts) + the seed-1 features -> registered pose, stats,
                  per-iteration pose trace
  voxel.npz       VoxelGrid inputs / outputs at leaves 0.2 and 0.4 plus the int32-overflow case
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

from feature_base_pointcloud_registration_amd import synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import (POINT_XYZI,  # noqa: E402
                                                                default_params)
import pyoracle as O  # noqa: E402

H, W = 16, 900


def scans():
    gt1, g1 = synth.job(1)
    gt2, g2 = synth.job(2)
    return (synth.scan(gt1, H, W, seed=1), gt1, g1), (synth.scan(gt2, H, W, seed=2), gt2, g2)


def main():
    P = default_params(H, W)
    (s1, gt1, g1), (s2, gt2, g2) = scans()
    pr = O.project(P, s1)
    st = O.Stream(P)
    f1 = st.features(s1)
    f2 = st.features(s2)  # stream mode: stale state of scan 1 carried into scan 2
    np.savez_compressed(
        os.path.join(HERE, "vlp16_w900.npz"), scan1=s1, scan2=s2, gt1=gt1, guess1=g1, gt2=gt2, guess2=g2,
        start_ring=pr["start_ring"], end_ring=pr["end_ring"], col_ind=pr["col_ind"], range=pr["range"],
        cloud=pr["cloud"], label1=f1["label"], corner1=f1["corner"], surf1=f1["surf"], label2=f2["label"],
        corner2=f2["corner"], surf2=f2["surf"])

    corner_map, surf_map = synth.prior_map(radius=20.0, surf_density=2.5, corner_density=5.0, seed=5)
    m = O.Map(P, corner_map, surf_map)
    mc, ms = m.arrays()
    pose, stats, trace = m.register(f1["corner"], f1["surf"], g1)
    np.savez_compressed(
        os.path.join(HERE, "reg_small.npz"), corner_map=corner_map, surf_map=surf_map,
        corner=f1["corner"], surf=f1["surf"], guess=g1, gt=gt1, pose=pose,
        stats=np.array([stats[k] for k in sorted(stats)], np.int32),
        stats_keys=np.array(sorted(stats)), trace=trace)

    rng = np.random.default_rng(3)
    pts = np.zeros(6000, POINT_XYZI)
    pts["x"] = rng.uniform(-20, 20, 6000)
    pts["y"] = rng.uniform(-20, 20, 6000)
    pts["z"] = rng.uniform(-2, 5, 6000)
    pts["intensity"] = rng.uniform(0, 255, 6000)
    clustered = pts.copy()  # many points per voxel: exercises the centroid sums
    clustered["x"] = np.round(clustered["x"] / 0.5) * 0.5 + rng.uniform(-0.05, 0.05, 6000)
    clustered["y"] = np.round(clustered["y"] / 0.5) * 0.5 + rng.uniform(-0.05, 0.05, 6000)
    huge = pts[:50].copy()
    huge["x"][0] = -5e6
    huge["x"][1] = 5e6
    np.savez_compressed(
        os.path.join(HERE, "voxel.npz"), pts=pts, clustered=clustered, huge=huge,
        out_02=O.voxel_grid(pts, 0.2), out_04=O.voxel_grid(pts, 0.4), clustered_04=O.voxel_grid(clustered, 0.4),
        huge_001=O.voxel_grid(huge, 0.01))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
