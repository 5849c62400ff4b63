"""LIO-SAM keyframe local map: extractSurroundingKeyFrames -> extractNearby /
extractForLoopClosure -> extractCloud (mapOptmization.h:857-978) on the device, and
scan2MapOptimization against that map (no CropBox), checked against the oracle's restatement.

Parity bars:
  * cloudToExtract size, local-map sizes and voxel order: exact (the key-pose transforms are built
    with the host libm as in the reference and applied with the same float operations);
  * local-map centroids: |d| <= 2e-4 (PCL sums a voxel's points in unstable-sort order);
  * registered pose: within 1e-4 m / 1e-4 rad, equal iteration counts.
"""
import ctypes

import numpy as np
import pytest

import pyoracle as O
from feature_base_pointcloud_registration_amd import api, synth
from feature_base_pointcloud_registration_amd.fbr_types import (KEYPOSE, FbrKeyframeParams, POINT_XYZI,
                                                                default_params, keyframe_params)

POSE_TOL = 1e-4
MAP_ATOL = 2e-4


def test_keyframe_params_default_matches_params_yaml():
    p = FbrKeyframeParams()
    api.lib().fbr_keyframe_params_default(ctypes.byref(p))
    q = keyframe_params()
    for name, _ in FbrKeyframeParams._fields_:
        assert getattr(p, name) == getattr(q, name), name
    assert (p.search_radius, p.pose_density, p.loop_closure, p.submap_size) == (50.0, 2.0, 0, 25)


def make_keyframes(n, H=16, W=1800, seed=7, step=1.5):
    """n keyframes along a trajectory: GT key poses, the scans' DS'd corner/surf features (the
    laserCloud{Corner,Surf}LastDS that saveKeyFramesAndFactor stores)."""
    P = default_params(H, W)
    traj = synth.trajectory(seed, n + 1, step=step)
    poses = np.zeros(n, KEYPOSE)
    corners, surfs = [], []
    for k in range(n):
        gt = traj[k]
        f = O.Stream(P).features(synth.scan(gt, H, W, seed=100 + k))
        corners.append(O.voxel_grid(f["corner"], P.mapping_corner_leaf_size))
        surfs.append(O.voxel_grid(f["surf"], P.mapping_surf_leaf_size))
        poses[k] = (gt[3], gt[4], gt[5], k, gt[0], gt[1], gt[2], 0.0, 2.0 * k)
    return P, poses, corners, surfs, traj[n]


def test_oracle_keyframe_extraction_properties():
    P, poses, corners, surfs, _ = make_keyframes(6, step=3.0)
    kp = keyframe_params(loop_closure=1, submap_size=3)
    c, s, nf = O.kf_extract(P, poses, corners, surfs, kp, 12.0)
    assert nf == 4  # extractForLoopClosure: while size <= surroundingKeyframeSize (:863)
    # transformPointCloud of keyframes 5..2, then the mapping VoxelGrids
    ref_c = np.concatenate([_transform(corners[k], poses[k]) for k in (5, 4, 3, 2)])
    exp = O.voxel_grid(ref_c, P.mapping_corner_leaf_size)
    assert len(exp) == len(c) and np.array_equal(exp.view(np.uint8), c.view(np.uint8))
    kp = keyframe_params(search_radius=4.0)  # nearby: only keyframes within 4 m of the last one
    c2, s2, nf2 = O.kf_extract(P, poses, corners, surfs, kp, 10.5)
    assert 1 <= nf2 and len(c2) < len(c)


def _transform(cloud, pose):
    m = O.affine_from_pose(np.array([pose["roll"], pose["pitch"], pose["yaw"], pose["x"], pose["y"], pose["z"]],
                                    np.float32))
    out = cloud.copy()
    for r, k in enumerate("xyz"):
        out[k] = m[r, 0] * cloud["x"] + m[r, 1] * cloud["y"] + m[r, 2] * cloud["z"] + m[r, 3]
    return out


def _close_maps(a, b):
    assert len(a) == len(b)
    A, B = a.view(np.float32).reshape(-1, 4), b.view(np.float32).reshape(-1, 4)
    assert np.abs(A[:, :3] - B[:, :3]).max(initial=0) <= MAP_ATOL
    inv = np.float32(1.0)  # same voxel for every output point at the map leaves
    assert np.abs(A[:, 3] - B[:, 3]).max(initial=0) <= 1e-2 * inv


def _pose_close(p, q):
    p, q = np.asarray(p, np.float64), np.asarray(q, np.float64)
    assert np.abs(p[3:] - q[3:]).max() <= POSE_TOL, (p, q)
    assert np.abs(np.angle(np.exp(1j * (p[:3] - q[:3])))).max() <= POSE_TOL, (p, q)


@pytest.mark.gpu
@pytest.mark.parametrize("loop", [0, 1])
def test_keyframe_local_map_and_registration(loop):
    P, poses, corners, surfs, gt_next = make_keyframes(10)
    kp = keyframe_params(loop_closure=loop, submap_size=5, search_radius=12.0)
    stamp = float(poses["time"][-1]) + 1.0
    oc, os_, onf = O.kf_extract(P, poses, corners, surfs, kp, stamp)
    _, guess = synth.job(77)
    guess = np.asarray(gt_next, np.float32).copy()
    guess[:3] += np.float32([0.01, -0.01, 0.02])
    guess[3:] += np.float32([0.2, -0.15, 0.05])
    f = O.Stream(P).features(synth.scan(gt_next, 16, 1800, seed=999))
    po, so, _ = O.Map(P, oc, os_, raw=True).register(f["corner"], f["surf"], guess)
    with api.Context(P) as ctx:
        for k in range(len(poses)):
            pk = poses[k].copy()
            pk["intensity"] = -1.0  # ignored: the store sets the key index
            ctx.keyframes_add(pk, corners[k], surfs[k])
        assert ctx.keyframes_count() == len(poses)
        nc, ns, nf = ctx.extract_surrounding_keyframes(stamp, kp)
        assert (nc, ns, nf) == (len(oc), len(os_), onf)
        gc, gs = ctx.get_map()
        _close_maps(gc, oc)
        _close_maps(gs, os_)
        pg, sg = ctx.register(f["corner"], f["surf"], guess)
    assert sg["status"] == so["status"] == 0 and sg["iterations"] == so["iterations"]
    assert (sg["n_corner_map"], sg["n_surf_map"]) == (so["n_corner_map"], so["n_surf_map"]) == (len(oc), len(os_))
    _pose_close(pg, po)
    assert np.abs(pg[3:] - np.asarray(gt_next[3:], np.float32)).max() < 0.05


@pytest.mark.gpu
def test_keyframe_correct_poses_and_map_switch():
    """correctPoses rewrites key poses (fbr_keyframes_set_pose); fbr_set_map restores the prior map
    and its CropBox; with no keyframes the previous map is kept (:967-968)."""
    P, poses, corners, surfs, gt_next = make_keyframes(6)
    kp = keyframe_params()
    moved = poses.copy()
    moved["x"] += 0.05
    moved["yaw"] += 0.002
    stamp = float(poses["time"][-1]) + 0.5
    oc, os_, onf = O.kf_extract(P, moved, corners, surfs, kp, stamp)
    cmap, smap = synth.config_map("C1")
    with api.Context(P) as ctx:
        ctx.set_map(cmap, smap)
        assert ctx.extract_surrounding_keyframes(stamp, kp) == (0, 0, 0)  # no keyframe yet: prior map kept
        assert len(ctx.get_map()[1]) == len(O.Map(P, cmap, smap).arrays()[1])
        for k in range(len(poses)):
            ctx.keyframes_add(poses[k], corners[k], surfs[k])
        for k in range(len(poses)):
            ctx.keyframes_set_pose(k, moved[k])
        nc, ns, nf = ctx.extract_surrounding_keyframes(stamp, kp)
        assert (nc, ns, nf) == (len(oc), len(os_), onf)
        _close_maps(ctx.get_map()[0], oc)
        ctx.set_map(cmap, smap)  # back to the prior map (CropBox registration)
        f = O.Stream(P).features(synth.scan(gt_next, 16, 1800, seed=5))
        guess = np.asarray(gt_next, np.float32)
        pg, sg = ctx.register(f["corner"], f["surf"], guess)
        po, so, _ = O.Map(P, cmap, smap).register(f["corner"], f["surf"], guess)
        assert (sg["n_corner_map"], sg["n_surf_map"]) == (so["n_corner_map"], so["n_surf_map"])
        _pose_close(pg, po)
        ctx.keyframes_reset()
        assert ctx.keyframes_count() == 0
