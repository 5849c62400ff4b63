"""Synthetic scans, maps and registration jobs (ctypes front-end of csrc/fbr_synth.cpp).

Implements the input spec of SURVEY.md §8d / BASELINE.md: beam tables for VLP-16 (16 rows),
HDL-64 (64 rows, kitti2bag.py:242-243 elevation range), Ouster-128 and a dense 512-row sensor;
firing-order emission with azimuth jitter, 1 cm range noise, 5 % dropouts, 0.5 % sub-1 m returns;
ground-truth viewpoints near the origin of a procedural plaza and guesses perturbed by
U(+-0.3 m) / U(+-2 deg).  Everything is seeded and deterministic.
"""
import ctypes
import os

import numpy as np

from .fbr_types import IMU_SAMPLE, POINT_XYZI, POINT_XYZIRT, ptr

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "libfbr_synth.so")
        if not os.path.exists(path):
            raise RuntimeError("libfbr_synth.so missing: run __graft_entry__.build()")
        L = ctypes.CDLL(path)
        L.fbr_synth_scan.restype = ctypes.c_int64
        L.fbr_synth_scan.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_double), ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.fbr_synth_map.restype = ctypes.c_int
        L.fbr_synth_map.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double, ctypes.c_void_p,
                                    ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
                                    ctypes.POINTER(ctypes.c_int64)]
        _LIB = L
    return _LIB


SCENE_SEED = 7

# Config -> (N_SCAN, Horizon_SCAN, map radius, surf density /m^2, corner density /m)
CONFIGS = {
    "C1": (16, 1800, 45.0, 12.0, 12.0),
    "C2": (64, 1800, 45.0, 12.0, 12.0),     # ~100k-point local map (BASELINE configs[1])
    "C3": (128, 2048, 60.0, 100.0, 100.0),  # ~500k-point local map (configs[2])
    "C5": (512, 2048, 40.0, 600.0, 250.0),  # ~5M-point map inside the crop box (configs[4])
}
# Mapping leaf sizes (mappingCornerLeafSize, mappingSurfLeafSize) of the denser configs: with the
# params.yaml leaves (0.2 / 0.4) the start-up VoxelGrid (mapOptmization.h:251-257) caps a 60 x 60 m
# local map far below the 500k / 5M points BASELINE.json names, so these configs use finer leaves.
MAP_LEAVES = {"C3": (0.1, 0.2), "C5": (0.05, 0.05)}


def config_params(config, **overrides):
    """default_params for a config: its scan shape and its mapping leaf sizes."""
    from .fbr_types import default_params
    H, W = CONFIGS[config][:2]
    kw = {}
    if config in MAP_LEAVES:
        kw["mapping_corner_leaf_size"], kw["mapping_surf_leaf_size"] = MAP_LEAVES[config]
    kw.update(overrides)
    return default_params(H, W, **kw)


def scan(pose_world, n_scan, horizon_scan, seed, scene_seed=SCENE_SEED):
    """Ray-cast one scan at world pose [roll,pitch,yaw,x,y,z]; returns POINT_XYZIRT array."""
    out = np.zeros(n_scan * horizon_scan, dtype=POINT_XYZIRT)
    pose = (ctypes.c_double * 6)(*[float(v) for v in pose_world])
    n = lib().fbr_synth_scan(scene_seed, n_scan, horizon_scan, pose, seed, None, ptr(out))
    return out[:n].copy()


def prior_map(radius=45.0, surf_density=5.0, corner_density=5.0, seed=11,
              scene_seed=SCENE_SEED):
    """World-frame prior (corner, surf) feature maps of the scene (POINT_XYZI arrays)."""
    L = lib()
    nc, ns = ctypes.c_int64(), ctypes.c_int64()
    L.fbr_synth_map(scene_seed, seed, radius, surf_density, corner_density, None,
                    ctypes.byref(nc), None, ctypes.byref(ns))
    corner = np.zeros(nc.value, dtype=POINT_XYZI)
    surf = np.zeros(ns.value, dtype=POINT_XYZI)
    L.fbr_synth_map(scene_seed, seed, radius, surf_density, corner_density, ptr(corner),
                    ctypes.byref(nc), ptr(surf), ctypes.byref(ns))
    return corner, surf


def job(seed, max_offset=6.0):
    """(ground-truth pose, perturbed guess) for job `seed`, poses as [roll,pitch,yaw,x,y,z]."""
    rng = np.random.default_rng(seed)
    r = rng.uniform(0.0, max_offset)
    a = rng.uniform(-np.pi, np.pi)
    gt = np.array([rng.uniform(-0.01, 0.01), rng.uniform(-0.01, 0.01), rng.uniform(-np.pi, np.pi),
                   r * np.cos(a), r * np.sin(a), 1.8], dtype=np.float64)
    guess = gt.copy()
    guess[:3] += rng.uniform(-np.deg2rad(2.0), np.deg2rad(2.0), 3)
    guess[3:] += rng.uniform(-0.3, 0.3, 3)
    return gt, guess.astype(np.float32)


def trajectory(seed, n, step=0.4, dyaw=np.deg2rad(1.0)):
    """n consecutive ground-truth poses of a sensor driving forward (odometry-stream tests: each
    registration starts from the previous result, as cloudHandler's static pose chain does)."""
    gt0, _ = job(seed)
    out = []
    for k in range(n):
        p = gt0.copy()
        p[2] = gt0[2] + k * dyaw
        p[3] = gt0[3] + k * step * np.cos(gt0[2])
        p[4] = gt0[4] + k * step * np.sin(gt0[2])
        out.append(p)
    return out


def make_jobs(config, n_jobs, base_seed=1000, threads=16):
    """n_jobs independent (scan, guess, gt) registration jobs of a config (C4: seed 1000+j).  The
    ray casting runs in a thread pool (the C generator releases the GIL); results are identical to
    a serial loop."""
    import concurrent.futures
    n_scan, w, *_ = CONFIGS[config]

    def one(j):
        gt, guess = job(base_seed + j)
        return scan(gt, n_scan, w, seed=base_seed + j), guess, gt

    nth = max(1, min(threads, n_jobs, len(os.sched_getaffinity(0))))
    with concurrent.futures.ThreadPoolExecutor(nth) as ex:
        return list(ex.map(one, range(n_jobs)))


def config_map(config, seed=11):
    _, _, radius, sd, cd = CONFIGS[config]
    return prior_map(radius, sd, cd, seed=seed)


def imu_queue(t0, t1, rate=200.0, gyro=(0.04, -0.03, 0.5), rpy0=(0.01, -0.02, 0.3), seed=0):
    """IMU samples (IMU_SAMPLE, lidar frame) at `rate` Hz over [t0, t1]: angular velocity `gyro`
    rad/s plus N(0, 0.002) noise, orientation the integrated attitude from `rpy0` (x, y, z, w),
    gravity-only acceleration.  Input of fbr_imu_deskew_info (imuDeskewInfo's queue)."""
    rng = np.random.default_rng(seed)
    ts = np.arange(t0, t1 + 0.5 / rate, 1.0 / rate)
    q = np.zeros(len(ts), IMU_SAMPLE)
    q["stamp"] = ts
    q["angular_velocity"] = np.asarray(gyro) + rng.normal(0.0, 0.002, (len(ts), 3))
    q["linear_acceleration"] = (0.0, 0.0, 9.80511)
    rpy = np.asarray(rpy0) + np.outer(ts - ts[0], gyro)
    cr, sr = np.cos(rpy[:, 0] / 2), np.sin(rpy[:, 0] / 2)
    cp, sp = np.cos(rpy[:, 1] / 2), np.sin(rpy[:, 1] / 2)
    cy, sy = np.cos(rpy[:, 2] / 2), np.sin(rpy[:, 2] / 2)
    q["orientation"] = np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                                 cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy], axis=1)
    return q
