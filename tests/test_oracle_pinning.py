"""Pin the oracle and the device restatements against the reference's real third-party dependencies.

The reference is unbuildable here (no ROS/PCL/OpenCV/Eigen/FLANN) and has no golden vectors, but two
of its parity-critical dependencies ARE in this image and are exactly what the reference links on
its Ubuntu toolchains:
  * glibc atan2f   -- the column index of every point (imageProjection.cpp:605);
  * libstdc++ 11 std::sort -- the visit order of the feature picks (featureExtraction.h:203).
The oracle calls both directly; the kernels carry restatements (fbr_fdlibm.h, fbr_sort.h) that are
compiled for the host here and compared bit for bit.
"""
import ctypes
import ctypes.util

import numpy as np
import pytest

import pyoracle as O
from feature_base_pointcloud_registration_amd.fbr_types import ptr

libm = ctypes.CDLL(ctypes.util.find_library("m"))
libm.atan2f.restype = ctypes.c_float
libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]


def glibc_atan2f_vec(y, x):
    return np.array([libm.atan2f(float(a), float(b)) for a, b in zip(y, x)], np.float32)


def test_fdlibm_atan2f_port_matches_glibc_bitwise(probe_lib):
    rng = np.random.default_rng(12)
    n = 400_000
    scale = rng.choice([1e-30, 1e-6, 0.3, 1.0, 5.0, 100.0, 1e6, 1e30], size=(2, n))
    y = (rng.standard_normal(n) * scale[0]).astype(np.float32)
    x = (rng.standard_normal(n) * scale[1]).astype(np.float32)
    special = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 1e-45, 3.4e38], np.float32)
    yy, xx = np.meshgrid(special, special)
    y = np.concatenate([y, yy.ravel()]).astype(np.float32)
    x = np.concatenate([x, xx.ravel()]).astype(np.float32)
    out = np.zeros_like(y)
    probe_lib.probe_atan2f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64]
    probe_lib.probe_atan2f(ptr(y), ptr(x), ptr(out), len(y))
    # glibc reference for a subsample (ctypes per call is slow) plus every special pair
    idx = np.concatenate([rng.choice(n, 60_000, replace=False), np.arange(n, len(y))])
    ref = glibc_atan2f_vec(y[idx], x[idx])
    a, b = out[idx], ref
    same = (a.view(np.int32) == b.view(np.int32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), f"{(~same).sum()} mismatches"


def test_glibc_sincosf_port_matches_glibc(probe_lib):
    """fbr_sincosf.h (the device's sinf / cosf in pcl::getTransformation and LMOptimization,
    mapOptmization.h:444-448, 1259-1264) equals the host glibc bit for bit: exhaustively for every
    float below 8 in magnitude (all pose angles; both reduction paths up to 120 are sampled too),
    and on a 1/97 stride over the whole 32-bit range (large-argument reduction, inf, NaN)."""
    import os
    probe_lib.probe_sincosf_range.restype = ctypes.c_uint64
    probe_lib.probe_sincosf_range.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_int]
    th = min(8, os.cpu_count() or 1)
    eight = int(np.float32(8.0).view(np.uint32))
    assert probe_lib.probe_sincosf_range(0, eight, 1, th) == 0
    assert probe_lib.probe_sincosf_range(0x80000000, 0x80000000 + eight, 1, th) == 0
    assert probe_lib.probe_sincosf_range(0, 1 << 32, 97, th) == 0


def test_range_gate_without_square_root():
    """k_project tests range < 1.0 (imageProjection.cpp:618-621) on the squared sum: a correctly
    rounded float sqrt is below 1 exactly when its argument is, NaN and inf included."""
    lo, hi = np.float32(0.98).view(np.uint32), np.float32(1.02).view(np.uint32)
    s = np.arange(lo, hi, dtype=np.uint32).view(np.float32)
    s = np.concatenate([s, np.array([0.0, 1e-45, 1.0, np.inf, np.nan, 3.4e38], np.float32)])
    with np.errstate(invalid="ignore"):
        assert np.array_equal(np.sqrt(s) < np.float32(1.0), s < np.float32(1.0))


@pytest.mark.parametrize("nvals", [1, 2, 3, 7, 50, 10_000_000])
def test_sort_emulation_matches_libstdcxx(probe_lib, nvals):
    rng = np.random.default_rng(nvals)
    probe_lib.probe_sort.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    for trial in range(300):
        n = int(rng.integers(0, 700))
        v = rng.integers(0, nvals, n).astype(np.float32)
        if trial % 17 == 0 and n:
            v[rng.integers(0, n, max(1, n // 9))] = np.nan
        mine = np.zeros(n, np.int64)
        probe_lib.probe_sort(ptr(v), n, ptr(mine))
        ref = O.sort_smoothness(v)
        assert np.array_equal(mine, ref), (trial, n)


def test_oracle_projection_rejects_nonfinite_like_x86():
    """NaN x/y make the reference's double->int column conversion INT_MIN -> point skipped."""
    from feature_base_pointcloud_registration_amd.fbr_types import POINT_XYZIRT, default_params
    P = default_params(4, 360)
    pts = np.zeros(4, POINT_XYZIRT)
    pts["x"] = [np.nan, 5.0, 3.0, 2.0]
    pts["y"] = [1.0, np.nan, 4.0, 2.0]
    pts["z"] = [0.0, 0.0, 0.0, np.inf]
    pts["ring"] = [0, 1, 2, 3]
    pr = O.project(P, pts)
    assert len(pr["col_ind"]) == 2  # the finite point and the inf-range point (range < 1 is false)


# ---- the wave-parallel std::sort used by k_features.hip for segments with tied curvatures ----
def _lg(n):
    r = -1
    while n:
        n >>= 1
        r += 1
    return r


def _move_median_to_first(a, res, x, y, z):  # libstdc++ __move_median_to_first
    v = lambda i: a[i][0]  # noqa: E731
    if v(x) < v(y):
        if v(y) < v(z):
            a[res], a[y] = a[y], a[res]
        elif v(x) < v(z):
            a[res], a[z] = a[z], a[res]
        else:
            a[res], a[x] = a[x], a[res]
    elif v(x) < v(z):
        a[res], a[x] = a[x], a[res]
    elif v(y) < v(z):
        a[res], a[z] = a[z], a[res]
    else:
        a[res], a[y] = a[y], a[res]


def _closed_form_partition(a, lo, hi, p):
    """k_features.hip wave_partition: k-th left stopper <-> k-th right stopper while left < right;
    cut = min(g_K, r_{K-1})."""
    L = [i for i in range(lo, hi) if not (a[i][0] < p)]
    R = [i for i in range(hi - 1, lo - 1, -1) if not (p < a[i][0])]
    k1 = 0
    while k1 < min(len(L), len(R)) and L[k1] < R[k1]:
        k1 += 1
    for k in range(k1):
        a[L[k]], a[R[k]] = a[R[k]], a[L[k]]
    cut = L[k1] if k1 < len(L) else 1 << 30
    if k1 > 0:
        cut = min(cut, R[k1 - 1])
    return min(cut, hi)


def _wave_std_sort(vals):
    a = [(np.float32(v), i) for i, v in enumerate(vals)]
    stack = [(0, len(a), 2 * _lg(len(a)))]
    while stack:
        first, last, depth = stack.pop()
        while last - first > 16:
            assert depth > 0  # heap-sort fallback not exercised by these inputs
            depth -= 1
            _move_median_to_first(a, first, first + 1, first + (last - first) // 2, last - 1)
            cut = _closed_form_partition(a, first + 1, last, a[first][0])
            stack.append((cut, last, depth))
            last = cut
    order = sorted(range(len(a)), key=lambda t: (a[t][0], t))  # the stable final insertion pass
    return [a[t][1] for t in order]


def test_wave_parallel_std_sort_formula_matches_std_sort():
    """The closed-form partition + stable final pass equals libstdc++ std::sort (the oracle calls
    the real std::sort) on tie-heavy segments, the case k_features resolves wave-parallel."""
    rng = np.random.default_rng(1)
    for _ in range(400):
        n = int(rng.integers(1, 400))
        q = rng.choice([0.5, 0.1, 0.01, 1.0])
        v = (np.round(rng.uniform(0, 5, n) / q) * q).astype(np.float32)
        if rng.random() < 0.3:
            v[rng.random(n) < 0.5] = 0
        assert list(O.sort_smoothness(v)) == _wave_std_sort(v)
