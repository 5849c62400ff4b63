"""Python front-end of libfbr_hip.so (the extern "C" boundary of include/fbr.h).

The classes mirror the reference's per-scan operator interface so that tests read like the
reference's own call sites:

  ImageProjection.projectPointCloud/cloudExtraction  -> Context.project()      imageProjection.cpp:583-670
  FeatureExtraction.featureExtra                     -> Context.extract_features() featureExtraction.h:79
  mapOptimization.registration                       -> Context.register()     mapOptmization.h:263
  cloudHandler (projection -> features -> registration) -> Context.process_scan()  imageProjection.cpp:182

There is no CPU fallback: if the HIP library or a GPU is missing every call raises.
"""
import ctypes
import os

import numpy as np

from .fbr_types import (DESKEW_TABLE, IMU_SAMPLE, KEYPOSE, PF_FLOAT32, POINT_XYZI, POINT_XYZIRT, REG_STATS, FbrParams,
                        FbrRegStats, PointCloud2, default_params, ptr)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_VP = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32

EXPORTED_SYMBOLS = [
    "fbr_params_default", "fbr_strerror", "fbr_abi_version", "fbr_device_count", "fbr_create",
    "fbr_destroy", "fbr_set_map", "fbr_get_map", "fbr_project", "fbr_extract_features",
    "fbr_register", "fbr_register_trace", "fbr_process_scan", "fbr_reset_stream",
    "fbr_process_batch", "fbr_ingest_bytes", "fbr_debug_counters", "fbr_map_grid_info", "fbr_batch_stage", "fbr_batch_launch", "fbr_batch_wait",
    "fbr_batch_flush", "fbr_batch_export_ready", "fbr_batch_results", "fbr_batch_set_full_masks", "fbr_batch_labels", "fbr_batch_export", "fbr_batch_bytes", "fbr_set_profiling", "fbr_set_profiling_kernels", "fbr_kernel_time", "fbr_stream",
    "fbr_voxel_grid", "fbr_affine_from_pose", "fbr_pose_from_affine", "fbr_selftest_math", "fbr_selftest_eigen6", "fbr_selftest_eig_certified", "fbr_selftest_voxel_order", "fbr_selftest_radix_sort",
    "fbr_load_map", "fbr_pcd_read", "fbr_pcd_write_ascii", "fbr_pcd_write_binary",
    "fbr_msg_to_points", "fbr_points_to_msg_data", "fbr_project_msg", "fbr_process_msg",
    "fbr_imu_convert", "fbr_imu_deskew_info", "fbr_set_deskew", "fbr_stream_copy_bandwidth", "fbr_valu_peak",
    "fbr_keyframe_params_default", "fbr_keyframes_add", "fbr_keyframes_set_pose", "fbr_keyframes_count",
    "fbr_keyframes_reset", "fbr_extract_surrounding_keyframes",
    "fbr_comm_unique_id", "fbr_comm_create", "fbr_comm_create_local", "fbr_comm_destroy", "fbr_batch_allgather",
]


class FbrError(RuntimeError):
    def __init__(self, status, where=""):
        self.status = status
        super().__init__(f"{where}: {strerror(status)} ({status})")


def lib_path():
    # FBR_LIB selects a diagnostic build (tools/); the default is the shipped library
    return os.environ.get("FBR_LIB") or os.path.join(_HERE, "libfbr_hip.so")


def lib():
    """Load the HIP library (raises if it was not built: no silent fallback)."""
    global _LIB
    if _LIB is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: the HIP extension is not built "
                               "(run __graft_entry__.build())")
        L = ctypes.CDLL(path)
        sig = {
            "fbr_params_default": (None, [_VP]),
            "fbr_strerror": (ctypes.c_char_p, [ctypes.c_int]),
            "fbr_abi_version": (ctypes.c_int, []),
            "fbr_device_count": (ctypes.c_int, [_VP]),
            "fbr_create": (ctypes.c_int, [_VP, _VP, ctypes.c_int]),
            "fbr_destroy": (ctypes.c_int, [_VP]),
            "fbr_set_map": (ctypes.c_int, [_VP, _VP, _I64, _VP, _I64]),
            "fbr_get_map": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
            "fbr_project": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP, _VP, _VP, _VP]),
            "fbr_extract_features": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
            "fbr_register": (ctypes.c_int, [_VP, _VP, _I64, _VP, _I64, _VP, _VP]),
            "fbr_register_trace": (ctypes.c_int, [_VP, _VP, _I64, _VP, _I64, _VP, _VP, _VP]),
            "fbr_process_scan": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_double, _VP, _VP]),
            "fbr_reset_stream": (ctypes.c_int, [_VP]),
            "fbr_process_batch": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, _VP, _VP]),
            "fbr_ingest_bytes": (ctypes.c_int, [_VP, _VP]),
            "fbr_map_grid_info": (ctypes.c_int, [_VP, _VP]),
            "fbr_debug_counters": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int]),
            "fbr_batch_stage": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, _VP]),
            "fbr_batch_launch": (ctypes.c_int, [_VP]),
            "fbr_batch_wait": (ctypes.c_int, [_VP]),
            "fbr_batch_results": (ctypes.c_int, [_VP, _VP, _VP]),
            "fbr_batch_export": (ctypes.c_int, [_VP, _VP]),
            "fbr_batch_set_full_masks": (ctypes.c_int, [_VP, ctypes.c_int]),
            "fbr_batch_labels": (ctypes.c_int, [_VP, ctypes.c_int, _VP, _I64, _VP]),
            "fbr_batch_flush": (ctypes.c_int, [_VP]),
            "fbr_batch_export_ready": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
            "fbr_batch_bytes": (ctypes.c_int, [_VP, _VP, _VP]),
            "fbr_set_profiling": (ctypes.c_int, [_VP, ctypes.c_int]),
            "fbr_set_profiling_kernels": (ctypes.c_int, [_VP, ctypes.c_char_p]),
            "fbr_kernel_time": (ctypes.c_int, [_VP, ctypes.c_char_p, _VP, _VP]),
            "fbr_stream": (_VP, [_VP]),
            "fbr_voxel_grid": (ctypes.c_int, [_VP, _VP, _I64, ctypes.c_float, _VP, _VP]),
            "fbr_affine_from_pose": (None, [_VP, _VP]),
            "fbr_pose_from_affine": (None, [_VP, _VP]),
            "fbr_selftest_math": (ctypes.c_int, [ctypes.c_int, _VP, _VP, _VP]),
            "fbr_selftest_eigen6": (ctypes.c_int, [ctypes.c_int, _VP, _VP]),
            "fbr_selftest_eig_certified": (ctypes.c_int, [ctypes.c_int, _VP, ctypes.c_float, _VP]),
            "fbr_selftest_voxel_order": (ctypes.c_int, [_I64, _VP, ctypes.c_int, _VP]),
            "fbr_selftest_radix_sort": (ctypes.c_int, [_I64, ctypes.c_int, ctypes.c_int, _VP, _VP]),
            "fbr_load_map": (ctypes.c_int, [_VP, ctypes.c_char_p, ctypes.c_char_p]),
            "fbr_pcd_read": (ctypes.c_int, [ctypes.c_char_p, _VP, _I64, _VP]),
            "fbr_pcd_write_ascii": (ctypes.c_int, [ctypes.c_char_p, _VP, _I64]),
            "fbr_pcd_write_binary": (ctypes.c_int, [ctypes.c_char_p, _VP, _I64]),
            "fbr_msg_to_points": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP]),
            "fbr_points_to_msg_data": (ctypes.c_int, [_VP, _I64, _VP]),
            "fbr_project_msg": (ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP]),
            "fbr_process_msg": (ctypes.c_int, [_VP, _VP, ctypes.c_double, _VP, _VP, _VP]),
            "fbr_imu_convert": (ctypes.c_int, [_VP, _VP, _VP]),
            "fbr_imu_deskew_info": (ctypes.c_int, [_VP, _I64, ctypes.c_double, ctypes.c_double, _VP, _VP]),
            "fbr_set_deskew": (ctypes.c_int, [_VP, _VP, ctypes.c_int]),
            "fbr_stream_copy_bandwidth": (ctypes.c_int, [ctypes.c_int, _I64, ctypes.c_int, _VP]),
            "fbr_valu_peak": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP, _VP]),
            "fbr_keyframe_params_default": (None, [_VP]),
            "fbr_keyframes_add": (ctypes.c_int, [_VP, _VP, _VP, _I64, _VP, _I64]),
            "fbr_keyframes_set_pose": (ctypes.c_int, [_VP, _I64, _VP]),
            "fbr_keyframes_count": (ctypes.c_int, [_VP, _VP]),
            "fbr_keyframes_reset": (ctypes.c_int, [_VP]),
            "fbr_extract_surrounding_keyframes": (ctypes.c_int, [_VP, ctypes.c_double, _VP, _VP, _VP, _VP]),
            "fbr_comm_unique_id": (ctypes.c_int, [_VP]),
            "fbr_comm_create": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
            "fbr_comm_create_local": (ctypes.c_int, [_VP, _VP, ctypes.c_int, ctypes.c_int]),
            "fbr_comm_destroy": (ctypes.c_int, [_VP]),
            "fbr_batch_allgather": (ctypes.c_int, [_VP, _VP, _I64, _VP, _VP, _VP]),
        }
        diag = bool(os.environ.get("FBR_LIB"))  # an A/B build of another round may lack newer entry points
        for name, (res, args) in sig.items():
            if diag and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


def strerror(status):
    return lib().fbr_strerror(status).decode()


def _check(status, where):
    if status != 0:
        raise FbrError(status, where)


def device_count():
    n = ctypes.c_int(0)
    _check(lib().fbr_device_count(ctypes.byref(n)), "fbr_device_count")
    return n.value


def debug_counters(reset=False):
    """(kernel launches, blocking host syncs, GN flag polls) since the last reset (process-wide)."""
    v = [ctypes.c_longlong() for _ in range(3)]
    _check(lib().fbr_debug_counters(*[ctypes.byref(x) for x in v], int(reset)), "fbr_debug_counters")
    return tuple(x.value for x in v)


def host_times(reset=False):
    """Host wall time (s) of the single-scan calls since the last reset: (upload, stage enqueue,
    result wait, whole call) -- diagnostic (fbr_diag_host_times)."""
    f = lib().fbr_diag_host_times
    f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
    v = (ctypes.c_longlong * 4)()
    _check(f(v, int(reset)), "fbr_diag_host_times")
    return tuple(x * 1e-9 for x in v)


def wait_stats(reset=False):
    """Host waits on device results since the last reset -- diagnostic (fbr_diag_wait_stats):
    (fallbacks: a flag or direct result not visible although its stream drained, waits longer than
    1 ms, the longest wait in s, stream queries)."""
    if not hasattr(lib(), "fbr_diag_wait_stats"):  # an A/B build of an earlier round (FBR_LIB)
        return -1, -1, -1.0, -1
    f = lib().fbr_diag_wait_stats
    f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
    v = (ctypes.c_longlong * 4)()
    _check(f(v, int(reset)), "fbr_diag_wait_stats")
    return int(v[0]), int(v[1]), v[2] * 1e-9, int(v[3])


def batch_times(reset=False):
    """Host wall time (s) of fbr_batch_launch calls since the last reset, and the part of it spent
    waiting for the Gauss-Newton iteration flags -- diagnostic (fbr_diag_batch_times)."""
    f = lib().fbr_diag_batch_times
    f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
    v = (ctypes.c_longlong * 2)()
    _check(f(v, int(reset)), "fbr_diag_batch_times")
    return tuple(x * 1e-9 for x in v)


def knn_tile_stats(reset=False):
    """Block-tile kNN counters since the last reset: (queries, binned queries, tiles built, points
    in tiles, points scanned by the tile loads, tiles over capacity, 0, 0), or None unless
    FBR_KNN_TILE_STATS=1 -- diagnostic (fbr_diag_knn_tile_stats, k_knn_tile.hip)."""
    f = lib().fbr_diag_knn_tile_stats
    f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
    v = (ctypes.c_ulonglong * 8)()
    if f(v, int(reset)) != 0:
        return None
    return tuple(int(x) for x in v)


def selftest_math(a, b):
    """Device sqrt(|a|), a/b, atan2f(a,b), a*b+b*a-a, sinf(a), cosf(a) (see fbr_selftest_math)."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    out = np.zeros((len(a), 6), np.float32)
    _check(lib().fbr_selftest_math(len(a), ptr(a), ptr(b), ptr(out)), "fbr_selftest_math")
    return out


def selftest_eigen6(mats):
    """cv::eigen of symmetric 6x6 float matrices on the device (see fbr_selftest_eigen6): returns
    (single-lane (W, V), wave-parallel (W, V)), W (n, 6) descending, V (n, 6, 6) rows = vectors."""
    a = np.ascontiguousarray(mats, np.float32).reshape(-1, 36)
    out = np.zeros((len(a), 84), np.float32)
    _check(lib().fbr_selftest_eigen6(len(a), ptr(a), ptr(out)), "fbr_selftest_eigen6")
    n = len(a)
    return ((out[:, :6], out[:, 6:42].reshape(n, 6, 6)), (out[:, 42:48], out[:, 48:].reshape(n, 6, 6)))


def selftest_eig_certified(mats, thr=100.0):
    """1 where the device certifies every eigenvalue of a symmetric 6x6 float matrix above thr
    without the Jacobi (fbr_selftest_eig_certified: the iteration-0 degeneracy fast path)."""
    a = np.ascontiguousarray(mats, np.float32).reshape(-1, 36)
    out = np.zeros(len(a), np.int32)
    _check(lib().fbr_selftest_eig_certified(len(a), ptr(a), ctypes.c_float(thr), ptr(out)), "fbr_selftest_eig_certified")
    return out


def selftest_voxel_order(keys, lds=False):
    """Device emulation of the VoxelGrid index sort (fbr_selftest_voxel_order): the point order
    std::sort leaves (keys[i], i) in, i.e. the stable key sort of the partitioned sequence."""
    k = np.ascontiguousarray(keys, np.uint32)
    perm = np.zeros(len(k), np.uint32)
    _check(lib().fbr_selftest_voxel_order(len(k), ptr(k), int(lds), ptr(perm)), "fbr_selftest_voxel_order")
    return perm[np.argsort(k[perm], kind="stable")].astype(np.int64)


def selftest_radix_sort(keys, nbits, variant):
    """One of the VoxelGrid kernels' radix sorts on the device (fbr_selftest_radix_sort): (sorted
    keys, source index of every sorted position)."""
    k = np.ascontiguousarray(keys, np.uint32).copy()
    perm = np.zeros(len(k), np.uint32)
    _check(lib().fbr_selftest_radix_sort(len(k), int(nbits), int(variant), ptr(k), ptr(perm)), "fbr_selftest_radix_sort")
    return k, perm.astype(np.int64)


def stream_copy_bandwidth(device=0, nbytes=2 << 30, iters=20):
    """Achievable HBM GB/s of a device float4 copy (read + write), fbr_stream_copy_bandwidth."""
    g = ctypes.c_double()
    _check(lib().fbr_stream_copy_bandwidth(device, nbytes, iters, ctypes.byref(g)), "fbr_stream_copy_bandwidth")
    return g.value


def valu_peak(device=0, waves_per_simd=4, kind=0, iters=4096, reps=5):
    """(wave-level VALU G instr/s, ms per launch) of the fbr_valu_peak probe: kind 0 v_fma_f32,
    1 v_add_u32, 2 v_pk_fma_f32, 3 v_cmp_lt_u64, 4 v_cmp_lt_u32, waves_per_simd waves on every SIMD."""
    g, ms = ctypes.c_double(), ctypes.c_double()
    _check(lib().fbr_valu_peak(device, waves_per_simd, kind, iters, reps, ctypes.byref(g), ctypes.byref(ms)),
           "fbr_valu_peak")
    return g.value, ms.value


def affine_from_pose(pose):
    m = np.zeros(16, np.float32)
    lib().fbr_affine_from_pose(ptr(np.ascontiguousarray(pose, np.float32)), ptr(m))
    return m.reshape(4, 4)


def pose_from_affine(m):
    p = np.zeros(6, np.float32)
    lib().fbr_pose_from_affine(ptr(np.ascontiguousarray(m, np.float32).reshape(16)), ptr(p))
    return p


def pcd_read(path):
    """pcl::io::loadPCDFile<PointXYZI> (mapOptmization.h:247-248) -> POINT_XYZI array (host only)."""
    p = os.fsencode(path)
    n = _I64()
    _check(lib().fbr_pcd_read(p, None, 0, ctypes.byref(n)), f"fbr_pcd_read({path})")
    out = np.zeros(max(n.value, 1), POINT_XYZI)
    _check(lib().fbr_pcd_read(p, ptr(out), len(out), ctypes.byref(n)), f"fbr_pcd_read({path})")
    return out[:n.value].copy()


def pcd_write(path, points, binary=False):
    """pcl::io::savePCDFileASCII (mapOptmization.h:511-515), or DATA binary when `binary`."""
    pts = _as_points(points, POINT_XYZI)
    f = lib().fbr_pcd_write_binary if binary else lib().fbr_pcd_write_ascii
    _check(f(os.fsencode(path), ptr(pts) if len(pts) else None, len(pts)), f"fbr_pcd_write({path})")


def msg_to_points(msg):
    """cachePointCloud's fromROSMsg + checks (imageProjection.cpp:253-298) on the host.
    Returns (POINT_XYZIRT array, msg_flags)."""
    n, fl = _I64(), _I32()
    _check(lib().fbr_msg_to_points(ctypes.byref(msg.c), None, 0, ctypes.byref(n), ctypes.byref(fl)),
           "fbr_msg_to_points")
    out = np.zeros(max(n.value, 1), POINT_XYZIRT)
    _check(lib().fbr_msg_to_points(ctypes.byref(msg.c), ptr(out), len(out), ctypes.byref(n), ctypes.byref(fl)),
           "fbr_msg_to_points")
    return out[:n.value].copy(), fl.value


def points_to_msg(points):
    """pcl::toROSMsg of a PointXYZI cloud (publishCloud, utility.h:255-264) -> PointCloud2."""
    pts = _as_points(points, POINT_XYZI)
    data = np.zeros(32 * len(pts), np.uint8)
    _check(lib().fbr_points_to_msg_data(ptr(pts) if len(pts) else None, len(pts), ptr(data) if len(pts) else None),
           "fbr_points_to_msg_data")
    fields = [("x", 0, PF_FLOAT32, 1), ("y", 4, PF_FLOAT32, 1), ("z", 8, PF_FLOAT32, 1),
              ("intensity", 16, PF_FLOAT32, 1)]
    return PointCloud2(data.tobytes(), fields, width=len(pts), point_step=32)


def imu_convert(ext, samples):
    """imuConverter (utility.h:219-253) on each sample (IMU_SAMPLE array) with IMU_EXTRINSICS `ext`."""
    samples = _as_points(np.atleast_1d(samples), IMU_SAMPLE)
    ext = np.ascontiguousarray(ext)
    out = np.zeros_like(samples)
    for i in range(len(samples)):
        _check(lib().fbr_imu_convert(ptr(ext), ctypes.c_void_p(samples.ctypes.data + i * IMU_SAMPLE.itemsize),
                                     ctypes.c_void_p(out.ctypes.data + i * IMU_SAMPLE.itemsize)), "fbr_imu_convert")
    return out


def imu_deskew_info(queue, time_scan_cur, time_scan_next, previous=None):
    """deskewInfo + imuDeskewInfo (imageProjection.cpp:303-393) on a queue of converted samples.
    Returns (DESKEW_TABLE record, number of leading samples popped).  `previous` carries the
    imu*Init fields forward as the reference's cloudInfo member does."""
    queue = _as_points(np.atleast_1d(queue), IMU_SAMPLE)
    tab = np.zeros(1, DESKEW_TABLE) if previous is None else np.array(previous, DESKEW_TABLE).reshape(1).copy()
    n_pop = _I64()
    _check(lib().fbr_imu_deskew_info(ptr(queue) if len(queue) else None, len(queue), ctypes.c_double(time_scan_cur),
                                     ctypes.c_double(time_scan_next), ptr(tab), ctypes.byref(n_pop)),
           "fbr_imu_deskew_info")
    return tab[0], n_pop.value


def _as_points(a, dtype):
    a = np.ascontiguousarray(a)
    if a.dtype != dtype:
        raise TypeError(f"expected dtype {dtype}, got {a.dtype}")
    return a


class Context:
    """One fbr_ctx: a HIP device, a stream, HBM buffers for `max_batch` scans."""

    def __init__(self, params=None, device=0, **kw):
        self.params = params if params is not None else default_params(**kw)
        self._h = ctypes.c_void_p()
        _check(lib().fbr_create(ctypes.byref(self._h), ctypes.byref(self.params), device), "fbr_create")

    def close(self):
        if self._h:
            lib().fbr_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- map (mapOptmization.h:245-260) ----
    def set_map(self, corner, surf):
        corner = _as_points(corner, POINT_XYZI)
        surf = _as_points(surf, POINT_XYZI)
        _check(lib().fbr_set_map(self._h, ptr(corner), len(corner), ptr(surf), len(surf)), "fbr_set_map")

    def load_map(self, corner_pcd, surf_pcd):
        """loadPCDFile(cloudCorner.pcd / cloudSurf.pcd) + the start-up DS (mapOptmization.h:245-260)."""
        _check(lib().fbr_load_map(self._h, os.fsencode(corner_pcd), os.fsencode(surf_pcd)), "fbr_load_map")

    def get_map(self):
        nc, ns = _I64(), _I64()
        _check(lib().fbr_get_map(self._h, ctypes.byref(nc), ctypes.byref(ns), None, None), "fbr_get_map")
        c = np.zeros(max(nc.value, 1), POINT_XYZI)
        s = np.zeros(max(ns.value, 1), POINT_XYZI)
        _check(lib().fbr_get_map(self._h, None, None, ptr(c), ptr(s)), "fbr_get_map")
        return c[:nc.value].copy(), s[:ns.value].copy()

    # ---- A2+A4 ----
    def project(self, pts):
        pts = _as_points(pts, POINT_XYZIRT)
        n_in, H = len(pts), self.params.n_scan
        start = np.zeros(H, np.int32)
        end = np.zeros(H, np.int32)
        cap = max(n_in, 1)
        col = np.zeros(cap, np.int32)
        rng = np.zeros(cap, np.float32)
        cloud = np.zeros(cap, POINT_XYZI)
        n = _I64()
        _check(lib().fbr_project(self._h, ptr(pts), n_in, ptr(start), ptr(end), ptr(col), ptr(rng),
                                 ptr(cloud), ctypes.byref(n)), "fbr_project")
        k = n.value
        return dict(start_ring=start, end_ring=end, col_ind=col[:k].copy(), range=rng[:k].copy(),
                    cloud=cloud[:k].copy())

    # ---- A6-A9 ----
    def extract_features(self, n_points):
        H, W = self.params.n_scan, self.params.horizon_scan
        label = np.zeros(max(n_points, 1), np.int8)
        corner = np.zeros(120 * H, POINT_XYZI)
        surf = np.zeros(max(H * W, 1), POINT_XYZI)
        nc, ns = _I64(), _I64()
        _check(lib().fbr_extract_features(self._h, ptr(label), ptr(corner), ctypes.byref(nc), ptr(surf),
                                          ctypes.byref(ns)), "fbr_extract_features")
        return dict(label=label[:n_points].copy(), corner=corner[:nc.value].copy(),
                    surf=surf[:ns.value].copy())

    def features(self, pts):
        pr = self.project(pts)
        f = self.extract_features(len(pr["col_ind"]))
        f["n_points"] = len(pr["col_ind"])
        return f

    # ---- A10-A18 ----
    def register(self, corner, surf, pose, trace=False):
        corner = _as_points(corner, POINT_XYZI)
        surf = _as_points(surf, POINT_XYZI)
        pose = np.ascontiguousarray(pose, dtype=np.float32).copy()
        st = FbrRegStats()
        if trace:
            tr = np.zeros((self.params.max_iterations, 6), np.float32)
            _check(lib().fbr_register_trace(self._h, ptr(corner), len(corner), ptr(surf), len(surf),
                                            ptr(pose), ctypes.byref(st), ptr(tr)), "fbr_register_trace")
            d = st.as_dict()
            return pose, d, tr[:d["iterations"]].copy()
        _check(lib().fbr_register(self._h, ptr(corner), len(corner), ptr(surf), len(surf), ptr(pose),
                                  ctypes.byref(st)), "fbr_register")
        return pose, st.as_dict()

    def process_scan(self, pts, stamp, pose):
        pts = _as_points(pts, POINT_XYZIRT)
        pose = np.ascontiguousarray(pose, dtype=np.float32).copy()
        st = FbrRegStats()
        _check(lib().fbr_process_scan(self._h, ptr(pts), len(pts), ctypes.c_double(stamp), ptr(pose),
                                      ctypes.byref(st)), "fbr_process_scan")
        return pose, st.as_dict()

    def project_msg(self, msg):
        """project() from a raw PointCloud2 (unpacked on the device); also returns msg_flags."""
        H = self.params.n_scan
        cap = max(msg.c.width * msg.c.height, 1)
        start, end = np.zeros(H, np.int32), np.zeros(H, np.int32)
        col, rng, cloud = np.zeros(cap, np.int32), np.zeros(cap, np.float32), np.zeros(cap, POINT_XYZI)
        n, fl = _I64(), _I32()
        _check(lib().fbr_project_msg(self._h, ctypes.byref(msg.c), ptr(start), ptr(end), ptr(col), ptr(rng),
                                     ptr(cloud), ctypes.byref(n), ctypes.byref(fl)), "fbr_project_msg")
        k = n.value
        return dict(start_ring=start, end_ring=end, col_ind=col[:k].copy(), range=rng[:k].copy(),
                    cloud=cloud[:k].copy(), msg_flags=fl.value)

    def process_msg(self, msg, stamp, pose):
        pose = np.ascontiguousarray(pose, dtype=np.float32).copy()
        st, fl = FbrRegStats(), _I32()
        _check(lib().fbr_process_msg(self._h, ctypes.byref(msg.c), ctypes.c_double(stamp), ptr(pose),
                                     ctypes.byref(st), ctypes.byref(fl)), "fbr_process_msg")
        return pose, st.as_dict(), fl.value

    def set_deskew(self, tables):
        """IMU deskew tables (DESKEW_TABLE records) for the following calls: job j of a batch uses
        tables[j], single-scan calls tables[0]; None restores the reference's runtime path."""
        if tables is None:
            _check(lib().fbr_set_deskew(self._h, None, 0), "fbr_set_deskew")
            return
        t = np.ascontiguousarray(np.array(tables, DESKEW_TABLE).reshape(-1))
        _check(lib().fbr_set_deskew(self._h, ptr(t), len(t)), "fbr_set_deskew")

    # ---- LIO-SAM keyframe local map (mapOptmization.h:857-978) ----
    def keyframes_add(self, pose, corner, surf):
        """cloudKeyPoses3D/6D + corner/surfCloudKeyFrames push_back (pose: KEYPOSE record)."""
        p = np.array(pose, KEYPOSE).reshape(1)
        corner = _as_points(corner, POINT_XYZI)
        surf = _as_points(surf, POINT_XYZI)
        _check(lib().fbr_keyframes_add(self._h, ptr(p), ptr(corner) if len(corner) else None, len(corner),
                                       ptr(surf) if len(surf) else None, len(surf)), "fbr_keyframes_add")

    def keyframes_set_pose(self, index, pose):
        p = np.array(pose, KEYPOSE).reshape(1)
        _check(lib().fbr_keyframes_set_pose(self._h, index, ptr(p)), "fbr_keyframes_set_pose")

    def keyframes_count(self):
        n = _I64()
        _check(lib().fbr_keyframes_count(self._h, ctypes.byref(n)), "fbr_keyframes_count")
        return n.value

    def keyframes_reset(self):
        _check(lib().fbr_keyframes_reset(self._h), "fbr_keyframes_reset")

    def extract_surrounding_keyframes(self, stamp, kparams):
        """extractSurroundingKeyFrames: the local map becomes the registration map (no CropBox).
        Returns (n_corner_map, n_surf_map, n_frames)."""
        nc, ns, nf = _I64(), _I64(), ctypes.c_int32()
        _check(lib().fbr_extract_surrounding_keyframes(self._h, ctypes.c_double(stamp), ctypes.byref(kparams),
                                                       ctypes.byref(nc), ctypes.byref(ns), ctypes.byref(nf)),
               "fbr_extract_surrounding_keyframes")
        return nc.value, ns.value, nf.value

    @property
    def stream_handle(self):
        """The context's primary hipStream_t (int address): batch results and exports are ordered on it."""
        return lib().fbr_stream(self._h) or 0

    def reset_stream(self):
        _check(lib().fbr_reset_stream(self._h), "fbr_reset_stream")

    # ---- batches of independent jobs ----
    def _scan_ptrs(self, scans):
        scans = [_as_points(s, POINT_XYZIRT) for s in scans]
        arr = (ctypes.c_void_p * len(scans))(*[s.ctypes.data for s in scans])
        n_in = np.array([len(s) for s in scans], np.int64)
        return scans, arr, n_in

    def process_batch(self, scans, guesses):
        keep, arr, n_in = self._scan_ptrs(scans)
        poses = np.ascontiguousarray(np.asarray(guesses, np.float32).reshape(-1, 6)).copy()
        stats = np.zeros(len(keep), REG_STATS)
        _check(lib().fbr_process_batch(self._h, arr, ptr(n_in), len(keep), ptr(poses), ptr(stats)),
               "fbr_process_batch")
        return poses, stats

    def map_grid_info(self):
        """The map's kNN grid: dict(sparse, dims, box_cells, stored, n_corner, n_surf)."""
        v = np.zeros(8, np.int64)
        _check(lib().fbr_map_grid_info(self._h, ptr(v)), "fbr_map_grid_info")
        return dict(sparse=bool(v[0]), dims=tuple(int(x) for x in v[1:4]), box_cells=int(v[4]), stored=int(v[5]),
                    n_corner=int(v[6]), n_surf=int(v[7]))

    def ingest_bytes(self):
        """Host-to-device scan bytes of the last process_batch."""
        v = ctypes.c_double()
        _check(lib().fbr_ingest_bytes(self._h, ctypes.byref(v)), "fbr_ingest_bytes")
        return v.value

    def batch_stage(self, scans, guesses):
        keep, arr, n_in = self._scan_ptrs(scans)
        g = np.ascontiguousarray(np.asarray(guesses, np.float32).reshape(-1, 6))
        _check(lib().fbr_batch_stage(self._h, arr, ptr(n_in), len(keep), ptr(g)), "fbr_batch_stage")
        self._staged = len(keep)

    def batch_launch(self):
        _check(lib().fbr_batch_launch(self._h), "fbr_batch_launch")

    def batch_wait(self):
        _check(lib().fbr_batch_wait(self._h), "fbr_batch_wait")

    def batch_results(self):
        poses = np.zeros((self._staged, 6), np.float32)
        stats = np.zeros(self._staged, REG_STATS)
        _check(lib().fbr_batch_results(self._h, ptr(poses), ptr(stats)), "fbr_batch_results")
        return poses, stats

    def batch_set_full_masks(self, on=True):
        """Later batch launches compute whole feature masks (fbr_batch_set_full_masks)."""
        _check(lib().fbr_batch_set_full_masks(self._h, int(bool(on))), "fbr_batch_set_full_masks")

    def batch_labels(self, job):
        """cloudLabel of batch job `job` of the latest (full-mask) launch: int8 [n_points]."""
        n = _I64()
        rc = lib().fbr_batch_labels(self._h, int(job), None, 0, ctypes.byref(n))
        if rc not in (0, -4):  # FBR_ERR_CAPACITY: the count is in n
            _check(rc, "fbr_batch_labels")
        out = np.zeros(max(n.value, 1), np.int8)
        _check(lib().fbr_batch_labels(self._h, int(job), ptr(out), len(out), ctypes.byref(n)), "fbr_batch_labels")
        return out[:n.value]

    def batch_export(self, device_ptr):
        """Enqueue the 32 B/job pose records into device memory at `device_ptr` (int address)."""
        _check(lib().fbr_batch_export(self._h, ctypes.c_void_p(device_ptr)), "fbr_batch_export")

    def batch_flush(self):
        """Enqueue the rest of every launch in flight (no device synchronisation)."""
        _check(lib().fbr_batch_flush(self._h), "fbr_batch_flush")

    def batch_export_ready(self, device_ptr, wait_stream=0):
        """Pipelined export: the records of the latest fully enqueued, not yet exported launch into
        `device_ptr`, after the work queued on `wait_stream` (a HIP stream handle, 0 = none).
        Returns (launch_id, export stream handle); launch_id -1 = nothing exported."""
        st, lid = _VP(), _I64()
        _check(lib().fbr_batch_export_ready(self._h, ctypes.c_void_p(device_ptr), ctypes.c_void_p(wait_stream or None),
                                            ctypes.byref(st), ctypes.byref(lid)), "fbr_batch_export_ready")
        return lid.value, st.value or 0

    def diag_ring_filter(self, kernel):
        """Diagnostic: the per-ring surf filter kernel of this context (-1 by launch size, 0 the
        512-thread kernel, 2 four waves per ring; fbr_diag_ring_filter)."""
        f = lib().fbr_diag_ring_filter
        f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
        _check(f(self._h, int(kernel)), "fbr_diag_ring_filter")

    def diag_force_capacity_error(self, job):
        """Diagnostic: batch job `job` of the following launches is reported as over the feature
        capacity (fbr_diag_force_capacity_error); job < 0 clears it."""
        f = lib().fbr_diag_force_capacity_error
        f.restype, f.argtypes = ctypes.c_int, [_VP, ctypes.c_int]
        _check(f(self._h, int(job)), "fbr_diag_force_capacity_error")

    def batch_bytes(self):
        t, g = ctypes.c_double(), ctypes.c_double()
        _check(lib().fbr_batch_bytes(self._h, ctypes.byref(t), ctypes.byref(g)), "fbr_batch_bytes")
        return t.value, g.value

    def set_profiling(self, on=True, kernels=None):
        """Time kernels with HIP events on the ctx stream; `kernels` restricts it to those names."""
        names = None if not kernels else ",".join(kernels).encode()
        _check(lib().fbr_set_profiling_kernels(self._h, names), "fbr_set_profiling_kernels")
        _check(lib().fbr_set_profiling(self._h, 1 if on else 0), "fbr_set_profiling")

    def kernel_time(self, name):
        ms, n = ctypes.c_double(), _I64()
        _check(lib().fbr_kernel_time(self._h, name.encode(), ctypes.byref(ms), ctypes.byref(n)),
               "fbr_kernel_time")
        return ms.value, n.value

    def voxel_grid(self, pts, leaf):
        pts = _as_points(pts, POINT_XYZI)
        out = np.zeros(max(len(pts), 1), POINT_XYZI)
        n = _I64()
        _check(lib().fbr_voxel_grid(self._h, ptr(pts), len(pts), ctypes.c_float(leaf), ptr(out),
                                    ctypes.byref(n)), "fbr_voxel_grid")
        return out[:n.value].copy()


def comm_unique_id():
    """fbr_comm_unique_id: the 128-byte RCCL id rank 0 makes and hands to the other ranks."""
    buf = (ctypes.c_uint8 * 128)()
    _check(lib().fbr_comm_unique_id(buf), "fbr_comm_unique_id")
    return bytes(buf)


class Comm:
    """The pose-record communicator of one rank (fbr_comm_create): RCCL over the context's device.
    allgather(launch_id, recv_ptr, wait_stream) all-gathers that launch's 32-B records of every rank
    into the device buffer recv_ptr ([nranks][max_jobs][8] f32), after the work queued on
    wait_stream (the caller's stream still reading recv, or None), and returns the HIP stream to
    wait on before reading recv."""

    def __init__(self, ctx, uid, nranks, rank, max_jobs):
        self._h = _VP()
        idb = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().fbr_comm_create(ctypes.byref(self._h), ctx._h, idb, int(nranks), int(rank), int(max_jobs)),
               "fbr_comm_create")
        self._ctx = ctx
        self.nranks, self.rank, self.max_jobs = int(nranks), int(rank), int(max_jobs)

    def allgather(self, launch_id, recv_ptr, wait_stream=None):
        st = _VP()
        _check(lib().fbr_batch_allgather(self._ctx._h, self._h, int(launch_id), ctypes.c_void_p(recv_ptr),
                                         ctypes.c_void_p(wait_stream or None), ctypes.byref(st)), "fbr_batch_allgather")
        return st.value or 0

    def close(self):
        if self._h:
            _check(lib().fbr_comm_destroy(self._h), "fbr_comm_destroy")
            self._h = _VP()


__all__ = ["Context", "Comm", "comm_unique_id", "FbrError", "FbrParams", "default_params", "lib", "device_count",
           "affine_from_pose", "pose_from_affine", "pcd_read", "pcd_write", "msg_to_points", "points_to_msg", "PointCloud2",
           "imu_convert", "imu_deskew_info",
           "EXPORTED_SYMBOLS"]
