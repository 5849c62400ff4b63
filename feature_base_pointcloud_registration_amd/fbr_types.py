"""ctypes / numpy mirrors of the C-ABI types declared in include/fbr.h.

The layouts follow the reference's data model: ``POINT_XYZIRT`` is the PointXYZIRT payload of
/root/reference/src/imageProjection.cpp:8-21, ``POINT_XYZI`` is pcl::PointXYZI
(/root/reference/include/utility.h:55), ``FbrParams`` carries config/params.yaml plus the constants
mapOptmization.h hard-codes, ``FbrRegStats`` reports what registration() decided.
"""
import ctypes

import numpy as np

POINT_XYZIRT = np.dtype(
    [("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("intensity", "<f4"), ("ring", "<u2"),
     ("pad_", "<u2"), ("time", "<f4")], align=True)
assert POINT_XYZIRT.itemsize == 24

POINT_XYZI = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("intensity", "<f4")])
assert POINT_XYZI.itemsize == 16

REG_STATS_FIELDS = ["status", "iterations", "converged", "degenerate", "n_sel", "n_corner_ds",
                    "n_surf_ds", "n_corner_map", "n_surf_map", "n_points", "n_corner", "n_surf"]
REG_STATS = np.dtype([(f, "<i4") for f in REG_STATS_FIELDS])

# IMU deskew (include/fbr.h "IMU deskew"): sensor_msgs/Imu fields, extrinsics, imuDeskewInfo table
IMU_QUEUE = 500  # queueLength, imageProjection.cpp:23
IMU_SAMPLE = np.dtype([("stamp", "<f8"), ("linear_acceleration", "<f8", 3), ("angular_velocity", "<f8", 3),
                       ("orientation", "<f8", 4)])
assert IMU_SAMPLE.itemsize == 88
IMU_EXTRINSICS = np.dtype([("ext_rot", "<f8", 9), ("ext_rpy", "<f8", 9)])
DESKEW_TABLE = np.dtype([("status", "<i4"), ("imu_available", "<i4"), ("imu_pointer_cur", "<i4"),
                         ("imu_roll_init", "<f4"), ("imu_pitch_init", "<f4"), ("imu_yaw_init", "<f4"),
                         ("time_scan_cur", "<f8"), ("imu_time", "<f8", IMU_QUEUE), ("imu_rot_x", "<f8", IMU_QUEUE),
                         ("imu_rot_y", "<f8", IMU_QUEUE), ("imu_rot_z", "<f8", IMU_QUEUE)], align=True)
assert DESKEW_TABLE.itemsize == 32 + 4 * 8 * IMU_QUEUE
FBR_DESKEW_READY, FBR_DESKEW_WAIT_IMU = 0, 1

# LIO-SAM keyframe store (include/fbr.h "LIO-SAM keyframe local map")
KEYPOSE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("intensity", "<f4"), ("roll", "<f4"),
                    ("pitch", "<f4"), ("yaw", "<f4"), ("pad_", "<f4"), ("time", "<f8")])
assert KEYPOSE.itemsize == 40


class FbrKeyframeParams(ctypes.Structure):
    _fields_ = [("search_radius", ctypes.c_float), ("pose_density", ctypes.c_float),
                ("loop_closure", ctypes.c_int32), ("submap_size", ctypes.c_int32),
                ("recent_window", ctypes.c_double)]


def keyframe_params(**kw):
    """fbr_keyframe_params_default (params.yaml:66-71, the 10 s window of mapOptmization.h:900)."""
    p = FbrKeyframeParams(50.0, 2.0, 0, 25, 10.0)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


FBR_OK = 0
FBR_REG_OK = 0
FBR_REG_NOT_ENOUGH_FEATURES = 1
FBR_REG_SKIPPED_INTERVAL = 2
FBR_REG_FEATURE_CAPACITY = 3  # batch job over the device feature capacity: pose = guess


class FbrParams(ctypes.Structure):
    _fields_ = [
        ("n_scan", ctypes.c_int32),
        ("horizon_scan", ctypes.c_int32),
        ("edge_threshold", ctypes.c_float),
        ("surf_threshold", ctypes.c_float),
        ("edge_feature_min_valid_num", ctypes.c_int32),
        ("surf_feature_min_valid_num", ctypes.c_int32),
        ("odometry_surf_leaf_size", ctypes.c_float),
        ("mapping_corner_leaf_size", ctypes.c_float),
        ("mapping_surf_leaf_size", ctypes.c_float),
        ("z_tollerance", ctypes.c_float),
        ("rotation_tollerance", ctypes.c_float),
        ("number_of_cores", ctypes.c_int32),
        ("mapping_process_interval", ctypes.c_double),
        ("crop_half", ctypes.c_float * 3),
        ("max_iterations", ctypes.c_int32),
        ("max_points_per_scan", ctypes.c_int32),
        ("max_batch", ctypes.c_int32),
        ("exact_voxel_order", ctypes.c_int32),
        ("pipeline_depth", ctypes.c_int32),
        ("reserved_", ctypes.c_int32 * 2),
    ]


class FbrRegStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int32) for f in REG_STATS_FIELDS]

    def as_dict(self):
        return {f: getattr(self, f) for f in REG_STATS_FIELDS}


def default_params(n_scan=16, horizon_scan=1800, **overrides):
    """fbr_params_default(): params.yaml values + the reference's hard-coded constants."""
    p = FbrParams()
    p.n_scan = n_scan
    p.horizon_scan = horizon_scan
    p.edge_threshold = 1.0
    p.surf_threshold = 0.1
    p.edge_feature_min_valid_num = 10
    p.surf_feature_min_valid_num = 100
    p.odometry_surf_leaf_size = 0.4
    p.mapping_corner_leaf_size = 0.2
    p.mapping_surf_leaf_size = 0.4
    p.z_tollerance = 1000.0
    p.rotation_tollerance = 1000.0
    p.number_of_cores = 4
    p.mapping_process_interval = 0.15
    p.crop_half[0], p.crop_half[1], p.crop_half[2] = 30.0, 30.0, 10.0
    p.max_iterations = 30
    p.max_points_per_scan = n_scan * horizon_scan
    p.max_batch = 1
    for k, v in overrides.items():
        if k == "crop_half":
            for i in range(3):
                p.crop_half[i] = v[i]
        else:
            setattr(p, k, v)
    return p


def ptr(a, ctype=ctypes.c_void_p):
    """Raw pointer of a contiguous numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return ctypes.cast(a.ctypes.data, ctype)


# ---- sensor_msgs/PointCloud2 (include/fbr.h "PointCloud2 wire format") ----
PF_INT8, PF_UINT8, PF_INT16, PF_UINT16, PF_INT32, PF_UINT32, PF_FLOAT32, PF_FLOAT64 = range(1, 9)
FBR_ERR_MSG = -8
FBR_MSG_NO_TIME, FBR_MSG_RING_UNMAPPED, FBR_MSG_XYZI_UNMAPPED = 1, 2, 4
_PF_OF_NUMPY = {"i1": PF_INT8, "u1": PF_UINT8, "i2": PF_INT16, "u2": PF_UINT16, "i4": PF_INT32,
                "u4": PF_UINT32, "f4": PF_FLOAT32, "f8": PF_FLOAT64}


class FbrPointField(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("offset", ctypes.c_uint32), ("datatype", ctypes.c_uint8),
                ("count", ctypes.c_uint32)]


class FbrPointCloud2(ctypes.Structure):
    _fields_ = [("height", ctypes.c_uint32), ("width", ctypes.c_uint32),
                ("fields", ctypes.POINTER(FbrPointField)), ("n_fields", ctypes.c_int32),
                ("is_bigendian", ctypes.c_uint8), ("point_step", ctypes.c_uint32),
                ("row_step", ctypes.c_uint32), ("data", ctypes.c_void_p), ("data_size", ctypes.c_uint64),
                ("is_dense", ctypes.c_uint8)]


class PointCloud2:
    """A sensor_msgs/PointCloud2 view for the C-ABI: keeps the byte buffer and field names alive.

    fields: list of (name, offset, datatype, count).  `data` is bytes-like of at least
    (height-1)*row_step + width*point_step bytes."""

    def __init__(self, data, fields, width, height=1, point_step=None, row_step=None, is_dense=True):
        self.buf = np.frombuffer(bytes(data), np.uint8)
        self.fields = [(str(n), int(o), int(t), int(c)) for n, o, t, c in fields]
        self._names = [n.encode() for n, _, _, _ in self.fields]
        self._fa = (FbrPointField * max(len(self.fields), 1))()
        for k, ((_, o, t, c), nm) in enumerate(zip(self.fields, self._names)):
            self._fa[k] = FbrPointField(nm, o, t, c)
        ps = point_step if point_step is not None else (len(self.buf) // max(width * height, 1))
        m = FbrPointCloud2()
        m.height, m.width = height, width
        m.fields = ctypes.cast(self._fa, ctypes.POINTER(FbrPointField))
        m.n_fields = len(self.fields)
        m.is_bigendian = 0
        m.point_step = ps
        m.row_step = row_step if row_step is not None else ps * width
        m.data = self.buf.ctypes.data if len(self.buf) else None
        m.data_size = len(self.buf)
        m.is_dense = 1 if is_dense else 0
        self.c = m

    @classmethod
    def from_array(cls, arr, height=1, is_dense=True):
        """Message whose points are the records of a numpy structured array (fields by dtype)."""
        arr = np.ascontiguousarray(arr)
        fields = []
        for name in arr.dtype.names:
            dt, off = arr.dtype.fields[name][:2]
            base, shape = (dt.subdtype if dt.subdtype else (dt, ()))
            count = int(np.prod(shape)) if shape else 1
            fields.append((name, off, _PF_OF_NUMPY[base.str[1:]], count))
        return cls(arr.tobytes(), fields, width=len(arr) // height, height=height,
                   point_step=arr.dtype.itemsize, is_dense=is_dense)
