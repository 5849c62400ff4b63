"""MI355X-native feature-based scan-to-map registration (drop-in for the per-scan hot path of
qpc001/Feature_Base_Pointcloud_Registration: projection -> LOAM features -> scan-to-map GN).

The product is libfbr_hip.so (HIP kernels for gfx950 behind the C-ABI of include/fbr.h);
`api` is its Python front-end, `synth` generates synthetic inputs.
"""
from .fbr_types import POINT_XYZI, POINT_XYZIRT, REG_STATS, FbrParams, default_params  # noqa: F401

__version__ = "0.1.0"
