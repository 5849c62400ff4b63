"""Diagnostic: build a k_voxel_ring variant with s_memtime phase stamps (wave 0 of each ring) and
print where a ring's time goes and how many rings run at once."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import build  # noqa: E402

diag = os.environ.get("FBR_DIAG_LIB") or build.build_hip(defines=("FBR_VR_STAMPS",), name="libfbr_hip_vrdiag.so")  # prebuilt diag lib (GPU box)
os.environ["FBR_LIB"] = diag
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import default_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
EXACT = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # 1: exact_voxel_order (std::sort's partition phase)
H, W = 64, 1800
P = default_params(H, W, max_batch=B, exact_voxel_order=EXACT)
cm, sm = synth.config_map("C2")
jobs = synth.make_jobs("C2", B)
ctx = api.Context(P)
ctx.set_map(cm, sm)
L = api.lib()
L.fbr_diag_feature_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.fbr_diag_feature_stamps(ctx._h, None)  # allocate the stamp buffer
ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
ctx.batch_launch(); ctx.batch_wait()
out = np.zeros((B * H, 12), np.uint64)
L.fbr_diag_feature_stamps(ctx._h, out.ctypes.data)
t = out[:, :5].astype(np.int64)
ok = t[:, 4] > 0
t = t[ok]
d = np.diff(t, axis=1).astype(np.float64)
names = ["load+compact+minmax", "keys" + (" + partition phase" if EXACT else ""), "run sort", "emit"]
print(f"rings stamped: {ok.sum()} of {len(out)}; mean ticks per ring {d.sum(1).mean():.0f} (s_memtime, 100 MHz)")
for n, v in zip(names, d.mean(0)):
    print(f"  {n:22s} {v:10.1f}  {100 * v / d.sum(1).mean():5.1f}%")
span = t[:, 4].max() - t[:, 0].min()
print(f"launch span {span} ticks; mean ring duration {(t[:, 4] - t[:, 0]).mean():.0f}; "
      f"mean concurrent rings {(t[:, 4] - t[:, 0]).sum() / span:.0f}")
ctx.set_profiling(True); ctx.batch_launch(); ctx.batch_wait()
print("voxel_ring kernel ms:", ctx.kernel_time("voxel_ring"))
