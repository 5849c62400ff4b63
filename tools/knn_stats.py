"""Diagnostic: per-query work of the grid kNN (k_gn_knn) on a C2 batch — rows considered /
scanned, points scanned / inserted — for the grid cell sizes given (FBR_KNN_CELL)."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import build  # noqa: E402

diag = os.environ.get("FBR_DIAG_LIB") or build.build_hip(defines=("FBR_KNN_STATS",), name="libfbr_hip_diag.so")  # prebuilt diag lib (GPU box)
os.environ["FBR_LIB"] = diag
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import default_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
CFG = os.environ.get("CFG", "C2")  # BASELINE config of the jobs and map
ITERS = int(os.environ.get("ITERS", "0"))  # cap the GN iterations (1: iteration 0 alone)
P = synth.config_params(CFG, max_batch=B, **({"max_iterations": ITERS} if ITERS else {}))
cm, sm = synth.config_map(CFG)
jobs = synth.make_jobs(CFG, B)
L = api.lib()
L.fbr_diag_knn_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
for cell in (sys.argv[2:] or ["0.5"]):  # "YZ" or "YZ/X" cell sizes in m
    if cell != "default":
        os.environ["FBR_KNN_CELL"] = cell.split("/")[0]
    if "/" in cell:
        os.environ["FBR_KNN_CELL_X"] = cell.split("/")[1]
    ctx = api.Context(P)
    ctx.set_map(cm, sm)
    ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
    ctx.batch_launch(); ctx.batch_wait()
    L.fbr_diag_knn_stats(None, 1)
    ctx.set_profiling(True)
    ctx.batch_launch(); ctx.batch_wait()
    st = np.zeros(48, np.uint64)
    L.fbr_diag_knn_stats(st.ctypes.data, 0)
    q = float(st[0])
    print(f"cell {cell}: queries {int(q)} (corner {int(st[6])}) accepted {st[5] / q:.3f} | per query: rows considered "
          f"{st[1] / q:.1f}, rows scanned {st[2] / q:.1f}, points scanned {st[3] / q:.1f}, inserted {st[4] / q:.1f} | "
          f"gn_knn ms {ctx.kernel_time('gn_knn')} | point-loop lane efficiency "
          f"{float(st[3]) / (64.0 * float(st[7])):.3f} (points scanned / (64 x wave iterations)) | "
          f"neighbours unchanged from the previous iteration: {float(st[9]) / max(float(st[8]), 1.0):.3f} "
          f"of {int(st[8])} warm-started queries")
    if st[10]:
        h = st[12:46].astype(np.float64) / float(st[10])
        cum = np.cumsum(h)
        print(f"  flat queries {int(st[10])}: points within the static cut {st[11] / float(st[10]):.2f} per query; "
              f"share with more than 8 / 12 / 16 / 24 / 31: {1 - cum[8]:.4f} / {1 - cum[12]:.4f} / {1 - cum[16]:.4f} / "
              f"{1 - cum[24]:.4f} / {1 - cum[31]:.4f}; >= 64: {h[33]:.5f}; flat walk: {st[46] / float(st[10]):.2f} points "
              f"per query, lane efficiency {float(st[46]) / (64.0 * float(max(st[47], 1))):.3f}")
    ctx.close()
