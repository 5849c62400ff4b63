"""Diagnostic: marginal cost of k_features phases.  Builds variants with one phase skipped
(-DFBR_FEAT_SKIP_{CM,CORNER,SURF}; their results are wrong, only the kernel time is used) and
prints the features kernel time of each on a C2 batch."""
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = sys.argv[1] if len(sys.argv) > 1 else "128"
CHILD = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np
from feature_base_pointcloud_registration_amd import api, synth
from feature_base_pointcloud_registration_amd.fbr_types import default_params
B = int(sys.argv[1])
P = default_params(64, 1800, max_batch=B)
jobs = synth.make_jobs("C2", B)
ctx = api.Context(P)
ctx.set_map(*synth.config_map("C2"))
ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
ctx.batch_launch(); ctx.batch_wait()
ctx.set_profiling(True, ["features"])
for _ in range(5):
    ctx.batch_launch()
ctx.batch_wait()
ms, n = ctx.kernel_time("features")
print(f"{os.environ.get('FBR_VARIANT', 'base'):8s} features {ms / n:.3f} ms/launch")
""" % R
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import build  # noqa: E402
for var, defs in [("base", ()), ("no_cm", ("FBR_FEAT_SKIP_CM",)), ("no_corner", ("FBR_FEAT_SKIP_CORNER",)),
                  ("no_surf", ("FBR_FEAT_SKIP_SURF",)), ("no_stale", ("FBR_FEAT_SKIP_STALE",))]:
    lib = build.build_hip(defines=defs + ("FBR_DIAG_VARIANT",), name=f"libfbr_hip_{var}.so") if defs else \
        build.build_hip()
    env = dict(os.environ, FBR_LIB=lib, FBR_VARIANT=var)
    subprocess.run([sys.executable, "-c", CHILD, B], env=env, check=True)
