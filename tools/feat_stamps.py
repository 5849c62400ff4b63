"""Diagnostic: build a k_features variant with s_memtime phase stamps and print where a ring's
cycles go (shares, not absolute times: the stamps themselves perturb the kernel)."""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import build  # noqa: E402

diag = os.environ.get("FBR_DIAG_LIB") or build.build_hip(defines=("FBR_FEAT_STAMPS",), name="libfbr_hip_diag.so")  # prebuilt diag lib (GPU box)
os.environ["FBR_LIB"] = diag
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import default_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
H, W = 64, 1800
P = default_params(H, W, max_batch=B)
cm, sm = synth.config_map("C2")
jobs = synth.make_jobs("C2", B)
ctx = api.Context(P)
ctx.set_map(cm, sm)
L = api.lib()
L.fbr_diag_feature_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
L.fbr_diag_feature_stamps(ctx._h, None)  # allocate the stamp buffer
ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
ctx.batch_launch(); ctx.batch_wait()
out = np.zeros((8 * B * H, 12), np.uint64)  # the buffer spans every launch slot (<= 8)
L.fbr_diag_feature_stamps(ctx._h, out.ctypes.data)
out = out[:B * H]  # slot 0: the first launch
names = ["load", "flags+picked", "seg: sort", "seg: members/cm", "seg: corner rounds", "seg: cap+apply",
         "seg: surf rounds", "seg: apply surf", "seg: candidates", "outputs", "seg: direct cm", "seg: direct rank"]
tot = out.astype(np.float64).mean(0)
print("mean cycles per ring (s_memtime ticks):", int(tot.sum()))
for n, v in zip(names, tot):
    print(f"  {n:20s} {v:12.0f}  {100 * v / tot.sum():5.1f}%")
per_ring = out.astype(np.float64).reshape(B, H, 12)
tot_r = per_ring.sum(2)  # [B][H]
print(f"per-ring totals: ring 0 mean {tot_r[:, 0].mean():.0f}, rings 1.. mean {tot_r[:, 1:].mean():.0f}, "
      f"max {tot_r.max():.0f} (ring {int(tot_r.argmax() % H)}), median {np.median(tot_r):.0f}")
r0 = per_ring[:, 0, :].mean(0)
print("ring 0 breakdown:", ", ".join(f"{n} {v:.0f}" for n, v in zip(names, r0) if v > 0))
flat = per_ring.reshape(B * H, 12)
tot_f = flat.sum(1)
for i in np.argsort(-tot_f)[:6]:  # the slowest rings (a single scan waits for its slowest ring)
    print(f"ring {i % H} of job {i // H}: {tot_f[i]:.0f}:", ", ".join(f"{n} {v:.0f}" for n, v in zip(names, flat[i]) if v > 0))
print(f"rings above 1.5x the median: {int((tot_f > 1.5 * np.median(tot_f)).sum())} of {len(tot_f)}")
ctx.set_profiling(True); ctx.batch_launch(); ctx.batch_wait()
print("features kernel ms:", ctx.kernel_time("features"))
