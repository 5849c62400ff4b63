import sys, time, numpy as np
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R,'oracle'))
from feature_base_pointcloud_registration_amd import synth, api
from feature_base_pointcloud_registration_amd.fbr_types import default_params
import pyoracle as O
print("devices", api.device_count())
for cfg in ["C1", "C2"]:
    H, W, *_ = synth.CONFIGS[cfg]
    P = default_params(H, W, max_batch=4)
    ctx = api.Context(P)
    gt, guess = synth.job(1000)
    pts = synth.scan(gt, H, W, seed=1000)
    a = O.project(P, pts); b = ctx.project(pts)
    ok = all(np.array_equal(a[k], b[k]) for k in ["start_ring", "end_ring", "col_ind"]) and a["range"].view(np.int32).tolist() == b["range"].view(np.int32).tolist() and np.array_equal(a["cloud"].view(np.float32), b["cloud"].view(np.float32))
    print(cfg, "projection bit-exact:", ok, len(a["col_ind"]), len(b["col_ind"]))
    s = O.Stream(P); fo = s.features(pts); fg = ctx.extract_features(len(b["col_ind"]))
    print(cfg, "labels equal:", np.array_equal(fo["label"], fg["label"]), "corner equal:", np.array_equal(fo["corner"].view(np.float32), fg["corner"].view(np.float32)), len(fo["corner"]), len(fg["corner"]), "surf n:", len(fo["surf"]), len(fg["surf"]))
    if len(fo["surf"]) == len(fg["surf"]):
        d = np.abs(fo["surf"].view(np.float32).reshape(-1,4) - fg["surf"].view(np.float32).reshape(-1,4)).max(); print("  surf max abs diff", d)
    corner, surf = synth.config_map(cfg)
    om = O.Map(P, corner, surf); mc, ms = om.arrays()
    ctx.set_map(mc, ms)
    gmc, gms = ctx.get_map(); print(cfg, "map DS sizes", len(mc), len(ms), len(gmc), len(gms))
    po, so, to = om.register(fo["corner"], fo["surf"], guess)
    t = time.time(); pg, sg, tg = ctx.register(fo["corner"], fo["surf"], guess, trace=True); dt = time.time() - t
    print(cfg, "oracle", po, so["iterations"], so["n_sel"]); print(cfg, "gpu   ", pg, sg["iterations"], sg["n_sel"], "%.3fs" % dt)
    print(cfg, "pose diff", np.abs(po - pg).max())
    ctx.close()
