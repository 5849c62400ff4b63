import sys, os, numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'oracle'))
from feature_base_pointcloud_registration_amd import synth, api
from feature_base_pointcloud_registration_amd.fbr_types import default_params
import pyoracle as O
for cfg in ["C1", "C2"]:
    H, W, *_ = synth.CONFIGS[cfg]
    P = default_params(H, W, max_batch=4)
    ctx = api.Context(P)
    for j in range(3):
        gt, guess = synth.job(1000 + j)
        pts = synth.scan(gt, H, W, seed=1000 + j)
        a = O.project(P, pts); b = ctx.project(pts)
        for k in ["start_ring", "end_ring", "col_ind"]:
            if not np.array_equal(a[k], b[k]):
                d = np.nonzero(a[k] != b[k])[0]; print(cfg, j, k, "differs at", d[:10], a[k][d[:5]], b[k][d[:5]])
        ra, rb = a["range"].view(np.int32), b["range"].view(np.int32)
        if not np.array_equal(ra, rb):
            d = np.nonzero(ra != rb)[0]; print(cfg, j, "range differs", len(d), d[:5], a["range"][d[:5]], b["range"][d[:5]])
        ca, cb = a["cloud"].view(np.int32).reshape(-1, 4), b["cloud"].view(np.int32).reshape(-1, 4)
        if not np.array_equal(ca, cb):
            d = np.nonzero((ca != cb).any(1))[0]; print(cfg, j, "cloud differs", len(d), d[:5], a["cloud"][d[:3]], b["cloud"][d[:3]])
        s = O.Stream(P); fo = s.features(pts); fg = ctx.extract_features(len(b["col_ind"]))
        if not np.array_equal(fo["label"], fg["label"]):
            d = np.nonzero(fo["label"] != fg["label"])[0]
            print(cfg, j, "label differs", len(d), d[:20], fo["label"][d[:20]], fg["label"][d[:20]], "n=", len(fo["label"]))
            print("   start", a["start_ring"][:8], "end", a["end_ring"][:8])
        else:
            print(cfg, j, "labels equal", int((fo["label"] == 1).sum()), int((fo["label"] == -1).sum()))
        ctx.reset_stream()
    ctx.close()
rng = np.random.default_rng(0)
a = (rng.standard_normal(1 << 20) * rng.choice([1e-3, 1.0, 50.0, 1e4], 1 << 20)).astype(np.float32)
b = (rng.standard_normal(1 << 20) * rng.choice([1e-3, 1.0, 50.0, 1e4], 1 << 20)).astype(np.float32)
out = api.selftest_math(a, b)
ref_sqrt = np.sqrt(np.abs(a)); ref_div = a / b
with np.errstate(all='ignore'):
    ref_mul = a * b + b * a - a
print("sqrt mismatches", int((out[:, 0].view(np.int32) != ref_sqrt.view(np.int32)).sum()))
print("div mismatches", int((out[:, 1].view(np.int32) != ref_div.view(np.int32)).sum()))
print("muladd mismatches", int((out[:, 3].view(np.int32) != ref_mul.view(np.int32)).sum()))
