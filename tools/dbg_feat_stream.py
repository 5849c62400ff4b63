import sys, os, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle')
from feature_base_pointcloud_registration_amd import api, synth
from feature_base_pointcloud_registration_amd.fbr_types import default_params
import pyoracle as O
cfg = sys.argv[1]
H, W = synth.CONFIGS[cfg][:2]
P = default_params(H, W)
st = O.Stream(P)
with api.Context(P) as ctx:
    for seed in range(20, 24):
        gt, _ = synth.job(seed)
        pts = synth.scan(gt, H, W, seed=seed)
        pr = ctx.project(pts)
        print("seed", seed, "n", len(pr["col_ind"]), "start", pr["start_ring"][:3], "end", pr["end_ring"][:3], flush=True)
        fo = st.features(pts)
        fg = ctx.extract_features(len(pr["col_ind"]))
        print("  labels equal", np.array_equal(fo["label"], fg["label"]), flush=True)
