#!/usr/bin/env python3
"""CPU model of k_features' greedy rounds (k_features.hip greedy_rounds), to size alternatives
before touching the kernel.  For C2 scans: the oracle's projection, then per segment the corner
and surf candidates, the conflict structure (+-5 reach stopped by column gaps > 10) and the
number of rounds the wave needs (corner walk over the whole segment; batch surf walk over the
window [m-63, m] with the candidates left of it frozen).
usage: feat_rounds_model.py [scans]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle as O  # noqa: E402
from feature_base_pointcloud_registration_amd import synth  # noqa: E402


def reach(gap, li, L):
    f = 0
    while f < 5 and li + f < L - 1 and not gap[li + f]:
        f += 1
    b = 0
    while b < 5 and li - 1 - b >= 0 and not gap[li - 1 - b]:
        b += 1
    return f, b


def rounds(cand, prio, nbrs):
    """Greedy MIS by priority in rounds (the kernel's rule incl. same-round suppression)."""
    und = set(np.flatnonzero(cand).tolist())
    tak = set()
    r = 0
    while und:
        r += 1
        new_t = [u for u in und if not any(v in tak for v in nbrs[u] if prio[v] > prio[u])
                 and not any(v in und for v in nbrs[u] if prio[v] > prio[u])]
        tak |= set(new_t)
        new_n = [u for u in und if u not in new_t and any(v in tak for v in nbrs[u] if prio[v] > prio[u])]
        und -= set(new_t) | set(new_n)
        if r > 1000:
            break
    return r, len(tak)


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    P = synth.config_params("C2")
    H = P.n_scan
    stats = {"corner": [], "surf": [], "ccand": [], "scand": [], "m": []}
    for pts, _, _ in synth.make_jobs("C2", ns, base_seed=1000):
        pr = O.project(P, pts)
        r = pr["range"].astype(np.float32)
        col = pr["col_ind"]
        n = len(r)
        curv = np.zeros(n, np.float32)
        for i in range(5, n - 5):
            d = np.float32(0)
            for k in range(-5, 6):
                d = np.float32(d + (np.float32(-10) * r[i] if k == 0 else r[i + k]))
            curv[i] = d * d
        gap = np.ones(n, bool)
        gap[:-1] = np.abs(np.diff(col)) > 10
        picked = np.zeros(n, bool)  # occlusion marks ignored: a slight overcount of candidates
        for ring in range(H):
            s, e = pr["start_ring"][ring], pr["end_ring"][ring]
            for j in range(6):
                sp = (s * (6 - j) + e * j) // 6
                ep = (s * (5 - j) + e * (j + 1)) // 6 - 1
                if sp >= ep:
                    continue
                m = ep - sp
                idx = np.arange(sp, ep + 1)
                nb = []
                for u in range(m + 1):
                    f, b = reach(gap, sp + u, n)
                    nb.append([u + d for d in range(1, f + 1) if u + d <= m] + [u - d for d in range(1, b + 1) if u - d >= 0])
                cv = curv[idx]
                # corner: ep first, then descending curvature
                pc = cv.astype(np.float64).copy()
                pc[m] = np.inf
                cc = (~picked[idx]) & (cv > P.edge_threshold)
                rc, _ = rounds(cc, pc, nb)
                # surf window: ascending curvature, ep last
                ps = -cv.astype(np.float64)
                ps[m] = -np.inf
                sc = (~picked[idx]) & (cv < P.surf_threshold)
                lo = max(0, m - 63)
                win = sc.copy()
                win[:max(0, lo - 5)] = False
                rs, _ = rounds(win, ps, nb)
                stats["corner"].append(rc)
                stats["surf"].append(rs)
                stats["ccand"].append(int(cc.sum()))
                stats["scand"].append(int(win.sum()))
                stats["m"].append(m)
    for k, v in stats.items():
        v = np.array(v)
        print(f"{k:6s} mean {v.mean():7.2f}  p50 {np.median(v):6.1f}  p90 {np.percentile(v, 90):6.1f}  max {v.max()}")


if __name__ == "__main__":
    main()
