#!/usr/bin/env python3
"""CPU cost model of the first Gauss-Newton iteration's kNN (no warm start), to size a two-pass
design before writing it: a flat walk (fbr_gn.h knn5_grid<.., kFlat>) under a static bound b, exact
whenever the query's 5th distance is <= b, with the current rank-ordered walk rerun for the lanes
where it is not.

For C2 jobs, the mapping-DS queries in Morton order transformed by the GUESS pose (iteration 0),
the 1 m (y, z) x 0.25 m (x) grid of the DS maps.  Per 64-query wave:
  current   sum over the 9 row slots of the max over lanes of the points the lane scans in that slot
            (rows in near-side-first rank order, cut = the running 5th distance, capped below 1.0)
  two-pass  max over lanes of the points in the rows within b (flat: one counted loop), plus the
            current walk's cost over the lanes whose 5th distance exceeds b (or that have fewer
            than 5 neighbours below 1.0)
usage: knn_iter0_model.py [jobs]
"""
import os
import sys
from collections import defaultdict

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import pyoracle as O  # noqa: E402
from feature_base_pointcloud_registration_amd import synth  # noqa: E402
from knn_union_sim import ds_morton, transform  # noqa: E402

F = np.float32
BELOW1 = F(0.99999994)


def rank_offset(k, s):
    return 0 if k == 0 else (s * ((k + 1) >> 1) if k & 1 else -s * (k >> 1))


def axis_lb(q, f, o, c):
    if o == 0:
        return F(0)
    return F(F(f + o) * c - q) if o > 0 else F(q - F(f + o + 1) * c)


class Grid:
    def __init__(self, pts):
        self.p = pts
        cx = np.floor(pts[:, 0] * F(4)).astype(np.int64)
        cy = np.floor(pts[:, 1]).astype(np.int64)
        cz = np.floor(pts[:, 2]).astype(np.int64)
        rows = defaultdict(list)
        for i, (x, y, z) in enumerate(zip(cx.tolist(), cy.tolist(), cz.tolist())):
            rows[(z, y)].append((x, i))
        self.rows = {k: (np.array([a for a, _ in sorted(v)]), np.array([b for _, b in sorted(v)])) for k, v in rows.items()}

    def row(self, z, y, x0, x1):
        r = self.rows.get((z, y))
        if r is None:
            return np.zeros(0, np.int64)
        xs, ids = r
        a, b = np.searchsorted(xs, x0, "left"), np.searchsorted(xs, x1, "right")
        return ids[a:b]


def walk(g, q, bound, flat):
    """Points scanned per row slot (9), the final sorted 5 d2 (< 1.0)."""
    qx, qy, qz = q
    fx, fy, fz = np.floor(qx * F(4)), np.floor(qy), np.floor(qz)
    sgy = 1 if qy - fy >= 0.5 else -1
    sgz = 1 if qz - fz >= 0.5 else -1
    best = []
    slots = []
    for ksum in range(5):
        for ky in range(3):
            kz = ksum - ky
            if kz < 0 or kz > 2:
                continue
            oy = ky - 1 if flat else rank_offset(ky, sgy)
            oz = kz - 1 if flat else rank_offset(kz, sgz)
            ly, lz = axis_lb(qy, fy, oy, F(1)), axis_lb(qz, fz, oz, F(1))
            lb = F(F(ly * ly) + F(lz * lz))
            k5 = best[4] if len(best) == 5 else F(1)
            cut = min(k5, bound, BELOW1) if not flat else min(bound, BELOW1)
            if lb > cut:
                slots.append(0)
                continue
            xa = xb = 0
            ga = gb = True
            for o in range(1, 5):
                ta = F(F(axis_lb(qx, fx, -o, F(0.25)) ** 2) + F(ly * ly)) + F(lz * lz)
                tb = F(F(axis_lb(qx, fx, o, F(0.25)) ** 2) + F(ly * ly)) + F(lz * lz)
                ga = ga and not ta > cut
                gb = gb and not tb > cut
                if ga:
                    xa = -o
                if gb:
                    xb = o
            ids = g.row(int(fz) + oz, int(fy) + oy, int(fx) + xa, int(fx) + xb)
            slots.append(len(ids))
            if len(ids):
                d = g.p[ids] - np.array(q, F)
                d2 = ((F(0) + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
                best = sorted(best + [v for v in d2.tolist() if v < 1.0])[:5]
    return slots, best


def main():
    nj = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    P = synth.config_params("C2")
    cmap, smap = synth.config_map("C2")
    omap = O.Map(P, cmap, smap)
    mc, ms = omap.arrays()
    grids = {"corner": Grid(np.stack([mc["x"], mc["y"], mc["z"]], 1).astype(F)),
             "surf": Grid(np.stack([ms["x"], ms["y"], ms["z"]], 1).astype(F))}
    bounds = [F(0.09), F(0.16), F(0.25), F(0.36)]
    cur_tot, new_tot, waves, fails = 0, {b: 0 for b in bounds}, 0, {b: 0 for b in bounds}
    nq = 0
    for pts, guess, _ in synth.make_jobs("C2", nj, base_seed=1000):
        f = O.Stream(P).features(pts)
        for name, cloud, leaf in (("corner", f["corner"], P.mapping_corner_leaf_size),
                                  ("surf", f["surf"], P.mapping_surf_leaf_size)):
            q = transform(guess, ds_morton(cloud, leaf))
            g = grids[name]
            for w0 in range(0, len(q), 64):
                lanes = q[w0:w0 + 64]
                cur = [walk(g, tuple(x), F(np.inf), False) for x in lanes]
                cur_cost = sum(max(c[0][s] for c in cur) for s in range(9))
                cur_tot += cur_cost
                waves += 1
                nq += len(lanes)
                for b in bounds:
                    flat = [walk(g, tuple(x), b, True) for x in lanes]
                    flat_cost = max(sum(c[0]) for c in flat)
                    bad = [i for i, c in enumerate(cur) if len(c[1]) < 5 or c[1][4] > b]
                    fails[b] += len(bad)
                    rerun = sum(max(cur[i][0][s] for i in bad) for s in range(9)) if bad else 0
                    new_tot[b] += flat_cost + rerun
    print(f"{waves} waves, {nq} queries; current walk {cur_tot / waves:.1f} trips per wave")
    for b in bounds:
        print(f"  b = {b:.2f}: two-pass {new_tot[b] / waves:.1f} trips per wave ({new_tot[b] / cur_tot:.2f}x), "
              f"rerun lanes {fails[b] / nq:.3f}")


if __name__ == "__main__":
    main()
