#!/usr/bin/env python3
"""How much the path's kernels run side by side, from a rocprofv3 --kernel-trace CSV of the bench.

Over the timed region of a `bench.py --steps STEPS` run (from the k_project dispatch of the first
timed launch -- the last STEPS of them -- to the end of the last kernel; pipelined launches make
the gaps between k_project dispatches uneven, so only the whole region is divided by STEPS), per
kernel family: summed dispatch time per launch, the part of it during which no other kernel ran
("alone"), and the families it overlapped most.  Plus the concurrency profile (time with 0 / 1 /
2 / 3 / 4+ kernels running).

usage: concurrency.py KERNEL_TRACE.csv STEPS
"""
import csv
import re
import sys
from collections import defaultdict

FAM = [("project", r"k_project\b"), ("extract", r"k_compact|k_rowcount"), ("features", r"k_features"),
       ("voxel_ring", r"k_voxel_ring"), ("concat", r"k_concat"), ("voxel_scan", r"k_voxel_grid"),
       ("gn_knn", r"k_gn_knn"), ("gn_residual", r"k_gn_residual"), ("gn_solve", r"k_gn_solve"),
       ("gn_loop", r"k_gn_loop"), ("gn_init", r"k_gn_init"), ("gn_finalize", r"k_gn_finalize"), ("crop", r"k_crop"),
       ("pack", r"k_pack|k_export")]


def fam(name):
    for f, rx in FAM:
        if re.search(rx, name):
            return f
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nsteps = int(sys.argv[2])
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"])) for r in rows)
    proj = [e[0] for e in ev if e[2] == "project"]
    if len(proj) < nsteps:
        sys.exit(f"need >= {nsteps} launches")
    t0, t1 = proj[-nsteps], max(b for _, b, _ in ev)
    seg = [(max(a, t0), min(b, t1), f) for a, b, f in ev if b > t0 and a < t1]
    # elementary intervals
    cuts = sorted({t for a, b, _ in seg for t in (a, b)})
    total = defaultdict(float)
    alone = defaultdict(float)
    pair = defaultdict(float)
    level = defaultdict(float)
    for x0, x1 in zip(cuts, cuts[1:]):
        act = [f for a, b, f in seg if a <= x0 and b >= x1]
        d = (x1 - x0) / 1e3
        level[min(len(act), 4)] += d
        for f in act:
            total[f] += d
            if len(act) == 1:
                alone[f] += d
        fs = sorted(set(act))
        for i in range(len(fs)):
            for j in range(i + 1, len(fs)):
                pair[(fs[i], fs[j])] += d
    span = (t1 - t0) / 1e3
    print(f"{nsteps} launches, {span / nsteps:.1f} us per launch; time with 0/1/2/3/4+ kernels: " +
          " / ".join(f"{level[k] / span:.3f}" for k in range(5)))
    print(f"{'family':12s} {'us/launch':>9s} {'alone':>7s}  top overlaps (us/launch)")
    for f, v in sorted(total.items(), key=lambda t: -t[1]):
        ov = sorted(((g if g != f else h, w) for (g, h), w in pair.items() if f in (g, h)), key=lambda t: -t[1])[:3]
        print(f"{f:12s} {v / nsteps:9.1f} {alone[f] / max(v, 1e-9):7.3f}  " + ", ".join(f"{g} {w / nsteps:.0f}" for g, w in ov))


if __name__ == "__main__":
    main()
