#!/usr/bin/env python3
"""Timeline of bench steps from a rocprofv3 --kernel-trace CSV.

A step starts at every NSUB-th k_project dispatch (one per sub-batch).  For the last complete
steps it reports the span, the time the device runs at least one / two / three kernels, the
summed kernel time per family, and the idle gaps (no kernel running) with their positions, so a
small-batch step's exposed phases (front end, GN tail, host turn-around) can be read off.

usage: step_timeline.py KERNEL_TRACE.csv NSUB [STEPS]
"""
import csv
import re
import sys
from collections import defaultdict

FAM = [("project", r"k_project\b"), ("extract", r"k_compact|k_rowcount"), ("features", r"k_features"),
       ("voxel_ring", r"k_voxel_ring"), ("concat", r"k_concat"), ("voxel_scan", r"k_voxel_grid"),
       ("gn_knn", r"k_gn_knn"), ("gn_residual", r"k_gn_residual"), ("gn_solve", r"k_gn_solve"),
       ("gn_init", r"k_gn_init"), ("gn_finalize", r"k_gn_finalize"), ("crop", r"k_crop"),
       ("pack", r"k_pack|k_export")]


def fam(name):
    for f, rx in FAM:
        if re.search(rx, name):
            return f
    return "other"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    nsub = int(sys.argv[2])
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    proj = [i for i, e in enumerate(ev) if re.search(r"k_project\b", e[2])]
    starts = proj[::nsub]
    if len(starts) < nsteps + 1:
        sys.exit(f"need >= {nsteps + 1} steps, found {len(starts)}")
    for s in range(len(starts) - nsteps - 1, len(starts) - 1):
        seg = ev[starts[s]:starts[s + 1]]
        t0 = seg[0][0]
        t1 = ev[starts[s + 1]][0]
        # sweep: concurrency levels
        pts = []
        for a, b, _ in seg:
            pts.append((a, 1))
            pts.append((min(b, t1), -1))
        pts.sort()
        lvl, last = 0, t0
        at = defaultdict(int)
        gaps = []
        for t, d in pts:
            if t > last:
                at[lvl] += t - last
                if lvl == 0 and t - last > 2000:
                    gaps.append(((last - t0) / 1e3, (t - last) / 1e3))
            lvl += d
            last = max(last, t)
        span = t1 - t0
        ft = defaultdict(float)
        fc = defaultdict(int)
        for a, b, n in seg:
            ft[fam(n)] += (b - a) / 1e3
            fc[fam(n)] += 1
        busy1 = sum(v for k, v in at.items() if k >= 1)
        print(f"step span {span / 1e3:.1f} us, dispatches {len(seg)}; >=1 kernel {busy1 / span:.3f}, "
              f">=2 {sum(v for k, v in at.items() if k >= 2) / span:.3f}, >=3 {sum(v for k, v in at.items() if k >= 3) / span:.3f}, "
              f"idle {at[0] / 1e3:.1f} us")
        print("  kernel us (sum / count): " + ", ".join(f"{k} {v:.0f}/{fc[k]}" for k, v in sorted(ft.items(), key=lambda t: -t[1])))
        if gaps:
            print("  idle gaps > 2 us (at us, length us): " + ", ".join(f"({a:.0f}, {b:.1f})" for a, b in gaps[:20]))


if __name__ == "__main__":
    main()
