#!/usr/bin/env python3
"""Per-dispatch view of one bench step from a rocprofv3 --kernel-trace CSV: durations of the
GN kernels by iteration index, plus the other kernels, for the last complete step."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"] for r in rows]
# a step starts at each k_project dispatch
starts = [i for i, n in enumerate(names) if "k_project" in n]
if len(starts) < 2:
    sys.exit("need >= 2 steps")
seg = rows[starts[-2]:starts[-1]]
by = defaultdict(list)
for r in seg:
    nm = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fbr::", "")
    by[nm].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
t0 = int(seg[0]["Start_Timestamp"])
t1 = int(seg[-1]["End_Timestamp"])
print(f"step wall (first start -> last end): {(t1 - t0) / 1000.0:.1f} us, dispatches {len(seg)}")
busy = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in seg) / 1000.0
print(f"sum of kernel durations: {busy:.1f} us")
for nm, ds in by.items():
    s = " ".join(f"{d:.0f}" for d in ds[:32])
    print(f"{nm:40s} n={len(ds):3d} sum={sum(ds):8.1f} us | {s}")
