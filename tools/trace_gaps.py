#!/usr/bin/env python3
"""Per-scan device busy time vs wall time from a rocprofv3 kernel trace of tools/latency_probe.py.

Splits the dispatches into scans at each k_project launch (the first kernel of a scan), then per
scan reports the span (first dispatch start to last dispatch end), the summed kernel durations,
the idle gaps between dispatches, and the per-kernel durations (medians over the scans).

usage: trace_gaps.py KERNEL_TRACE.csv [SKIP_SCANS]
"""
import csv
import re
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
scans, cur = [], None
for r in rows:
    name = r["Kernel_Name"]
    if re.search(r"k_project\b", name):
        cur = []
        scans.append(cur)
    if cur is not None:
        cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
scans = scans[skip:]
span, busy, per = [], [], defaultdict(list)
for s in scans:
    span.append((s[-1][1] - s[0][0]) / 1e3)
    busy.append(sum(e - b for b, e, _ in s) / 1e3)
    agg = defaultdict(float)
    for b, e, nm in s:
        short = re.sub(r"\(.*", "", nm).replace("void ", "").replace("fbr::", "")
        agg[short] += (e - b) / 1e3
    for k, v in agg.items():
        per[k].append(v)
print(f"scans {len(scans)}: span median {np.median(span):.1f} us, kernel busy median {np.median(busy):.1f} us, "
      f"dispatches/scan {np.mean([len(s) for s in scans]):.1f}")
for k, v in sorted(per.items(), key=lambda kv: -np.median(kv[1])):
    print(f"  {k:50s} {np.median(v):8.1f} us")
