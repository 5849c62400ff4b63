#!/usr/bin/env python3
"""One scan's dispatch timeline (start offset, gap to the previous dispatch, duration) from a
rocprofv3 kernel trace of tools/latency_probe.py.  usage: scan_timeline.py KERNEL_TRACE.csv [SCAN]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
scans, cur = [], None
for r in rows:
    if re.search(r"k_project\b", r["Kernel_Name"]):
        cur = []
        scans.append(cur)
    if cur is not None:
        cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
s = scans[k]
t0 = prev = s[0][0]
for a, b, n in s:
    print(f"{(a - t0) / 1000:8.1f} gap {(a - prev) / 1000:6.1f} dur {(b - a) / 1000:6.1f}  {re.sub(r'fbr::', '', n)[:64]}")
    prev = max(prev, b)
print(f"next scan's first dispatch at {(scans[k + 1][0][0] - t0) / 1000:.1f} us")
