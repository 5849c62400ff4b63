#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv rows per kernel (name prefix) and print per-launch
means, one column per counter.  usage: pmc_summary.py CSV [CSV ...]"""
import csv
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
launches = defaultdict(set)
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"^(void )?(fbr::)?", "", r["Kernel_Name"]).split("(")[0].split("<")[0]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[name].add((path, r.get("Dispatch_Id", r.get("Correlation_Id", ""))))
counters = sorted({c for d in acc.values() for c in d})
print(f"{'kernel':24s} {'n':>5s} " + " ".join(f"{c[-18:]:>18s}" for c in counters))
for k in sorted(acc, key=lambda k: -sum(acc[k].values())):
    n = len(launches[k])
    print(f"{k[:24]:24s} {n:5d} " + " ".join(f"{acc[k].get(c, 0) / n:18.4g}" for c in counters))
