#!/usr/bin/env python3
"""Per-kernel-name totals of a rocprofv3 --pmc counter CSV (every counter of the pass), per dispatch.
usage: pmc_by_kernel.py COUNTER_COLLECTION.csv [name-regex]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    rx = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    disp = defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"]
        if rx and not rx.search(n):
            continue
        d = disp[(n, r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["dur_us"] = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3
    agg = defaultdict(lambda: defaultdict(float))
    for (n, _), d in disp.items():
        for k, v in d.items():
            agg[n][k] += v
        agg[n]["n"] += 1
    for n, g in sorted(agg.items(), key=lambda t: -t[1]["dur_us"]):
        c = g["n"]
        short = re.sub(r"\(.*", "", n)[:90]
        print(f"{short}  dispatches {int(c)}  " + "  ".join(f"{k} {v / c:.4g}" for k, v in sorted(g.items()) if k != "n"))


if __name__ == "__main__":
    main()
