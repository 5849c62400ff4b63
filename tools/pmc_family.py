"""Sum rocprofv3 PMC counters per kernel name over the dispatches of a kernel family.
usage: python3 tools/pmc_family.py NAME_SUBSTRING counter_collection.csv [more.csv ...]"""
import collections
import csv
import sys

fam = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if fam not in name:
            continue
        key = name.split("(")[0]
        tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if path == sys.argv[2]:
            calls[key].add(r["Dispatch_Id"])
for key, c in sorted(tot.items()):
    n = len(calls[key]) or 1
    print(key, "dispatches", n, " ".join(f"{k}={v / 1e6:.2f}M" for k, v in sorted(c.items())))
