#!/usr/bin/env python3
"""Vector-memory pipeline of the path kernels from one rocprofv3 pass:
`rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ
TCP_TCP_LATENCY TCP_TCC_READ_REQ_LATENCY GRBM_GUI_ACTIVE -- python3 bench.py ...`
(2 TA + 4 TCP + 1 GRBM counters; rocprofv3 serialises the pass's dispatches).

Per launcher (bench.py's kernel families), per launch:
  ta_busy        TA_TA_BUSY / (256 TA units x duration x f_clk): how much of the time the texture
                 address units (one per CU) are busy -- near 1 means the scattered loads, not the
                 VALU, set the pace
  read_waves     TA_FLAT_READ_WAVEFRONTS: wave-level vector load instructions
  l1_miss        TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES: vL1D read misses sent to L2
  l1_lat, l2_lat TCP_TCP_LATENCY / accesses and TCP_TCC_READ_REQ_LATENCY / L2 requests (cycles)

usage: mem_pmc.py COUNTER_COLLECTION.csv [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict

FAMILIES = [("project", r"k_project\b"), ("extract", r"k_rowcount|k_compact"), ("features", r"k_features"),
            ("voxel_ring", r"k_voxel_ring"), ("concat", r"k_concat"), ("voxel_scan", r"k_voxel_grid"),
            ("gn_knn", r"k_gn_knn"), ("gn_residual", r"k_gn_residual"), ("gn_solve", r"k_gn_solve")]


def main():
    disp = defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[1])):
        fam = next((f for f, rx in FAMILIES if re.search(rx, r["Kernel_Name"])), None)
        if fam is None:
            continue
        d = disp[(fam, r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg = defaultdict(lambda: defaultdict(float))
    for (fam, _), d in disp.items():
        for k, v in d.items():
            agg[fam][k] += v
        agg[fam]["n"] += 1
    res = {"source": sys.argv[1], "kernels": {}}
    print(f"{'kernel':12s} {'disp':>5s} {'avg us':>8s} {'TA busy':>8s} {'reads/launch':>13s} {'L1 miss':>8s} "
          f"{'L1 lat':>7s} {'L2 lat':>7s}")
    for fam, _ in FAMILIES:
        g = agg.get(fam)
        if not g or not g.get("TA_TA_BUSY"):
            continue
        clk = g["GRBM_GUI_ACTIVE"] / 8 / g["dur_ns"] if g.get("GRBM_GUI_ACTIVE") else 2.4
        acc = max(g.get("TCP_TOTAL_CACHE_ACCESSES", 0.0), 1.0)
        l2 = max(g.get("TCP_TCC_READ_REQ", 0.0), 1.0)
        e = {"dispatches": int(g["n"]), "avg_us_alone": g["dur_ns"] / g["n"] / 1e3,
             "ta_busy": g["TA_TA_BUSY"] / (256 * g["dur_ns"] * clk),
             "read_waves_per_launch": g.get("TA_FLAT_READ_WAVEFRONTS", 0.0) / g["n"],
             "l1_miss": g.get("TCP_TCC_READ_REQ", 0.0) / acc,
             "l1_latency": g.get("TCP_TCP_LATENCY", 0.0) / acc, "l2_latency": g.get("TCP_TCC_READ_REQ_LATENCY", 0.0) / l2}
        res["kernels"][fam] = e
        print(f"{fam:12s} {e['dispatches']:5d} {e['avg_us_alone']:8.1f} {e['ta_busy']:8.3f} "
              f"{e['read_waves_per_launch']:13.4g} {e['l1_miss']:8.3f} {e['l1_latency']:7.1f} {e['l2_latency']:7.1f}")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
