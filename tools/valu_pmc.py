#!/usr/bin/env python3
"""Per-launch VALU work of the path kernels from a rocprofv3 SQ counter pass -> profiles/valu_pmc.json.

Input: the counter_collection.csv of `rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py ...` (one pass: 4 SQ + 1 GRBM counters; rocprofv3
serialises a counter pass's dispatches, so every kernel runs alone).  Per launcher (bench.py's
kernel families; a launcher of two kernels counts its calls once):

  insts_valu_per_launch   SQ_INSTS_VALU summed over the launcher's dispatches / calls: wave-level
                          VALU instructions, a property of the work (the same under stream overlap)
  valu_cycles_per_launch  4 * SQ_ACTIVE_INST_VALU (quad-cycles) / calls: SIMD cycles the VALU was busy
                          with the launch's instructions (multi-cycle ones counted in full)
  valu_busy_alone         4 * SQ_ACTIVE_INST_VALU (quad-cycles) / (1024 SIMDs * cycles), cycles =
                          duration * effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration,
                          MI355X_MICROARCH.md "DVFS give-back"): VALU-busy of the kernel running alone
  eff_clock_ghz           that effective clock

bench.py turns valu_cycles_per_launch into the live VALU-busy fraction of a launch (the VALU roofline:
1024 SIMDs x 2.4 GHz of VALU cycles per second).  Every wave64 VALU instruction of these kernels
counts 4 cycles (valu_cycles / insts = 4.0-4.2: none is packed f32, whose 2-lane form doubles the
157 TF vector peak).

usage: valu_pmc.py COUNTER_COLLECTION.csv CONFIG BATCH [out.json]
"""
import csv
import json
import re
import sys
from collections import defaultdict

NAMES = {"gn_knn": [r"k_gn_knn"], "gn_residual": [r"k_gn_residual"], "features": [r"k_features"],
         "voxel_ring": [r"k_voxel_ring"], "voxel_scan": [r"k_voxel_grid"], "concat": [r"k_concat"],
         "project": [r"k_project\b"], "extract": [r"k_compact", r"k_rowcount"], "gn_solve": [r"k_gn_solve"]}
SIMDS = 1024
XCDS = 8


def main():
    path, cfg, batch = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else None
    disp = defaultdict(dict)  # (launcher, symbol index, dispatch id) -> counters, duration
    for r in csv.DictReader(open(path)):
        for key, rxs in NAMES.items():
            for i, rx in enumerate(rxs):
                if re.search(rx, r["Kernel_Name"]):
                    d = disp[(key, i, r["Dispatch_Id"])]
                    d[r["Counter_Name"]] = float(r["Counter_Value"])
                    d["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(lambda: defaultdict(int))
    for (key, i, _), d in disp.items():
        for k, v in d.items():
            agg[key][k] += v
        calls[key][i] += 1
    res = {"config": cfg, "batch": batch, "simds": SIMDS, "peak_issue_ginst_per_s": SIMDS * 2.4 / 2.0,
           "source": path, "kernels": {}}
    print(f"{'kernel':12s} {'calls':>6s} {'avg us':>9s} {'VALU inst/launch':>17s} {'busy alone':>10s} {'clk GHz':>8s}")
    for key in NAMES:
        g = agg.get(key)
        if not g or "SQ_INSTS_VALU" not in g:
            continue
        n = max(calls[key].values())
        clk = g["GRBM_GUI_ACTIVE"] / XCDS / g["dur_ns"] if g.get("GRBM_GUI_ACTIVE") else 2.4
        busy = 4.0 * g["SQ_ACTIVE_INST_VALU"] / (SIMDS * g["dur_ns"] * clk)
        ent = {"calls": n, "avg_us_alone": g["dur_ns"] / n / 1e3, "insts_valu_per_launch": g["SQ_INSTS_VALU"] / n,
               "valu_cycles_per_launch": 4.0 * g["SQ_ACTIVE_INST_VALU"] / n,
               "valu_busy_alone": busy, "eff_clock_ghz": clk,
               "wave_cycles_per_launch": g.get("SQ_WAVE_CYCLES", 0.0) * 4.0 / n}
        res["kernels"][key] = ent
        print(f"{key:12s} {n:6d} {ent['avg_us_alone']:9.1f} {ent['insts_valu_per_launch']:17.4g} {busy:10.3f} {clk:8.2f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
