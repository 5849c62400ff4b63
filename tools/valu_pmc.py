#!/usr/bin/env python3
"""Per-launch VALU work of the path kernels from a rocprofv3 SQ counter pass -> profiles/valu_pmc.json.

Input: the counter_collection.csv of `rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 bench.py ...` (one pass: 4 SQ + 1 GRBM counters; rocprofv3
serialises a counter pass's dispatches, so every kernel runs alone).  Per launcher (bench.py's
kernel families; a launcher of two kernels counts its calls once):

  insts_valu_per_launch   SQ_INSTS_VALU summed over the launcher's dispatches / calls: wave-level
                          VALU instructions, a property of the work (the same under stream overlap)
  valu_issue_alone        those instructions / the serialised duration / the measured issue peak
                          (profiles/valu_calib.json: 1079 G wave64 instr/s of v_fma_f32)
  eff_clock_ghz           GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md "DVFS give-back")

bench.py turns insts_valu_per_launch into the live VALU fraction of a launch.  SQ_ACTIVE_INST_VALU
is not busy time: the calibration's PMC pass shows it counts exactly one quad-cycle per wave64 VALU
instruction at every issue rate (1, 2, 4, 8 waves per SIMD), while the SIMD issues one every ~2.3
cycles with two or more waves; round 4 priced 4 x ACTIVE_INST_VALU as busy cycles, twice the truth.

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
CALIB = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))), "profiles", "valu_calib.json")


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
    peak = 1024 * 2.4 / 2.0
    try:
        peak = json.load(open(CALIB))["measured_peak_ginst_per_s"]
    except Exception:
        pass
    res = {"config": cfg, "batch": batch, "simds": SIMDS, "valu_peak_ginst_per_s": peak, "source": path, "kernels": {}}
    print(f"{'kernel':12s} {'calls':>6s} {'avg us':>9s} {'VALU inst/launch':>17s} {'issue alone':>11s} {'clk GHz':>8s}")
    for key in NAMES:
        g = agg.get(key)
        if not g or "SQ_INSTS_VALU" not in g:
            continue
        n = max(calls[key].values())
        clk = g["GRBM_GUI_ACTIVE"] / XCDS / g["dur_ns"] if g.get("GRBM_GUI_ACTIVE") else 2.4
        issue = g["SQ_INSTS_VALU"] / (g["dur_ns"] * 1e-9) / 1e9 / peak
        ent = {"calls": n, "avg_us_alone": g["dur_ns"] / n / 1e3, "insts_valu_per_launch": g["SQ_INSTS_VALU"] / n,
               "valu_issue_alone": issue, "eff_clock_ghz": clk,
               "wave_cycles_per_launch": g.get("SQ_WAVE_CYCLES", 0.0) * 4.0 / n}
        res["kernels"][key] = ent
        print(f"{key:12s} {n:6d} {ent['avg_us_alone']:9.1f} {ent['insts_valu_per_launch']:17.4g} {issue:11.3f} {clk:8.2f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
