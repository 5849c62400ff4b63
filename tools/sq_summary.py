#!/usr/bin/env python3
"""Per-kernel issue / wait mix and VALU-issue fraction from a rocprofv3 SQ counter pass.

Input: the counter_collection.csv of one `rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES` run (rocprofv3
serialises the dispatches of a counter pass, so every kernel runs alone).  Per kernel family:

  wave-state mix    ACTIVE_INST_ANY / WAIT_INST_ANY / WAIT_ANY as shares of WAVE_CYCLES (disjoint,
                    MI355X_MICROARCH.md "rocprofv3 PMC slots"): issuing, waiting to issue, parked on
                    memory / barriers
  VALU busy         4 * ACTIVE_INST_VALU (quad-cycles) / (1024 SIMDs * duration * f_clk)
  VALU issue        2 * INSTS_VALU / (1024 SIMDs * duration * f_clk): a wave64 VALU instruction
                    occupies a SIMD's issue for 2 cycles at best (v_fma_f32 throughput), so this is
                    the fraction of the chip's peak VALU issue slots the kernel filled

f_clk defaults to 2.4 GHz (the peak engine clock; under load the chip runs lower, so both VALU
fractions are lower bounds).

usage: sq_summary.py COUNTER_COLLECTION.csv [--clock-ghz 2.4]
"""
import argparse
import csv
import re
from collections import defaultdict

FAMILIES = [("project", r"k_project\b"), ("extract", r"k_rowcount|k_compact"), ("features", r"k_features"),
            ("voxel_ring", r"k_voxel_ring"), ("concat", r"k_concat"), ("voxel_scan", r"k_voxel_grid"),
            ("gn_knn", r"k_gn_knn"), ("gn_residual", r"k_gn_residual"), ("gn_solve", r"k_gn_solve")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--clock-ghz", type=float, default=2.4)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    disp = defaultdict(dict)  # (family, dispatch id) -> counters + duration
    for r in csv.DictReader(open(a.csv)):
        fam = next((f for f, rx in FAMILIES if re.search(rx, r["Kernel_Name"])), None)
        if fam is None:
            continue
        d = disp[(fam, r["Dispatch_Id"])]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg = defaultdict(lambda: defaultdict(float))
    for (fam, _), d in disp.items():
        for k, v in d.items():
            agg[fam][k] += v
        agg[fam]["dispatches"] += 1
    print(f"{'kernel':12s} {'disp':>5s} {'avg us':>8s} {'issuing':>8s} {'wait-iss':>8s} {'parked':>8s} "
          f"{'VALU busy':>9s} {'VALU issue':>10s} {'SALU/VALU':>9s}")
    for fam, _ in FAMILIES:
        g = agg.get(fam)
        if not g or not g.get("SQ_WAVE_CYCLES"):
            continue
        wc = g["SQ_WAVE_CYCLES"]
        cyc = g["dur_ns"] * a.clock_ghz
        busy = 4.0 * g["SQ_ACTIVE_INST_VALU"] / (a.simds * cyc)
        issue = 2.0 * g["SQ_INSTS_VALU"] / (a.simds * cyc)
        print(f"{fam:12s} {int(g['dispatches']):5d} {g['dur_ns'] / g['dispatches'] / 1e3:8.1f} "
              f"{g['SQ_ACTIVE_INST_ANY'] / wc:8.3f} {g['SQ_WAIT_INST_ANY'] / wc:8.3f} {g['SQ_WAIT_ANY'] / wc:8.3f} "
              f"{busy:9.3f} {issue:10.3f} {g['SQ_INSTS_SALU'] / max(g['SQ_INSTS_VALU'], 1):9.2f}")


if __name__ == "__main__":
    main()
