#!/usr/bin/env python3
"""What the path kernels wait on: per-launcher wave-state and instruction-mix decomposition from
rocprofv3 SQ passes of the bench workload -> JSON + a table.

Passes (each its own rocprofv3 run; rocprofv3 serialises a counter pass's dispatches, so every
kernel runs alone):
  A  SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
     SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
  B  SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_SMEM
     SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE

Per launcher (bench.py's kernel families), per launch:
  wave cycles split into issuing (ACTIVE_INST_ANY), waiting to issue (WAIT_INST_ANY: dependency /
  pipe stalls, of which WAIT_INST_LDS is the LDS-issue part) and parked (WAIT_ANY: s_waitcnt on
  memory / LDS returns and barriers) -- disjoint (MI355X_MICROARCH.md, rocprofv3 PMC slots);
  active-cycle shares of VALU / SALU / LDS / VMEM; instruction counts; VALU issue fraction
  = INSTS_VALU / (duration * f_clk * 1024 SIMDs / cycles-per-wave64-VALU-instruction) with the
  measured peak of profiles/valu_calib.json.

usage: sq_decomp.py PASS_A.csv PASS_B.csv [out.json] [--calib profiles/valu_calib.json] [--config C2]
                    [--batch 1024]
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

FAMILIES = [("project", r"k_project\b"), ("extract", r"k_rowcount|k_compact"), ("features", r"k_features"),
            ("voxel_ring", r"k_voxel_ring"), ("concat", r"k_concat"), ("voxel_scan", r"k_voxel_grid"),
            ("gn_knn", r"k_gn_knn"), ("gn_residual", r"k_gn_residual"), ("gn_solve", r"k_gn_solve")]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(path):
    disp = defaultdict(dict)
    for r in csv.DictReader(open(path)):
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
        agg[fam]["dispatches"] += 1
    return agg


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    calib = os.path.join(REPO, "profiles", "valu_calib.json")
    if "--calib" in sys.argv:
        calib = sys.argv[sys.argv.index("--calib") + 1]
        args.remove(calib)
    meta = {}
    for key, conv in (("--config", str), ("--batch", int)):
        if key in sys.argv:
            v = sys.argv[sys.argv.index(key) + 1]
            args.remove(v)
            meta[key[2:]] = conv(v)
    a, b = load(args[0]), load(args[1])
    out = args[2] if len(args) > 2 else None
    peak = 1024 * 2.4 / 2.0
    if os.path.exists(calib):
        peak = json.load(open(calib)).get("measured_peak_ginst_per_s", peak)
    res = {**meta, "valu_peak_ginst_per_s": peak, "sources": args[:2], "kernels": {}}
    hdr = (f"{'kernel':12s} {'disp':>5s} {'avg us':>8s} {'issue':>6s} {'w-iss':>6s} {'(lds)':>6s} {'parked':>6s} | "
           f"{'VALU':>5s} {'SALU':>5s} {'LDS':>5s} {'VMEM':>5s} | {'VALU/launch':>11s} {'SALU/V':>6s} {'LDS/V':>6s} "
           f"{'VMEM/V':>6s} {'BR/V':>5s} {'bankc/LDS':>9s} {'VALU iss':>8s}")
    print(hdr)
    for fam, _ in FAMILIES:
        ga, gb = a.get(fam), b.get(fam)
        if not ga or not gb or not ga.get("SQ_WAVE_CYCLES"):
            continue
        n = ga["dispatches"]
        wc = ga["SQ_WAVE_CYCLES"]
        act = ga["SQ_ACTIVE_INST_ANY"]
        clk = gb["GRBM_GUI_ACTIVE"] / 8 / gb["dur_ns"] if gb.get("GRBM_GUI_ACTIVE") else 2.4
        v = gb["SQ_INSTS_VALU"]
        e = {
            "dispatches": int(n), "avg_us_alone": ga["dur_ns"] / n / 1e3,
            "wave_state": {"issuing": act / wc, "waiting_to_issue": ga["SQ_WAIT_INST_ANY"] / wc,
                           "parked_waitcnt_or_barrier": ga["SQ_WAIT_ANY"] / wc},
            "active_share": {k: ga[f"SQ_ACTIVE_INST_{c}"] / act for k, c in
                             (("valu", "VALU"), ("salu", "SCA"), ("lds", "LDS"), ("vmem", "VMEM"))},
            "insts_per_launch": {k: gb[f"SQ_INSTS_{c}"] / n for k, c in
                                 (("valu", "VALU"), ("salu", "SALU"), ("lds", "LDS"), ("vmem", "VMEM"),
                                  ("branch", "BRANCH"), ("smem", "SMEM"))},
            "lds_bank_conflict_per_lds_inst": gb["SQ_LDS_BANK_CONFLICT"] / max(gb["SQ_INSTS_LDS"], 1.0),
            "eff_clock_ghz": clk,
            "valu_issue_frac_alone": v / (gb["dur_ns"] * 1e-9) / 1e9 / peak,
        }
        # WAIT_INST_LDS comes from pass B (same workload, so pass A's wave cycles are its denominator)
        e["wave_state"]["waiting_to_issue_lds"] = gb["SQ_WAIT_INST_LDS"] / wc
        res["kernels"][fam] = e
        ws, sh, ip = e["wave_state"], e["active_share"], e["insts_per_launch"]
        print(f"{fam:12s} {int(n):5d} {e['avg_us_alone']:8.1f} {ws['issuing']:6.3f} {ws['waiting_to_issue']:6.3f} "
              f"{ws['waiting_to_issue_lds']:6.3f} {ws['parked_waitcnt_or_barrier']:6.3f} | {sh['valu']:5.2f} "
              f"{sh['salu']:5.2f} {sh['lds']:5.2f} {sh['vmem']:5.2f} | {ip['valu']:11.4g} {ip['salu'] / ip['valu']:6.2f} "
              f"{ip['lds'] / ip['valu']:6.3f} {ip['vmem'] / ip['valu']:6.3f} {ip['branch'] / ip['valu']:5.2f} "
              f"{e['lds_bank_conflict_per_lds_inst']:9.2f} {e['valu_issue_frac_alone']:8.3f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
