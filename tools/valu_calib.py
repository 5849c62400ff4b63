#!/usr/bin/env python3
"""Calibrate the VALU roof on the box (fbr_valu_peak, k_selftest.hip) -> profiles/valu_calib.json.

  valu_calib.py run [OUT.json]      sweep 1 / 2 / 4 / 8 waves per SIMD x {v_fma_f32, v_add_u32,
                                    v_pk_fma_f32}: wave-level G instr/s timed with HIP events
  valu_calib.py pmc CSV IN.json OUT.json
                                    merge a rocprofv3 SQ pass of the same sweep (`rocprofv3 --pmc
                                    SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
                                    GRBM_GUI_ACTIVE -- python3 tools/valu_calib.py run`): per probe
                                    dispatch the counter's quad-cycles per instruction and the
                                    effective clock, i.e. what one SQ_ACTIVE_INST_VALU unit means

The measured issue peak (the best v_fma_f32 rate) is what bench.py prices a kernel's VALU
instructions against (VALU_PEAK_GINST): a kernel's VALU fraction = its wave-level VALU instructions
per launch / its live launch time / that peak.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
KINDS = {0: "v_fma_f32", 1: "v_add_u32", 2: "v_pk_fma_f32"}
WAVES = (1, 2, 4, 8)


def run(out=None):
    from feature_base_pointcloud_registration_amd import api
    res = {"probe": "fbr_valu_peak: 8 independent chains per lane, inline-asm VALU, 32 instructions per round",
           "simds": 1024, "guide_peak_ginst_per_s": 1024 * 2.4 / 2.0, "runs": []}
    for kind, name in KINDS.items():
        for w in WAVES:
            iters = 131072 // w
            g, ms = api.valu_peak(0, w, kind, iters, 5)
            res["runs"].append({"kind": name, "waves_per_simd": w, "iters": iters, "ginst_per_s": round(g, 2),
                                "ms_per_launch": round(ms, 4)})
            print(f"{name:14s} waves/SIMD {w}: {g:8.1f} G wave-instr/s  ({ms:.3f} ms/launch)", flush=True)
    fma = [r["ginst_per_s"] for r in res["runs"] if r["kind"] == "v_fma_f32"]
    res["measured_peak_ginst_per_s"] = max(fma)
    res["measured_vs_guide"] = round(max(fma) / res["guide_peak_ginst_per_s"], 4)
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
    return res


def pmc(path, inp, out):
    res = json.load(open(inp))
    disp = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        m = re.search(r"k_valu_peak<(\d)>", r["Kernel_Name"])
        if not m:
            continue
        d = disp[int(r["Dispatch_Id"])]
        d["kind"] = KINDS[int(m.group(1))]
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    # dispatches come in run order: per (kind, waves) one warm-up + 5 timed launches
    order = sorted(disp)
    runs = res["runs"]
    per = len(order) // max(len(runs), 1)
    for i, r in enumerate(runs):
        ds = [disp[k] for k in order[i * per:(i + 1) * per]][1:]  # skip the warm-up
        if not ds:
            continue
        insts = sum(d["SQ_INSTS_VALU"] for d in ds)
        active = sum(d["SQ_ACTIVE_INST_VALU"] for d in ds)
        dur = sum(d["dur_ns"] for d in ds)
        clk = sum(d.get("GRBM_GUI_ACTIVE", 0.0) for d in ds) / 8 / dur if dur else 0.0
        r["pmc"] = {"active_inst_valu_quads_per_inst": round(active / insts, 4) if insts else None,
                    "valu_cycles_per_inst": round(4.0 * active / insts, 4) if insts else None,
                    "eff_clock_ghz": round(clk, 4),
                    "issue_cycles_per_inst_per_simd": round(1024 * dur * clk / insts, 4) if insts else None,
                    "wave_cycles_per_inst": round(4.0 * sum(d.get("SQ_WAVE_CYCLES", 0.0) for d in ds) / insts, 4)
                    if insts else None}
        print(r["kind"], r["waves_per_simd"], r["pmc"])
    res["pmc_source"] = path
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2] if len(sys.argv) > 2 else None)
    elif sys.argv[1] == "pmc":
        pmc(sys.argv[2], sys.argv[3], sys.argv[4])
