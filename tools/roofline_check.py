#!/usr/bin/env python3
"""Recompute bench.py's roofline fractions from a rocprofv3 --stats kernel summary.

bench.py times every kernel family with the dispatches' own start / end timestamps; rocprofv3's
kernel trace reports the same per-dispatch durations.  This script takes a committed
`*_kernel_stats.csv` and the bench JSON line of the same command and prints, per kernel family,
the bench's average launch time next to rocprofv3's and the HBM fraction each gives for the
bench's algorithmic bytes per launch (bench.py kernel_bytes / DESIGN.md §4), and, where the line
carries them, the VALU-issue fraction each gives for the bench's VALU instructions per launch
(rocprofv3 SQ pass, tools/valu_pmc.py) against the measured issue peak (profiles/valu_calib.json).

With --trace KERNEL_TRACE.csv (the same run's rocprofv3 kernel trace) the rocprofv3 column covers
the timed region only: per launcher, the dispatches after the untimed launches' share (bench.py runs
`warmup` launches, then one profiled launch alone, then the `steps` timed ones; k_project dispatches
count the launches).  The stats summary averages the untimed launches too, which run with fewer
launches beside them, so their kernels are shorter than the overlapped ones the bench times.

usage: roofline_check.py KERNEL_STATS.csv BENCH.json [--trace KERNEL_TRACE.csv] [--peak 8000]
"""
import argparse
import csv
import json


def rocprof_avg_us(rows, symbols):
    """Mean duration of one launcher call: all rows matching any symbol, summed, over the launches
    of the most-called symbol (a launcher of two kernels, e.g. extract = k_rowcount + k_compact,
    counts as one launch of both)."""
    total_ns, calls = 0.0, 0
    for sym in symbols:
        c = 0
        for r in rows:
            if sym in r["Name"]:
                total_ns += float(r["TotalDurationNs"])
                c += int(r["Calls"])
        calls = max(calls, c)
    return (total_ns / calls / 1e3, calls) if calls else (None, 0)


def trace_avg_us(trace_rows, symbols, skip_frac):
    """Mean launcher-call duration from per-dispatch rows, dropping the first skip_frac of each
    symbol's dispatches (in start order)."""
    total_ns, calls = 0.0, 0
    for sym in symbols:
        d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in trace_rows if sym in r["Kernel_Name"])
        d = d[int(round(skip_frac * len(d))):]
        total_ns += sum(e - b for b, e in d)
        calls = max(calls, len(d))
    return (total_ns / calls / 1e3, calls) if calls else (None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("bench_json")
    ap.add_argument("--peak", type=float, default=8000.0, help="GB/s (MI355X HBM3E spec)")
    ap.add_argument("--trace", default=None, help="the same run's kernel_trace.csv: timed region only")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats_csv)))
    with open(a.bench_json) as f:
        line = [l for l in f.read().splitlines() if l.strip().startswith("{")][-1]
    res = json.loads(line)
    roof = res["roofline"]
    trace_rows, skip = None, 0.0
    if a.trace:
        trace_rows = list(csv.DictReader(open(a.trace)))
        nlaunch = sum(1 for r in trace_rows if "k_project" in r["Kernel_Name"])
        skip = (nlaunch - res["steps"]) / nlaunch if nlaunch else 0.0  # warmup + the profiled launch
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import KERNEL_SYMBOLS as symbols
    from bench import VALU_PEAK_GINST
    print(f"{'kernel':12s} {'bytes/launch':>14s} {'bench us':>10s} {'rocprof us':>11s} {'calls':>6s} "
          f"{'bench frac':>10s} {'rocprof frac':>12s} {'bench valu':>10s} {'rocprof valu':>12s}")
    nan = float("nan")
    for k, r in roof["kernels"].items():
        if trace_rows is not None:
            avg, calls = trace_avg_us(trace_rows, symbols.get(k, [k]), skip)
        else:
            avg, calls = rocprof_avg_us(rows, symbols.get(k, [k]))
        bpl = r["bytes_per_launch"]
        rf = bpl / (avg * 1e-6) / 1e9 / a.peak if avg else nan
        vb = r.get("valu_frac", nan)
        vr = r["valu_insts_per_launch"] / (avg * 1e-6) / 1e9 / VALU_PEAK_GINST if avg and "valu_insts_per_launch" in r else nan
        mark = " <- roofline kernel" if k == roof["kernel"] else ""
        print(f"{k:12s} {bpl:14.4g} {r['avg_launch_us']:10.1f} {avg if avg else nan:11.1f} {calls:6d} "
              f"{r['frac']:10.4f} {rf:12.4f} {vb:10.4f} {vr:12.4f}{mark}")
    print(f"bench line: kernel {roof['kernel']} bound {roof.get('bound')} frac {roof['frac']} "
          f"(hbm {roof.get('hbm_frac')}, valu {roof.get('valu_frac')})")


if __name__ == "__main__":
    main()
