#!/usr/bin/env python3
"""Print the headline of bench.py JSON lines found in the given log files."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        ks = " ".join(f"{k}={v:.3f}" for k, v in sorted(r["kernel_ms_per_step"].items(), key=lambda kv: -kv[1]))
        print(f"{path}: {r['value']:.0f} scans/s {r['ms_per_step']:.3f} ms/step iters={r['config']['mean_gn_iterations']} "
              f"roof={r['roofline']['kernel']}:{r['roofline']['frac']:.4f} | {ks}")
        if "pose_rmse_vs_ref" in r:
            print("   pose_rmse_vs_ref", r["pose_rmse_vs_ref"], "cpu", r["cpu_baseline"]["value"])
