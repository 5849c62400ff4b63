"""Summarise tools/ab_libs.sh logs: value and per-kernel ms per step for each variant."""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no bench line", e)
        continue
    k = d.get("kernel_ms_per_step", {})
    ks = " ".join(f"{n}={v:.3f}" for n, v in sorted(k.items(), key=lambda t: -t[1]) if v > 0.01)
    print(f"{f.split('/')[-1]:40s} {d['value']:9.0f} {d['unit']} {d['ms_per_step']:.3f} ms | {ks}")
    kr = d.get("roofline", {}).get("kernels", {})
    if kr:  # timed-region per-launch durations and HBM fractions
        print(" " * 42 + " ".join(f"{n}={v['avg_launch_us']:.0f}us/{v['frac']:.3f}" for n, v in kr.items()))
