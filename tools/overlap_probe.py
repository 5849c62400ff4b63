"""Diagnostic: throughput of one 128-job context vs two 64-job contexts driven from two host
threads (independent HIP streams overlapping on the device)."""
import os
import sys
import threading
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402
from feature_base_pointcloud_registration_amd.fbr_types import default_params  # noqa: E402

B = 128
jobs = synth.make_jobs("C2", B)
cmap = synth.config_map("C2")


def make(n, j0):
    ctx = api.Context(default_params(64, 1800, max_batch=n))
    ctx.set_map(*cmap)
    ctx.batch_stage([j[0] for j in jobs[j0:j0 + n]], np.stack([j[1] for j in jobs[j0:j0 + n]]))
    return ctx


def run(ctxs, steps):
    def worker(c):
        for _ in range(steps):
            c.batch_launch()
        c.batch_wait()
    for c in ctxs:  # warm
        c.batch_launch(); c.batch_wait()
    t0 = time.perf_counter()
    ts = [threading.Thread(target=worker, args=(c,)) for c in ctxs]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return time.perf_counter() - t0


one = [make(B, 0)]
dt1 = run(one, 20)
print(f"1 x {B} jobs: {20 * B / dt1:.0f} scans/s")
for parts in (2, 4):
    n = B // parts
    ctxs = [make(n, k * n) for k in range(parts)]
    dt = run(ctxs, 20)
    print(f"{parts} x {n} jobs (threads): {20 * B / dt:.0f} scans/s")
    for c in ctxs:
        c.close()
