"""Host-side cost of a batch step: wall ms per step, the fbr_batch_launch call's host time and the
part of it spent waiting for GN flags, kernel launches per step.  usage: batch_host.py B [steps] [cfg]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from feature_base_pointcloud_registration_amd import api, synth  # noqa: E402

B = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = sys.argv[3] if len(sys.argv) > 3 else "C2"
P = synth.config_params(cfg, max_batch=B)
jobs = synth.make_jobs(cfg, B, base_seed=1000)
with api.Context(P) as c:
    c.set_map(*synth.config_map(cfg))
    c.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]).astype(np.float32))
    for _ in range(5):
        c.batch_launch()
    c.batch_wait()
    api.debug_counters(reset=True)
    api.batch_times(reset=True)
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(steps):
        c.batch_launch()
    c.batch_wait()
    wall = time.perf_counter() - t0
    cpu = time.process_time() - c0
    launch_s, spin_s = api.batch_times()
    launches, syncs, polls = api.debug_counters()
print(f"B={B} {cfg}: {1e3 * wall / steps:.3f} ms/step ({B * steps / wall:.0f} scans/s); launch call {1e3 * launch_s / steps:.3f} ms/step "
      f"of which flag wait {1e3 * spin_s / steps:.3f}; process cpu {1e3 * cpu / steps:.3f} ms/step; "
      f"launches/step {launches / steps:.1f}, polls/step {polls / steps:.1f}")
