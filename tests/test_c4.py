"""C4 (BASELINE.json configs[3]) at its own size: 1,024 independent 64x1800 scan-to-map jobs.

* One 1,024-job C2 batch on one GPU: properties on every job, and 16 jobs spread over the batch
  against the CPU oracle (iterations, n_sel, pose within 1e-4).
* The strong split of the same 1,024 jobs over 8 ranks (128 per rank, C4's per-GPU share), all on
  the box's one GPU with a gloo group: the gathered pose records equal a world-1 run bit for bit.
  The jobs are independent (imageProjection.cpp:206-218 is the only cross-scan dependency and C4
  removes it), so any difference would be a sharding or buffer-reuse bug.
"""
import os

import numpy as np
import pytest

import pyoracle as O
from feature_base_pointcloud_registration_amd import api, shard, synth
from feature_base_pointcloud_registration_amd.fbr_types import default_params
from test_distributed import _run_bench

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4
C4_JOBS = 1024


def _close(p, q):
    p, q = np.asarray(p, np.float64), np.asarray(q, np.float64)
    return max(np.abs(p[3:] - q[3:]).max(), np.abs(np.angle(np.exp(1j * (p[:3] - q[:3])))).max())


@pytest.mark.timeout(900)
def test_c4_full_batch_1024_jobs():
    H, W = synth.CONFIGS["C2"][:2]
    P = default_params(H, W, max_batch=C4_JOBS)
    cmap, smap = synth.config_map("C2")
    jobs = synth.make_jobs("C2", C4_JOBS, base_seed=1000)  # job j uses seed 1000 + j
    scans = [j[0] for j in jobs]
    guesses = np.stack([j[1] for j in jobs]).astype(np.float32)
    gts = np.stack([j[2] for j in jobs])
    with api.Context(P) as ctx:
        ctx.set_map(cmap, smap)
        ctx.batch_stage(scans, guesses)
        ctx.batch_launch()
        ctx.batch_wait()
        poses, stats = ctx.batch_results()
    # every job: registered, converged, near ground truth, against the ~100k-point local map
    assert (stats["status"] == 0).all()
    assert (stats["converged"] == 1).all()
    assert np.abs(poses[:, 3:] - gts[:, 3:]).max() < 0.05
    m_local = stats["n_corner_map"] + stats["n_surf_map"]
    assert m_local.min() > 60000 and m_local.mean() > 80000
    assert (stats["n_points"] <= np.array([len(s) for s in scans])).all()
    # 16 jobs spread over the whole batch (every sub-batch, first and last job) against the oracle
    pick = sorted(set(np.linspace(0, C4_JOBS - 1, 16).round().astype(int).tolist()))
    omap = O.Map(P, cmap, smap)
    for j in pick:
        po, so = O.Stream(P).process_scan(omap, scans[j], 0.0, guesses[j], n_threads=8)
        assert so["status"] == 0
        assert (int(stats["iterations"][j]), int(stats["n_sel"][j])) == (so["iterations"], so["n_sel"]), j
        for f in ("n_points", "n_corner", "n_corner_map", "n_surf_map"):
            assert stats[f][j] == so[f], (j, f)
        assert _close(poses[j], po) <= POSE_TOL, (j, poses[j], po)


@pytest.mark.timeout(900)
def test_c4_strong_split_world8_matches_world1(tmp_path):
    """bench.py under torch.distributed.run: 1,024 jobs split into 8 contiguous blocks of 128 (each
    rank a 128-job context on device 0, gloo group) against one rank running all 1,024."""
    common = ["--total-jobs", str(C4_JOBS), "--backend", "gloo", "--latency", "0", "--ingest", "0",
              "--exact-line", "0", "--profile", "off"]
    r8, rec8 = _run_bench(8, common + ["--same-device"], tmp_path, "w8")
    r1, rec1 = _run_bench(1, common, tmp_path, "w1")
    assert r8["n_gpus"] == 8 and r8["scaling"] == "strong"
    assert r8["config"]["jobs_per_step"] == C4_JOBS and r8["config"]["jobs_per_gpu_per_step"] == C4_JOBS // 8
    assert r8["records_check"] == {"jobs": C4_JOBS, "mismatched_words": 0}
    assert r1["records_check"] == {"jobs": C4_JOBS, "mismatched_words": 0}
    assert rec1.shape == rec8.shape == (C4_JOBS * shard.RECORD_FLOATS,)
    assert np.array_equal(rec1.view(np.int32), rec8.view(np.int32))
    _, iters, status = shard.decode_records(rec1)
    assert (status == 0).all() and (iters > 0).all()


_PIPE_CHILD = r"""
import sys, json
import numpy as np
import torch  # torch's HIP runtime first: the library shares it (bench.py does the same)
torch.cuda.init()
sys.path.insert(0, %(repo)r)
from feature_base_pointcloud_registration_amd import api, shard, synth
from feature_base_pointcloud_registration_amd.fbr_types import default_params
H, W = synth.CONFIGS["C2"][:2]
B = 24
P = default_params(H, W, max_batch=B, pipeline_depth=%(pipe)d)
jobs = synth.make_jobs("C2", B, base_seed=6000)
buf = torch.zeros((4, B * shard.RECORD_FLOATS), dtype=torch.float32, device="cuda:0")
with api.Context(P) as ctx:
    ctx.set_map(*synth.config_map("C2"))
    ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
    ctx.batch_launch()
    ctx.batch_wait()
    p0, s0 = ctx.batch_results()
    ids = []

    def drain():  # every launch whose records are ready, oldest first
        while True:
            lid = ctx.batch_export_ready(buf[min(len(ids), 3)].data_ptr())[0]
            if lid < 0:
                return
            ids.append(lid)

    for k in range(3):
        ctx.batch_launch()
        drain()
    ctx.batch_flush()
    drain()
    again = ctx.batch_export_ready(buf[3].data_ptr())[0]
    ctx.batch_wait()
    p1, s1 = ctx.batch_results()
    # re-stage a different, smaller batch with job 5 over the feature capacity (diagnostic hook): the
    # launches of the old batch are never handed out again, and the new launch's exported records
    # carry what fbr_batch_results reports for every job (the capacity job: its guess, status 3)
    torch.cuda.synchronize()
    ex0 = [buf[k].cpu().numpy().copy() for k in range(4)]
    jobs2 = synth.make_jobs("C2", 16, base_seed=7000)
    g2 = np.stack([j[1] for j in jobs2]).astype(np.float32)
    ctx.diag_force_capacity_error(5)
    ctx.batch_stage([j[0] for j in jobs2], g2)
    buf.zero_()
    ctx.batch_launch()
    ids2 = []
    while True:
        lid = ctx.batch_export_ready(buf[0].data_ptr())[0]
        if lid < 0:
            break
        ids2.append(lid)
    ctx.batch_flush()
    while True:
        lid = ctx.batch_export_ready(buf[0].data_ptr())[0]
        if lid < 0:
            break
        ids2.append(lid)
    ctx.batch_wait()
    p2, s2 = ctx.batch_results()
    ctx.diag_force_capacity_error(-1)
torch.cuda.synchronize()
rec0 = shard.encode_records(p0, s0["iterations"], s0["status"])
rec2 = shard.encode_records(p2, s2["iterations"], s2["status"])
print(json.dumps({"ids": ids, "again": again, "ids_restaged": ids2,
                  "same_results": bool(np.array_equal(p0.view(np.int32), p1.view(np.int32)) and np.array_equal(s0, s1)),
                  "exports_equal": [bool(np.array_equal(ex0[k].view(np.int32), rec0.view(np.int32))) for k in range(4)],
                  "status_ok": int((s0["status"] == 0).sum()),
                  "restaged_export_equal": bool(np.array_equal(buf[0, :16 * shard.RECORD_FLOATS].cpu().numpy().view(np.int32),
                                                               rec2.view(np.int32))),
                  "cap_status": int(s2["status"][5]), "cap_pose_is_guess": bool(np.array_equal(p2[5], g2[5])),
                  "others_ok": int((np.delete(s2["status"], 5) == 0).sum())}))
"""


@pytest.mark.parametrize("pipe", [2, 3])
def test_pipelined_launches_are_bit_identical_and_export_in_order(pipe):
    """Consecutive fbr_batch_launch calls run fbr_params.pipeline_depth deep (rotating work slots and streams; a
    launch returns once the launch pipe - 1 before it is fully enqueued).  Every launch of the same
    staged batch gives the same bytes, and fbr_batch_export_ready hands out every launch's records
    once, in launch order (-1 while the oldest unexported launch is still being enqueued).  After a
    re-stage only the new batch's launch is handed out, and its records report a job over the
    feature capacity as fbr_batch_results does (guess + FBR_REG_FEATURE_CAPACITY).
    (Child process: torch, which allocates the export buffers, must initialise HIP first.)"""
    import json
    import subprocess
    import sys
    from conftest import REPO
    r = subprocess.run([sys.executable, "-c", _PIPE_CHILD % {"repo": REPO, "pipe": pipe}], capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["ids"] == [0, 1, 2, 3] and d["again"] == -1, d
    assert d["same_results"] and d["exports_equal"] == [True] * 4 and d["status_ok"] == 24, d
    # after a re-stage only the new launch is exported, once, with the capacity rule applied
    assert d["ids_restaged"] == [4], d
    assert d["restaged_export_equal"] and d["cap_status"] == 3 and d["cap_pose_is_guess"] and d["others_ok"] == 15, d
