"""World-size-2 gloo rehearsal of the multi-GPU path: job sharding + the pose-record all-gather."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_q):
    import torch
    import torch.distributed as dist
    from feature_base_pointcloud_registration_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    per_rank = 5
    seeds = shard.job_seeds(rank, world, per_rank)
    poses = np.array([[s, s + 0.5, -s, 1.0 * rank, 2.0, 3.0] for s in seeds], np.float32)
    rec = shard.encode_records(poses, iterations=[s % 30 for s in seeds], status=[rank] * per_rank)
    allrec = shard.gather_records(dist, torch.from_numpy(rec), world)
    out_q.put((rank, allrec.numpy()))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_shard_and_gather():
    import torch.multiprocessing as mp
    from feature_base_pointcloud_registration_amd import shard
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=90) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert np.array_equal(results[0], results[1])
    poses, iters, status = shard.decode_records(results[0])
    seeds = shard.job_seeds(0, world, 5) + shard.job_seeds(1, world, 5)
    assert seeds == list(range(1000, 1010))  # contiguous, disjoint blocks
    assert poses[:, 0].tolist() == [float(s) for s in seeds]
    assert iters.tolist() == [s % 30 for s in seeds]
    assert status.tolist() == [0] * 5 + [1] * 5


def test_job_block_strong_split_and_unpad():
    from feature_base_pointcloud_registration_amd import shard
    blocks = [shard.job_block(r, 8, 1024) for r in range(8)]  # C4: 1024 jobs over 8 GPUs
    assert blocks == [(128 * r, 128 * (r + 1)) for r in range(8)]
    blocks = [shard.job_block(r, 3, 10) for r in range(3)]
    assert blocks[0][0] == 0 and blocks[-1][1] == 10 and all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
    counts = [b - a for a, b in blocks]
    assert sorted(counts) == [3, 3, 4]
    pad = max(counts)
    g = np.full((3, pad, shard.RECORD_FLOATS), -1.0, np.float32)
    for r, (a, b) in enumerate(blocks):
        g[r, :b - a, 0] = np.arange(a, b)
    flat = shard.unpad_records(g.reshape(-1), counts)
    assert flat.reshape(-1, shard.RECORD_FLOATS)[:, 0].tolist() == list(range(10))


def test_record_roundtrip():
    from feature_base_pointcloud_registration_amd import shard
    p = np.random.default_rng(0).standard_normal((7, 6)).astype(np.float32)
    it = np.arange(7, dtype=np.int32)
    st = np.array([0, 1, 0, 2, 0, 0, 1], np.int32)
    p2, it2, st2 = shard.decode_records(shard.encode_records(p, it, st))
    assert np.array_equal(p, p2) and np.array_equal(it, it2) and np.array_equal(st, st2)


def _run_bench(nproc, extra, tmp_path, tag):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = str(tmp_path / f"records_{tag}.npy")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(repo, "bench.py"),
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dist", "--records-out", out, *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), np.load(out)


@pytest.mark.gpu
def test_bench_world2_strong_split_matches_world1(tmp_path):
    """C4's sharded path with two registering ranks (both on the box's one GPU, gloo process group):
    a strong split of 24 jobs into two contiguous blocks gathers records bit-identical to one rank
    running all 24 (the jobs are independent; sub-batching differs between the runs)."""
    r2, rec2 = _run_bench(2, ["--total-jobs", "24", "--backend", "gloo", "--same-device"], tmp_path, "w2")
    r1, rec1 = _run_bench(1, ["--total-jobs", "24", "--backend", "gloo"], tmp_path, "w1")
    assert r2["n_gpus"] == 2 and r2["scaling"] == "strong" and r2["config"]["jobs_per_step"] == 24
    assert r2["records_check"] == {"jobs": 24, "mismatched_words": 0}
    assert r1["records_check"] == {"jobs": 24, "mismatched_words": 0}
    assert rec1.shape == rec2.shape == (24 * 8,)
    assert np.array_equal(rec1.view(np.int32), rec2.view(np.int32))
    _, _, status = __import__("feature_base_pointcloud_registration_amd.shard", fromlist=["x"]).decode_records(rec1)
    assert (status == 0).all()


@pytest.mark.gpu
def test_bench_rccl_path_one_rank(tmp_path):
    """The multi-GPU bench path (torch.distributed.run launch, RCCL process group, device-side
    pose-record export, all_gather) end to end on the one GPU of the box (world size 1)."""
    import json
    import os
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(repo, "bench.py"), "--steps", "2", "--warmup", "1",
           "--batch", "16", "--no-cpu-baseline", "--dist"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 1 and res["value"] > 0 and res["registration_status_ok"] == 16
    assert res["records_check"] == {"jobs": 16, "mismatched_words": 0}


@pytest.mark.gpu
def test_bench_native_gather_one_rank_matches_torch_path(tmp_path):
    """bench.py --gather native: the pose records go through the library's own RCCL communicator
    (fbr_comm_create / fbr_batch_allgather, two launches behind the newest), torch only broadcasts
    the RCCL id; world 1 on the box's GPU.  The gathered records equal the torch-RCCL path's."""
    rn, recn = _run_bench(1, ["--total-jobs", "16", "--gather", "native"], tmp_path, "native")
    rt, rect = _run_bench(1, ["--total-jobs", "16"], tmp_path, "torch")
    assert rn["records_check"] == {"jobs": 16, "mismatched_words": 0}
    assert "fbr_batch_allgather" in rn["config"]["parallelism"]
    assert np.array_equal(recn.view(np.int32), rect.view(np.int32))


# ------------------------------------------------------------------ native RCCL path (no torch)
def _write_shard_input(path, H, W, cmap, smap, jobs):
    import struct
    with open(path, "wb") as f:
        f.write(struct.pack("<iiiqq", H, W, len(jobs), len(cmap), len(smap)))
        f.write(np.ascontiguousarray(cmap).tobytes())
        f.write(np.ascontiguousarray(smap).tobytes())
        for pts, guess, _ in jobs:
            f.write(np.asarray(guess, np.float32).tobytes())
            f.write(struct.pack("<q", len(pts)))
            f.write(np.ascontiguousarray(pts).tobytes())


def test_native_shard_demo_builds_and_reports_no_device(tmp_path):
    """CPU: the native sharding host (tests/native/shard_demo.cpp: fork one process per rank, fbr_comm_*
    + fbr_batch_allgather over RCCL) builds against the C-ABI; without a GPU fbr_create fails in the
    rank process and the demo exits 3."""
    import subprocess
    from conftest import build_shard_demo, has_gpu
    from feature_base_pointcloud_registration_amd import synth
    if has_gpu():
        pytest.skip("a GPU is visible")
    exe = build_shard_demo()
    H, W = 16, 1800
    inp = tmp_path / "in.bin"
    _write_shard_input(inp, H, W, *synth.config_map("C1"), synth.make_jobs("C1", 2, base_seed=90))
    r = subprocess.run([exe, str(inp), str(tmp_path / "out.bin"), "--ranks", "2"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "fbr_create" in r.stderr


def test_native_shard_demo_thread_mode_reports_no_device(tmp_path):
    """CPU: the one-process multi-device host (shard_demo --threads: one host thread, ctx and RCCL
    rank per device, the communicators made together by fbr_comm_create_local) fails cleanly
    without a GPU: fbr_create fails in the rank threads and the demo exits 3 before any collective."""
    import subprocess
    from conftest import build_shard_demo, has_gpu
    from feature_base_pointcloud_registration_amd import synth
    if has_gpu():
        pytest.skip("a GPU is visible")
    exe = build_shard_demo()
    inp = tmp_path / "in.bin"
    _write_shard_input(inp, 16, 1800, *synth.config_map("C1"), synth.make_jobs("C1", 2, base_seed=91))
    r = subprocess.run([exe, str(inp), str(tmp_path / "out.bin"), "--ranks", "2", "--threads"], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "fbr_create" in r.stderr


def test_comm_create_local_rejects_bad_arguments():
    """CPU: fbr_comm_create_local validates before touching RCCL or a device: null outputs / contexts,
    no ranks, no jobs -> FBR_ERR_INVALID_ARG."""
    import ctypes
    from feature_base_pointcloud_registration_amd import api
    L = api.lib()
    out = (ctypes.c_void_p * 2)()
    ctxs = (ctypes.c_void_p * 2)()  # null contexts
    assert L.fbr_comm_create_local(None, ctxs, 2, 8) == -1
    assert L.fbr_comm_create_local(out, None, 2, 8) == -1
    assert L.fbr_comm_create_local(out, ctxs, 0, 8) == -1
    assert L.fbr_comm_create_local(out, ctxs, 2, 0) == -1
    assert L.fbr_comm_create_local(out, ctxs, 2, 8) == -1  # null ctx entries
    assert out[0] is None and out[1] is None


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_rccl_thread_mode_world1_matches_batch_results(tmp_path):
    """GPU, one process with one host thread per device (the box has one device, so world 1): the
    communicator comes from fbr_comm_create_local (ncclGroupStart / ncclCommInitRank per device /
    ncclGroupEnd), the thread stages a C2 batch, runs three pipelined launches and all-gathers each;
    the records equal the rank's fbr_batch_results (inside the demo) and the process-mode run of
    the same jobs, bit for bit."""
    import subprocess
    from conftest import build_shard_demo
    from feature_base_pointcloud_registration_amd import synth
    exe = build_shard_demo()
    H, W = synth.CONFIGS["C2"][:2]
    cmap, smap = synth.config_map("C2")
    jobs = synth.make_jobs("C2", 8, base_seed=4300)
    inp = tmp_path / "in.bin"
    _write_shard_input(inp, H, W, cmap, smap, jobs)
    recs = []
    for mode in (["--threads"], []):
        out = tmp_path / f"out{len(mode)}.bin"
        r = subprocess.run([exe, str(inp), str(out), "--ranks", "1", "--launches", "3", *mode], capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, (mode, r.returncode, r.stderr[-2000:])
        recs.append(np.fromfile(out, np.float32))
    assert recs[0].shape == recs[1].shape == (8 * 8,)
    assert np.array_equal(recs[0].view(np.int32), recs[1].view(np.int32))


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_native_rccl_allgather_world1_matches_batch_results(tmp_path):
    """GPU, world 1 (RCCL refuses two ranks on one device, and the box has one): the native host
    stages a C2 batch, runs three pipelined launches and all-gathers each launch's records through
    fbr_comm_create / fbr_batch_allgather; the gathered records equal the rank's fbr_batch_results
    (checked inside the demo, exit 4 otherwise) and an in-process run of the same jobs, bit for
    bit, and a job over the feature capacity is not involved (every status 0)."""
    import subprocess
    from conftest import build_shard_demo
    from feature_base_pointcloud_registration_amd import api, shard, synth
    from feature_base_pointcloud_registration_amd.fbr_types import default_params
    exe = build_shard_demo()
    H, W = synth.CONFIGS["C2"][:2]
    cmap, smap = synth.config_map("C2")
    jobs = synth.make_jobs("C2", 12, base_seed=4100)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    _write_shard_input(inp, H, W, cmap, smap, jobs)
    r = subprocess.run([exe, str(inp), str(out), "--ranks", "1", "--launches", "3"], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    rec = np.fromfile(out, np.float32)
    assert rec.shape == (12 * shard.RECORD_FLOATS,)
    P = default_params(H, W, max_batch=12, max_points_per_scan=max(len(j[0]) for j in jobs))
    with api.Context(P) as ctx:
        ctx.set_map(cmap, smap)
        ctx.batch_stage([j[0] for j in jobs], np.stack([j[1] for j in jobs]))
        ctx.batch_launch()
        ctx.batch_wait()
        p, s = ctx.batch_results()
    mine = shard.encode_records(p, s["iterations"], s["status"])
    assert np.array_equal(rec.view(np.int32), mine.view(np.int32))
    _, iters, status = shard.decode_records(rec)
    assert (status == 0).all() and (iters > 0).all()
