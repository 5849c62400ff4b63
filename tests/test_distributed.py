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


def test_record_roundtrip():
    from feature_base_pointcloud_registration_amd import shard
    p = np.random.default_rng(0).standard_normal((7, 6)).astype(np.float32)
    it = np.arange(7, dtype=np.int32)
    st = np.array([0, 1, 0, 2, 0, 0, 1], np.int32)
    p2, it2, st2 = shard.decode_records(shard.encode_records(p, it, st))
    assert np.array_equal(p, p2) and np.array_equal(it, it2) and np.array_equal(st, st2)
