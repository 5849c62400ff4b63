"""Multi-GPU sharding of independent registration jobs (config C4).

Scans are independent (scan, guess) pairs against a shared read-only map, so the path shards with no
data-path collective: rank r owns a contiguous block of jobs, keeps its own copy of the map in its
HBM, and the only exchange is one all-gather of the 32-byte pose records
{pose[6] f32, iterations i32, status i32} at the end of each batch (RCCL over xGMI when the backend
is "nccl"; gloo on CPU in the tests).
"""
import numpy as np

RECORD_FLOATS = 8  # 32 bytes per job


def job_seeds(rank, world, per_rank, base=1000):
    """Seeds of the jobs rank `rank` owns: contiguous blocks of `per_rank` (job j uses seed base+j)."""
    assert 0 <= rank < world
    return [base + rank * per_rank + j for j in range(per_rank)]


def job_block(rank, world, total):
    """Strong split of `total` jobs: rank r owns the contiguous block [j0, j1) (sizes differ by at
    most one; the C4 config is 1024 jobs over 8 GPUs = 128 each)."""
    assert 0 <= rank < world and total >= world
    return total * rank // world, total * (rank + 1) // world


def encode_records(poses, iterations, status):
    """numpy [B,6] f32 + [B] i32 + [B] i32 -> flat f32 [B*8] (the layout fbr_batch_export writes)."""
    B = len(poses)
    rec = np.zeros((B, RECORD_FLOATS), np.float32)
    rec[:, :6] = poses
    rec[:, 6] = np.asarray(iterations, np.int32).view(np.float32)
    rec[:, 7] = np.asarray(status, np.int32).view(np.float32)
    return rec.reshape(-1)


def decode_records(flat):
    rec = np.ascontiguousarray(np.asarray(flat, np.float32).reshape(-1, RECORD_FLOATS))
    return rec[:, :6].copy(), rec[:, 6].view(np.int32).copy(), rec[:, 7].view(np.int32).copy()


def gather_records(dist, local, world):
    """All-gather equal-sized flat record tensors from every rank; returns one tensor in rank order."""
    import torch
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local)
    return torch.cat(parts)


def unpad_records(gathered, counts):
    """Rank-ordered records of a gather whose ranks padded their blocks to max(counts) jobs."""
    flat = np.asarray(gathered, np.float32).reshape(len(counts), -1, RECORD_FLOATS)
    return np.concatenate([flat[r, :c] for r, c in enumerate(counts)]).reshape(-1)
