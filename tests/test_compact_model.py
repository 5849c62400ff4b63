"""Index model of the cloud-extraction kernels (csrc/k_project.hip k_rowcount + k_compact).

The kernels write every claimed cell of the (job, ring, column) owner image to
rowoff[ring] + choff[ring][chunk] + rank-in-chunk, where the tiles are HB rows x CG columns and
the per-chunk offsets are produced by k_rowcount's 64-column steps.  cloudExtraction
(imageProjection.cpp:642-670) fixes the output order: ring-major, column-minor.  This CPU model
restates the kernels' index arithmetic (tile shapes, chunk-offset writes, the XCD deal of blocks)
and checks, over many (H, W) shapes and owner densities, that every launched tile maps to a
valid job, every chunk offset k_compact reads was written by k_rowcount, and the destinations
are exactly the row-major compaction positions (a permutation inside [0, n_valid)).  The device
kernels themselves are compared bit-exact with the oracle by the GPU tests
(test_gpu_parity.py::test_projection_*).
"""
import numpy as np
import pytest


def compact_tile(H, cells):
    """k_project.hip compact_tile: (HB, CG) for a tile of at most `cells` cells."""
    hb = min(H, 64, cells // 32)
    cg = 32
    while cg < 256 and 2 * cg * hb <= cells:
        cg *= 2
    return hb, cg


def compact_nchunk(cg, W):
    return (W + cg - 1) // cg


def rowcount(claimed, H, W, cg):
    """k_rowcount for one job: per-row counts and the chunk offsets it writes (-1 = never written)."""
    nch = compact_nchunk(cg, W)
    choff = np.full((H, nch), -1, np.int64)
    cnt = np.zeros(H, np.int64)
    for row in range(H):
        run = 0
        for c0 in range(0, W, 64):
            m = claimed[row, c0:c0 + 64]
            if c0 % cg == 0:
                choff[row, c0 // cg] = run
            if (c0 + 32) % cg == 0 and c0 + 32 < W:
                choff[row, (c0 + 32) // cg] = run + int(m[:32].sum())
            run += int(m.sum())
        cnt[row] = run
    return cnt, choff


def compact_destinations(claimed_jobs, H, W, cells):
    """k_compact over B jobs: {(job, row, col): dst} for every claimed cell, tiles dealt as launched."""
    B = len(claimed_jobs)
    HB, CG = compact_tile(H, cells)
    nch = compact_nchunk(CG, W)
    assert HB * CG <= cells and CG in (32, 64, 128, 256)
    nrb = (H + HB - 1) // HB
    tiles = nrb * nch
    groups = (B + 7) // 8
    per_job = [rowcount(cl, H, W, CG) for cl in claimed_jobs]
    out = {}
    seen_tiles = set()
    for b in range(groups * 8 * tiles):  # launch_extract's grid
        x, rest = b % 8, b // 8
        g, t = rest // tiles, rest % tiles
        job = g * 8 + x
        if job >= B:
            continue
        assert (job, t) not in seen_tiles
        seen_tiles.add((job, t))
        rb, ch = t // nch, t % nch
        r0, c0 = rb * HB, ch * CG
        nr, ncl = min(HB, H - r0), min(CG, W - c0)
        cnt, choff = per_job[job]
        base = int(cnt[:r0].sum())
        for r in range(nr):
            assert choff[r0 + r, ch] >= 0, "k_compact reads a chunk offset k_rowcount never wrote"
            rowoff = base + int(cnt[r0:r0 + r].sum()) + int(choff[r0 + r, ch])
            rank = 0
            for c in range(ncl):
                if claimed_jobs[job][r0 + r, c0 + c]:
                    out[(job, r0 + r, c0 + c)] = rowoff + rank
                    rank += 1
    assert len(seen_tiles) == B * tiles
    return out


@pytest.mark.parametrize("H,W", [(1, 1), (1, 31), (2, 300), (4, 900), (8, 512), (16, 900), (16, 1800), (24, 100),
                                 (32, 1024), (40, 77), (48, 2048), (64, 1800), (65, 200), (100, 96), (128, 2048),
                                 (129, 64), (16, 4096)])
@pytest.mark.parametrize("density", [0.0, 0.3, 1.0])
@pytest.mark.parametrize("cells", [512, 1024, 2048])
def test_compaction_index_model(H, W, density, cells):
    rng = np.random.default_rng(H * 10007 + W)
    B = 3 if H * W <= 4096 else 2  # job groups of 8 with a partial last group
    if H * W * B > 300_000:
        B = 1
    jobs = [rng.random((H, W)) < density for _ in range(B)]
    dst = compact_destinations(jobs, H, W, cells)
    for j, cl in enumerate(jobs):
        rows, cols = np.nonzero(cl)  # row-major order = cloudExtraction's order
        got = np.array([dst[(j, r, c)] for r, c in zip(rows, cols)], np.int64)
        assert np.array_equal(got, np.arange(len(rows)))


@pytest.mark.parametrize("cells", [512, 1024, 2048])
def test_tile_shapes_fit_lds(cells):
    for H in range(1, 257):
        HB, CG = compact_tile(H, cells)
        assert HB * CG <= cells and 256 % CG == 0 and CG >= 32
        assert HB <= 64  # rowoff[64] in LDS
        assert 24 * HB * CG <= 48 * 1024  # dynamic LDS of the deskew variant
