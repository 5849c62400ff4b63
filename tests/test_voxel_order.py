"""PCL VoxelGrid's point order inside a voxel = libstdc++ std::sort's order of the index vector
(voxel_grid.cpp; featureExtraction.h:288-292, mapOptmization.h:251-257, 981-993).

The device reproduces it as "introsort partition phase, then a stable sort by key"
(csrc/fbr_introsort.h).  The CPU test pins that decomposition -- the level-by-level partition
phase with the closed-form __unguarded_partition -- against the host's real std::sort (oracle
probe); the GPU test runs the device emulation (global and LDS variants) against it."""
import numpy as np
import pytest

import pyoracle as O
from feature_base_pointcloud_registration_amd import api


def lg(n):
    return n.bit_length() - 1

def median_to_first(k, v, result, a, b, c):
    def sw(i, j):
        k[i], k[j] = k[j], k[i]; v[i], v[j] = v[j], v[i]
    if k[a] < k[b]:
        if k[b] < k[c]: sw(result, b)
        elif k[a] < k[c]: sw(result, c)
        else: sw(result, a)
    elif k[a] < k[c]: sw(result, a)
    elif k[b] < k[c]: sw(result, c)
    else: sw(result, b)

def heap_sort(k, v, first, last):
    # std::partial_sort(first, last, last) == make_heap + sort_heap, restated (stl_heap.h)
    kk = list(k[first:last]); vv = list(v[first:last]); n = len(kk)
    def adjust(hole, length, val):
        top = hole; second = hole
        while second < (length - 1) // 2:
            second = 2 * (second + 1)
            if kk[second][0] < kk[second - 1][0]: second -= 1
            kk[hole] = kk[second]; hole = second
        if (length & 1) == 0 and second == (length - 2) // 2:
            second = 2 * (second + 1); kk[hole] = kk[second - 1]; hole = second - 1
        parent = (hole - 1) // 2
        while hole > top and kk[parent][0] < val[0]:
            kk[hole] = kk[parent]; hole = parent; parent = (hole - 1) // 2
        kk[hole] = val
    kk = [(kk[i], vv[i]) for i in range(n)]
    if n >= 2:
        parent = (n - 2) // 2
        while True:
            adjust(parent, n, kk[parent])
            if parent == 0: break
            parent -= 1
    last_ = n
    while last_ > 1:
        last_ -= 1
        val = kk[last_]; kk[last_] = kk[0]
        adjust(0, last_, val)
    for i in range(n):
        k[first + i], v[first + i] = kk[i]

def partition(k, v, lo, hi, p):
    # __unguarded_partition(lo, hi, pivot value p) in closed form
    idx = np.arange(lo, hi)
    ks = np.array(k[lo:hi])
    posL = idx[~(ks < p)]
    posR = idx[~(p < ks)][::-1]
    m = min(len(posL), len(posR))
    K = int(np.sum(posL[:m] < posR[:m]))
    assert np.all(posL[:K] < posR[:K])
    for j in range(K):
        x, y = posL[j], posR[j]
        k[x], k[y] = k[y], k[x]; v[x], v[y] = v[y], v[x]
    cut = posL[K] if K < len(posL) else 1 << 60
    if K > 0: cut = min(cut, posR[K - 1])
    return min(cut, hi)

def emulate(keys):
    """The decomposition the device implements, restated serially."""
    n = len(keys)
    k = [int(x) for x in keys]; v = list(range(n))
    frames = [(0, n, 2 * lg(n))] if n > 16 else []
    while frames:  # one level
        nxt = []
        for first, last, depth in frames:
            if depth == 0:
                heap_sort(k, v, first, last); continue
            depth -= 1
            mid = first + (last - first) // 2
            median_to_first(k, v, first, first + 1, mid, last - 1)
            cut = partition(k, v, first + 1, last, k[first])
            for f in ((first, cut, depth), (cut, last, depth)):
                if f[1] - f[0] > 16: nxt.append(f)
        frames = nxt
    order = sorted(range(n), key=lambda i: (k[i], i))  # stable sort by key of the partitioned array
    return np.array([v[i] for i in order])



def key_cases(rng, count, nmax):
    for t in range(count):
        n = int(rng.integers(1, nmax))
        kind = t % 6
        if kind == 0:
            keys = rng.integers(0, max(1, n // 6), n)  # voxel-like: ~6 points per key
        elif kind == 1:
            keys = np.repeat(rng.integers(0, 50, n // 7 + 1), 7)[:n]  # runs of equal keys
        elif kind == 2:
            keys = np.sort(rng.integers(0, 100, n))  # sorted with ties
        elif kind == 3:
            keys = rng.integers(0, 3, n)  # massive ties
        elif kind == 4:  # organ pipe: exhausts introsort's depth limit (heap-sorted frames)
            n = min(n, 3000)
            keys = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]])
        else:
            keys = rng.integers(0, 1 << 30, n)  # distinct-ish
        yield keys.astype(np.uint32)


def test_partition_phase_then_stable_sort_is_std_sort():
    rng = np.random.default_rng(1)
    for keys in key_cases(rng, 48, 1500):
        assert np.array_equal(O.sort_voxel_pairs(keys), emulate(keys)), len(keys)


@pytest.mark.gpu
@pytest.mark.parametrize("lds", [0, 1, 2])
def test_device_voxel_order_is_std_sort(lds):
    rng = np.random.default_rng(2 + lds)
    for keys in key_cases(rng, 120, {0: 60000, 1: 8000, 2: 18432}[lds]):
        assert np.array_equal(api.selftest_voxel_order(keys, lds=lds), O.sort_voxel_pairs(keys)), len(keys)
    for n in {0: (17, 2049, 18432, 18433), 1: (17, 2049, 8192), 2: (17, 2049, 8192, 18431, 18432)}[lds]:
        keys = rng.integers(0, max(1, n // 6), n).astype(np.uint32)
        assert np.array_equal(api.selftest_voxel_order(keys, lds=lds), O.sort_voxel_pairs(keys)), n
