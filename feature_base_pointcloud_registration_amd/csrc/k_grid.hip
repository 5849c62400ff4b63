// k_grid.hip — the kNN map grid, built on the device (fbr_set_map's prior map, the keyframe local
// map).  Replaces the reference's per-scan CropBox + KdTreeFLANN builds (mapOptmization.h:284-304,
// :1413-1414); see k_register.hip for why a radius-bounded grid search returns FLANN's neighbours.
//
// Two layouts over the same cells (1/inv_x along x, 1/inv_cell along y and z, powers of two):
//   dense   cell_start over the occupied bounding box (<= kDenseGridCells cells: 256 MB of
//           offsets).  Cell bounds (one reduction), per-cell counts (atomics), an exclusive scan
//           (rocprim), a scatter.  The order of points inside a cell is arbitrary: the kNN orders
//           candidates by (distance, map index) with the index in w.
//   sparse  prior maps of kilometres (LIO-SAM maps, mapOptmization.h:245-260), whose bounding box
//           would need billions of dense cells: every row of cells (fixed y, z) is cut into chunks
//           of kChunkX cells along x, and only occupied chunks exist.  Points are sorted by
//           (z, y, x) cell (rocprim radix sort of 64-bit keys), each chunk keeps kChunkX + 1 point
//           offsets, and an open-addressing hash (load <= 1/2) maps a chunk's (z, y, x / kChunkX)
//           key to it.  A kNN row range (<= 17 cells) spans at most two adjacent chunks, whose
//           points are contiguous in the sorted order, so the search keeps one contiguous point
//           range per row exactly as on the dense grid.
// Both give the kNN the same candidate sets.  HBM-bound builds: 16 B read + 16 B written per
// point plus the sort.
// Non-finite map points are never candidates (KdTreeFLANN skips them): they stay out of the cell
// bounds, the dense layout parks them in a phantom cell past the last real one (cell_start[n_cells]
// ends the real cells' points), and the sparse layout sorts them behind every chunk.  They keep
// their map index in by_id, which no neighbour list can name.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstdlib>

#include "fbr_common.h"
#include "fbr_kernels.h"

namespace fbr {

__global__ void __launch_bounds__(256)
k_grid_bounds(const float4* __restrict__ pts, int64_t n, float invx, float inv, int* bounds) {
  int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = pts[i];
    if (!map_point_finite(p)) {
      ++bad;
      continue;
    }
    const int c[3] = {(int)floorf(p.x * invx), (int)floorf(p.y * inv), (int)floorf(p.z * inv)};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      lo[d] = min(lo[d], c[d]);
      hi[d] = max(hi[d], c[d]);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    for (int o = 32; o > 0; o >>= 1) {
      lo[d] = min(lo[d], __shfl_xor(lo[d], o));
      hi[d] = max(hi[d], __shfl_xor(hi[d], o));
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&bounds[d], lo[d]);
      atomicMax(&bounds[3 + d], hi[d]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) bad += __shfl_xor(bad, o);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(&bounds[6], bad);
}

__device__ __forceinline__ void grid_cell3(const float4& p, const GridDesc& g, int& cx, int& cy, int& cz) {
  cx = (int)floorf(p.x * g.inv_x) - (int)g.origin[0];
  cy = (int)floorf(p.y * g.inv_cell) - (int)g.origin[1];
  cz = (int)floorf(p.z * g.inv_cell) - (int)g.origin[2];
}

// Dense cell of a map point; the phantom cell n_cells for a non-finite one.
__device__ __forceinline__ int64_t grid_cell_dense(const float4& p, const GridDesc& g) {
  if (!map_point_finite(p)) return g.n_cells;
  int cx, cy, cz;
  grid_cell3(p, g, cx, cy, cz);
  return ((int64_t)cz * g.dims[1] + cy) * g.dims[0] + cx;
}

// ---- dense ----
__global__ void __launch_bounds__(256) k_grid_count(const float4* __restrict__ pts, int64_t n, GridDesc g, int32_t* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicAdd(&cnt[grid_cell_dense(pts[i], g)], 1);
}

__global__ void __launch_bounds__(256)
k_grid_scatter(const float4* __restrict__ pts, int64_t n, GridDesc g, int32_t* fill, float4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = pts[i];
    const int slot = atomicAdd(&fill[grid_cell_dense(p, g)], 1);
    out[slot] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));  // w = map index (kNN tie-break)
  }
}

// ---- sparse (hashed chunks) ----
__global__ void __launch_bounds__(256)
k_chunk_keys(const float4* __restrict__ pts, int64_t n, GridDesc g, unsigned long long* keys, uint32_t* vals) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = pts[i];
    int cx, cy, cz;
    grid_cell3(p, g, cx, cy, cz);
    // (z, y, x) cell order; key >> log2(kChunkX) is the chunk key (chunk_key); non-finite points
    // sort behind every real key (z < 2^12) and are cut off before the chunk pass
    keys[i] = map_point_finite(p) ? ((unsigned long long)(unsigned)cz << 52) | ((unsigned long long)(unsigned)cy << 28) |
                                        (unsigned)cx
                                  : ~0ull;
    vals[i] = (uint32_t)i;
  }
}

constexpr int kChunkShift = 4;  // log2(kChunkX)
static_assert((1 << kChunkShift) == kChunkX, "chunk width");

// Sorted order: the points (w = map index), chunk heads (1 at each new chunk).
__global__ void __launch_bounds__(256)
k_chunk_scatter(const float4* __restrict__ src, int64_t n, const unsigned long long* __restrict__ keys,
                const uint32_t* __restrict__ vals, float4* __restrict__ out, uint32_t* __restrict__ head) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    const uint32_t i = vals[j];
    const float4 p = src[i];
    out[j] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));
    head[j] = (j == 0 || (keys[j] >> kChunkShift) != (keys[j - 1] >> kChunkShift)) ? 1u : 0u;
  }
}

// cs[chunk][x % kChunkX] = first point of each occupied cell, cs[chunk][kChunkX] = chunk end;
// chunk key of each chunk.  (cid = exclusive scan of the heads.)
__global__ void __launch_bounds__(256)
k_chunk_cells(int64_t n, const unsigned long long* __restrict__ keys, const uint32_t* __restrict__ cid,
              const uint32_t* __restrict__ head, int32_t* cs, unsigned long long* ckey) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    const unsigned long long k = keys[j];
    const uint32_t c = cid[j] + head[j] - 1u;  // inclusive: the chunk of point j
    if (j == 0 || keys[j - 1] != k) cs[(int64_t)c * (kChunkX + 1) + (int)(k & (kChunkX - 1))] = (int32_t)j;
    if (head[j]) ckey[c] = k >> kChunkShift;
    if (j == n - 1 || (keys[j + 1] >> kChunkShift) != (k >> kChunkShift)) cs[(int64_t)c * (kChunkX + 1) + kChunkX] = (int32_t)(j + 1);
  }
}

// Empty cells take the next occupied cell's start (so [cs[a], cs[b + 1]) is the range of cells
// a..b), then the chunk goes into the hash table.
__global__ void __launch_bounds__(256)
k_chunk_finish(int64_t nchunks, int32_t* cs, const unsigned long long* __restrict__ ckey, unsigned long long* hkeys,
               int32_t* hvals, uint32_t hmask) {
  for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < nchunks; c += (int64_t)gridDim.x * 256) {
    int32_t* r = cs + c * (kChunkX + 1);
    for (int k = kChunkX - 1; k >= 0; --k)
      if (r[k] < 0) r[k] = r[k + 1];
    const unsigned long long key = ckey[c];
    uint32_t h = chunk_hash(key) & hmask;
    for (uint32_t probe = 0; probe <= hmask; ++probe) {  // load <= 1/2: a free slot is always found
      const unsigned long long prev = atomicCAS(&hkeys[h], kChunkEmpty, key);
      if (prev == kChunkEmpty) {
        hvals[h] = (int32_t)c;
        break;
      }
      h = (h + 1) & hmask;
    }
  }
}

void free_grid(DevGrid& d) {
  for (void* p : {(void*)d.pts, (void*)d.cs, (void*)d.hkeys, (void*)d.hvals})
    if (p) (void)hipFree(p);
  d = DevGrid{};
}

namespace {
bool force_sparse_env() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_GRID_SPARSE");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}
}  // namespace

int grid_build_device(hipStream_t s, DevArena& ar, const float4* src, int64_t n, float invx, float inv,
                      bool force_sparse, DevGrid& out) {
  free_grid(out);
  // the kNN walks address map points with a 32-bit byte offset (fbr_gn.h): below 2^28 points
  if (n >= ((int64_t)1 << 28)) return FBR_ERR_CAPACITY;
  int rc = FBR_OK;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && !rc) rc = FBR_ERR_HIP;
    return rc == FBR_OK;
  };
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
  // cell bounds (min x, y, z, max x, y, z), read back once
  int b[7] = {0, 0, 0, 0, 0, 0, 0};  // cell min x, y, z, max x, y, z; non-finite points
  if (!ok(arena_reserve(ar, arena_bytes(sizeof(b)), s))) return rc;
  int* d_bounds = arena_take<int>(ar, sizeof(b));
  if (!d_bounds) return FBR_ERR_HIP;
  if (!ok(hipMemsetD32Async((hipDeviceptr_t)d_bounds, (unsigned)INT_MAX, 3, s)) ||
      !ok(hipMemsetD32Async((hipDeviceptr_t)(d_bounds + 3), (unsigned)INT_MIN, 3, s)) ||
      !ok(hipMemsetD32Async((hipDeviceptr_t)(d_bounds + 6), 0u, 1, s)))
    return rc;
  if (n > 0) fbr_launch(k_grid_bounds, dim3(grid), dim3(256), 0, s, src, n, invx, inv, d_bounds);
  ok(hipMemcpyAsync(b, d_bounds, sizeof(b), hipMemcpyDeviceToHost, s));
  ok(hipStreamSynchronize(s));
  if (rc) return rc;
  const int64_t nf = n - b[6];  // finite points: the only candidates
  if (nf == 0)
    for (int d = 0; d < 6; ++d) b[d] = 0;
  int64_t dims[3];
  for (int d = 0; d < 3; ++d) dims[d] = (int64_t)b[3 + d] - b[d] + 1;
  GridDesc& g = out.g;
  g.inv_cell = inv;
  g.inv_x = invx;
  for (int d = 0; d < 3; ++d) g.origin[d] = (float)b[d];
  g.n_points = n;
  // dense only when the box has at most kDenseGridCells cells; each factor is checked before the
  // product so that far outliers on every axis cannot overflow it
  const bool too_big = dims[0] > kDenseGridCells || dims[1] > kDenseGridCells / dims[0] ||
                       dims[2] > kDenseGridCells / (dims[0] * dims[1]);
  const bool sparse = force_sparse || force_sparse_env() || too_big;
  if (sparse && (dims[0] > ((int64_t)1 << 28) || dims[1] > ((int64_t)1 << 24) || dims[2] > ((int64_t)1 << 12)))
    return FBR_ERR_CAPACITY;
  for (int d = 0; d < 3; ++d) g.dims[d] = (int32_t)std::min<int64_t>(dims[d], INT32_MAX);
  if (!ok(hipMalloc((void**)&out.pts, sizeof(float4) * std::max<int64_t>(2 * n, 1)))) return rc;
  // [n, 2n): the points in map-index order (MapGrid::by_id)
  if (n) ok(hipMemcpyAsync(out.pts + n, src, sizeof(float4) * n, hipMemcpyDeviceToDevice, s));
  if (!sparse) {
    const int64_t ncell = dims[0] * dims[1] * dims[2];
    g.sparse = 0;
    g.hmask = 0;
    g.n_cells = (int32_t)ncell;
    size_t tb = 0;
    int32_t* null32 = nullptr;
    if (ok(rocprim::exclusive_scan(nullptr, tb, null32, null32, 0, (size_t)(ncell + 1), rocprim::plus<int32_t>(), s)) &&
        ok(arena_reserve(ar, arena_bytes(sizeof(int32_t) * (ncell + 1)) + arena_bytes(tb), s)) &&
        ok(hipMalloc((void**)&out.cs, sizeof(int32_t) * (ncell + 1)))) {
      int32_t* cnt = arena_take<int32_t>(ar, sizeof(int32_t) * (ncell + 1));
      void* tmp = arena_take<void>(ar, tb);
      if (!cnt || !tmp) rc = FBR_ERR_HIP;
      if (!rc && ok(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (ncell + 1), s))) {
        if (n > 0) fbr_launch(k_grid_count, dim3(grid), dim3(256), 0, s, src, n, g, cnt);
        // cell_start = exclusive scan of the counts (ncell + 1 entries: the last is n)
        if (ok(rocprim::exclusive_scan(tmp, tb, cnt, out.cs, 0, (size_t)(ncell + 1), rocprim::plus<int32_t>(), s)) &&
            ok(hipMemcpyAsync(cnt, out.cs, sizeof(int32_t) * (ncell + 1), hipMemcpyDeviceToDevice, s)) && n > 0)
          fbr_launch(k_grid_scatter, dim3(grid), dim3(256), 0, s, src, n, g, cnt, out.pts);
      }
    }
    ok(hipStreamSynchronize(s));
    return rc;
  }
  // ---- sparse ----
  g.sparse = 1;
  const size_t N = (size_t)std::max<int64_t>(n, 1);
  size_t tb_sort = 0, tb_scan = 0;
  unsigned long long* null64 = nullptr;
  uint32_t* nullu = nullptr;
  if (!ok(rocprim::radix_sort_pairs(nullptr, tb_sort, null64, null64, nullu, nullu, N, 0, 64, s)) ||
      !ok(rocprim::exclusive_scan(nullptr, tb_scan, nullu, nullu, 0u, N, rocprim::plus<uint32_t>(), s)) ||
      !ok(arena_reserve(ar, 3 * arena_bytes(8 * N) + 4 * arena_bytes(4 * N) + arena_bytes(std::max(tb_sort, tb_scan)), s)))
    return rc;
  unsigned long long* k0 = arena_take<unsigned long long>(ar, 8 * N);
  unsigned long long* k1 = arena_take<unsigned long long>(ar, 8 * N);
  unsigned long long* ckey = arena_take<unsigned long long>(ar, 8 * N);  // nchunks <= n
  uint32_t* v0 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* v1 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* head = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* cid = arena_take<uint32_t>(ar, 4 * N);
  void* tmp = arena_take<void>(ar, std::max(tb_sort, tb_scan));
  if (!k0 || !k1 || !ckey || !v0 || !v1 || !head || !cid || !tmp) return FBR_ERR_HIP;
  uint32_t nchunks = 0;
  if (nf > 0) {  // the non-finite points sort last and stay out of the chunks
    fbr_launch(k_chunk_keys, dim3(grid), dim3(256), 0, s, src, n, g, k0, v0);
    if (ok(rocprim::radix_sort_pairs(tmp, tb_sort, k0, k1, v0, v1, (size_t)n, 0, 64, s))) {
      fbr_launch(k_chunk_scatter, dim3(grid), dim3(256), 0, s, src, nf, k1, v1, out.pts, head);
      uint32_t last[2] = {0, 0};
      if (ok(rocprim::exclusive_scan(tmp, tb_scan, head, cid, 0u, (size_t)nf, rocprim::plus<uint32_t>(), s)) &&
          ok(hipMemcpyAsync(&last[0], cid + nf - 1, 4, hipMemcpyDeviceToHost, s)) &&
          ok(hipMemcpyAsync(&last[1], head + nf - 1, 4, hipMemcpyDeviceToHost, s)) && ok(hipStreamSynchronize(s)))
        nchunks = last[0] + last[1];
    }
  }
  uint32_t hsize = 1024;
  while (hsize < 2 * nchunks) hsize <<= 1;
  g.hmask = hsize - 1;
  g.n_cells = (int32_t)nchunks;
  if (!rc && ok(hipMalloc((void**)&out.cs, sizeof(int32_t) * (kChunkX + 1) * std::max<uint32_t>(nchunks, 1))) &&
      ok(hipMalloc((void**)&out.hkeys, sizeof(unsigned long long) * hsize)) &&
      ok(hipMalloc((void**)&out.hvals, sizeof(int32_t) * hsize)) &&
      ok(hipMemsetAsync(out.cs, 0xFF, sizeof(int32_t) * (kChunkX + 1) * std::max<uint32_t>(nchunks, 1), s)) &&
      ok(hipMemsetAsync(out.hkeys, 0xFF, sizeof(unsigned long long) * hsize, s)) && nchunks > 0) {
    fbr_launch(k_chunk_cells, dim3(grid), dim3(256), 0, s, nf, k1, cid, head, out.cs, ckey);
    const int cg = (int)std::max<int64_t>(1, std::min<int64_t>((nchunks + 255) / 256, 2048));
    fbr_launch(k_chunk_finish, dim3(cg), dim3(256), 0, s, (int64_t)nchunks, out.cs, ckey, out.hkeys, out.hvals,
               g.hmask);
  }
  ok(hipStreamSynchronize(s));
  return rc;
}

}  // namespace fbr
