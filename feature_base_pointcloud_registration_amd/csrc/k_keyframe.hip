// k_keyframe.hip — SURVEY §8(f) row 4: the LIO-SAM keyframe local map on the device, and a
// device-side build of the kNN map grid.
//
// Reference: /root/reference/src/mapOptmization.h
//   extractCloud()        :909-955  transformPointCloud of every selected keyframe's corner / surf
//                                    cloud (OpenMP), concatenation in selection order, then the
//                                    mapping-leaf VoxelGrids (reused: k_voxel.hip)
//   transformPointCloud() :405-425  pcl::getTransformation(x, y, z, roll, pitch, yaw) in float,
//                                    rows ((r0 x + r1 y) + r2 z) + t
// The keyframe selection (extractNearby / extractForLoopClosure, :857-907) is a serial pass over
// a few hundred key poses and runs on the host (fbr_api.hip).
//
// k_kf_transform: one workgroup per (selected entry, 1024-point chunk); each entry is a copy of
// one keyframe's cloud into its concatenation offset, transformed by that keyframe's pose.
// HBM-bound: 16 B read + 16 B written per point.
//
// Grid build (replaces the host counting sort of fbr_set_map when the map is rebuilt per scan):
// cell bounds (one reduction), per-cell counts (atomics), an exclusive scan (rocprim) and a
// scatter.  The order of points inside a cell is arbitrary: the kNN orders candidates by
// (distance, map index) with the index carried in w, so the neighbour sets do not depend on it.
#include <rocprim/device/device_scan.hpp>

#include "fbr_common.h"
#include "fbr_kernels.h"

namespace fbr {

__global__ void __launch_bounds__(256)
k_kf_transform(const float4* __restrict__ pool, const KfSeg* __restrict__ segs, int nseg, float4* __restrict__ out) {
  const int s = blockIdx.y;
  if (s >= nseg) return;
  const KfSeg g = segs[s];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < g.count; i += (int64_t)gridDim.x * 256) {
    const float4 p = pool[g.src + i];
    float4 q;
    q.x = g.T[0] * p.x + g.T[1] * p.y + g.T[2] * p.z + g.T[3];
    q.y = g.T[4] * p.x + g.T[5] * p.y + g.T[6] * p.z + g.T[7];
    q.z = g.T[8] * p.x + g.T[9] * p.y + g.T[10] * p.z + g.T[11];
    q.w = p.w;
    out[g.dst + i] = q;
  }
}

void launch_kf_transform(hipStream_t s, const float4* pool, const KfSeg* segs, int nseg, int64_t max_count, float4* out) {
  if (nseg <= 0 || max_count <= 0) return;
  const int gx = (int)std::min<int64_t>((max_count + 255) / 256, 64);
  for (int s0 = 0; s0 < nseg; s0 += 65535) {
    const int n = std::min(65535, nseg - s0);
    fbr_launch(k_kf_transform, dim3(gx, n), dim3(256), 0, s, pool, segs + s0, n, out);
  }
}

// ---- device grid build ----
__global__ void __launch_bounds__(256)
k_grid_bounds(const float4* __restrict__ pts, int64_t n, float invx, float inv, int* bounds) {
  int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = pts[i];
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
}

__device__ __forceinline__ int grid_cell(const float4& p, const GridDesc& g) {
  const int cx = (int)floorf(p.x * g.inv_x) - (int)g.origin[0];
  const int cy = (int)floorf(p.y * g.inv_cell) - (int)g.origin[1];
  const int cz = (int)floorf(p.z * g.inv_cell) - (int)g.origin[2];
  return (cz * g.dims[1] + cy) * g.dims[0] + cx;
}

__global__ void __launch_bounds__(256) k_grid_count(const float4* __restrict__ pts, int64_t n, GridDesc g, int32_t* cnt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    atomicAdd(&cnt[grid_cell(pts[i], g)], 1);
}

__global__ void __launch_bounds__(256)
k_grid_scatter(const float4* __restrict__ pts, int64_t n, GridDesc g, int32_t* fill, float4* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = pts[i];
    const int slot = atomicAdd(&fill[grid_cell(p, g)], 1);
    out[slot] = make_float4(p.x, p.y, p.z, __int_as_float((int)i));  // w = map index (kNN tie-break)
  }
}

int grid_bounds_device(hipStream_t s, const float4* pts, int64_t n, float invx, float inv, int* d_bounds,
                       int h_bounds[6]) {
  const int init[6] = {INT_MAX, INT_MAX, INT_MAX, INT_MIN, INT_MIN, INT_MIN};
  if (hipMemcpyAsync(d_bounds, init, sizeof(init), hipMemcpyHostToDevice, s) != hipSuccess) return FBR_ERR_HIP;
  if (n > 0) {
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 2048);
    fbr_launch(k_grid_bounds, dim3(grid), dim3(256), 0, s, pts, n, invx, inv, d_bounds);
  }
  if (hipMemcpyAsync(h_bounds, d_bounds, sizeof(int) * 6, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return FBR_ERR_HIP;
  return FBR_OK;
}

int grid_fill_device(hipStream_t s, const float4* pts, int64_t n, const GridDesc& g, int32_t* d_cs, float4* d_out) {
  const int64_t ncell = (int64_t)g.n_cells;
  int32_t* cnt = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  int rc = FBR_OK;
  if (hipMallocAsync((void**)&cnt, sizeof(int32_t) * (ncell + 1), s) != hipSuccess) return FBR_ERR_HIP;
  if (hipMemsetAsync(cnt, 0, sizeof(int32_t) * (ncell + 1), s) != hipSuccess) rc = FBR_ERR_HIP;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
  if (!rc && n > 0) fbr_launch(k_grid_count, dim3(grid), dim3(256), 0, s, pts, n, g, cnt);
  // cell_start = exclusive scan of the counts (ncell + 1 entries: the last is n)
  if (!rc && rocprim::exclusive_scan(nullptr, tmp_bytes, cnt, d_cs, 0, (size_t)(ncell + 1), rocprim::plus<int32_t>(), s) !=
                 hipSuccess)
    rc = FBR_ERR_HIP;
  if (!rc && hipMallocAsync(&tmp, std::max<size_t>(tmp_bytes, 16), s) != hipSuccess) rc = FBR_ERR_HIP;
  if (!rc && rocprim::exclusive_scan(tmp, tmp_bytes, cnt, d_cs, 0, (size_t)(ncell + 1), rocprim::plus<int32_t>(), s) !=
                 hipSuccess)
    rc = FBR_ERR_HIP;
  // reuse the counts as fill cursors
  if (!rc && hipMemcpyAsync(cnt, d_cs, sizeof(int32_t) * ncell, hipMemcpyDeviceToDevice, s) != hipSuccess) rc = FBR_ERR_HIP;
  if (!rc && n > 0) fbr_launch(k_grid_scatter, dim3(grid), dim3(256), 0, s, pts, n, g, cnt, d_out);
  if (tmp) (void)hipFreeAsync(tmp, s);
  (void)hipFreeAsync(cnt, s);
  return rc;
}

}  // namespace fbr
