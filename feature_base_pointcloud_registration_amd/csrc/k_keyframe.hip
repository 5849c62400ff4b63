// k_keyframe.hip — SURVEY §8(f) row 4: the LIO-SAM keyframe local map on the device (the kNN
// map grid over it is built by k_grid.hip's grid_build_device).
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

}  // namespace fbr
