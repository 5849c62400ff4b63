// k_voxel.hip — A9: pcl::VoxelGrid<PointXYZI>::filter as a segmented device kernel.
//
// Used for every down-sample on the path: the per-ring surf filter (featureExtraction.h:288-292,
// leaf odometrySurfLeafSize), downsampleCurrentScan (mapOptmization.h:981-993, leaves
// mappingCornerLeafSize / mappingSurfLeafSize) and the start-up map filter (:251-257).
// Semantics follow PCL 1.8 applyFilter: float min/max box, int64 overflow check (output = input),
// key = ijk0 + ijk1*div_x + ijk2*div_x*div_y with ijk = int(floor(p*inv_leaf) - float(min_b)),
// voxels emitted in ascending key order, centroid = float sum of x,y,z,intensity / count.
// PCL sorts (key, index) with the unstable std::sort, so the order of points inside one voxel —
// and hence the last bits of the centroid sum — is introsort-specific; this kernel sorts stably
// (ascending input index inside a voxel).  Voxel membership and output order are exact; centroids
// agree with the reference to float rounding (tests state the tolerance).
//
// Morton mode (downsampleCurrentScan only): the same voxels and centroids, emitted in Morton order
// of (i,j,k) so that consecutive output points are spatially compact.  The order of the mapping
// DS clouds only fixes the summation order of AtA (accumulated in fp64, so immaterial); it makes
// every 64-query wave of the registration kernels touch a compact patch of the map grid.
//
// One 256-thread workgroup per segment.  The (key, index) pairs are sorted by an LSD radix sort
// (8-bit digits, only as many passes as the key range needs) whose ping-pong buffers live in a
// per-segment global scratch (L2-resident at these sizes); stability inside a 256-element tile
// comes from wave ballot peer masks.
#include "fbr_common.h"
#include "fbr_kernels.h"

namespace fbr {

namespace {
constexpr int kVgThreads = 256;
constexpr int kVgWaves = kVgThreads / 64;
}  // namespace

// Block-wide stable LSD radix sort of n (key, val) pairs.  Returns the buffer index (0 or 1)
// holding the result.  Must be called by all 256 threads.
__device__ __forceinline__ uint32_t spread3_10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3FFu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

__device__ int block_radix_sort(uint32_t* k[2], uint32_t* v[2], uint32_t* hist, int n, int nbits,
                                uint32_t* lds_hist /*[256]*/, uint32_t* lds_wc /*[kVgWaves][256]*/,
                                uint32_t* lds_tot /*[256]*/) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = (n + kVgThreads - 1) / kVgThreads;
  const int passes = (nbits + 7) / 8;
  int cur = 0;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = 8 * pass;
    const uint32_t* kin = k[cur];
    const uint32_t* vin = v[cur];
    uint32_t* kout = k[cur ^ 1];
    uint32_t* vout = v[cur ^ 1];
    // 1) per-tile digit histograms
    for (int t = 0; t < ntiles; ++t) {
      lds_hist[tid] = 0;
      __syncthreads();
      const int i = t * kVgThreads + tid;
      if (i < n) atomicAdd(&lds_hist[(kin[i] >> shift) & 255u], 1u);
      __syncthreads();
      hist[t * 256 + tid] = lds_hist[tid];
      __syncthreads();
    }
    // 2) exclusive scan in digit-major, tile-minor order
    uint32_t run = 0;
    for (int t = 0; t < ntiles; ++t) {
      const uint32_t c = hist[t * 256 + tid];
      hist[t * 256 + tid] = run;
      run += c;
    }
    lds_tot[tid] = run;
    __syncthreads();
    if (tid == 0) {
      uint32_t acc = 0;
      for (int d = 0; d < 256; ++d) {
        const uint32_t c = lds_tot[d];
        lds_tot[d] = acc;
        acc += c;
      }
    }
    __syncthreads();
    const uint32_t base = lds_tot[tid];
    for (int t = 0; t < ntiles; ++t) hist[t * 256 + tid] += base;
    __syncthreads();
    // 3) stable scatter
    for (int t = 0; t < ntiles; ++t) {
      for (int w = 0; w < kVgWaves; ++w) lds_wc[w * 256 + tid] = 0;
      __syncthreads();
      const int i = t * kVgThreads + tid;
      const bool valid = i < n;
      const uint32_t key = valid ? kin[i] : 0u;
      const uint32_t d = (key >> shift) & 255u;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < 8; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
      const int rank = __popcll(peers & ((1ull << lane) - 1ull));
      if (valid && rank == 0) lds_wc[wave * 256 + d] = (uint32_t)__popcll(peers);
      __syncthreads();
      if (valid) {
        uint32_t off = hist[t * 256 + d] + rank;
        for (int w = 0; w < wave; ++w) off += lds_wc[w * 256 + d];
        kout[off] = key;
        vout[off] = vin[i];
      }
      __syncthreads();
    }
    cur ^= 1;
    __syncthreads();
  }
  return cur;
}

__global__ void __launch_bounds__(kVgThreads)
k_voxel_grid(VgArgs a) {
  __shared__ float red[6][kVgThreads];
  __shared__ uint32_t lds_hist[256];
  __shared__ uint32_t lds_wc[kVgWaves * 256];
  __shared__ uint32_t lds_tot[256];
  __shared__ int64_t sh_info[8];
  const int seg = blockIdx.x, tid = threadIdx.x;
  const int n = (int)min((int64_t)a.cnt_in[seg], a.stride_in);
  const float4* in = a.in + (int64_t)seg * a.stride_in;
  float4* out = a.out + (int64_t)seg * a.stride_out;
  if (n <= 0) {
    if (tid == 0) a.cnt_out[seg] = 0;
    return;
  }
  // getMinMax3D
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int i = tid; i < n; i += kVgThreads) {
    const float4 p = in[i];
    const float v[3] = {p.x, p.y, p.z};
    for (int d = 0; d < 3; ++d) {
      mn[d] = (v[d] < mn[d]) ? v[d] : mn[d];
      mx[d] = (mx[d] < v[d]) ? v[d] : mx[d];
    }
  }
  for (int d = 0; d < 3; ++d) {
    red[d][tid] = mn[d];
    red[3 + d][tid] = mx[d];
  }
  __syncthreads();
  for (int s = kVgThreads / 2; s > 0; s >>= 1) {
    if (tid < s)
      for (int d = 0; d < 3; ++d) {
        const float b = red[d][tid + s], c = red[3 + d][tid + s];
        red[d][tid] = (b < red[d][tid]) ? b : red[d][tid];
        red[3 + d][tid] = (red[3 + d][tid] < c) ? c : red[3 + d][tid];
      }
    __syncthreads();
  }
  for (int d = 0; d < 3; ++d) {
    mn[d] = red[d][0];
    mx[d] = red[3 + d][0];
  }
  const float inv = 1.0f / a.leaf;
  const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
  const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
  const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)INT32_MAX) {  // PCL: "Leaf size is too small" -> output = input
    for (int i = tid; i < n; i += kVgThreads) out[i] = in[i];
    if (tid == 0) a.cnt_out[seg] = n;
    return;
  }
  int min_b[3], div_b[3];
  for (int d = 0; d < 3; ++d) {
    min_b[d] = (int)floorf(mn[d] * inv);
    const int max_b = (int)floorf(mx[d] * inv);
    div_b[d] = max_b - min_b[d] + 1;
  }
  const uint32_t mul1 = (uint32_t)div_b[0], mul2 = (uint32_t)div_b[0] * (uint32_t)div_b[1];
  const bool morton = a.morton && div_b[0] <= 1024 && div_b[1] <= 1024 && div_b[2] <= 1024;
  uint32_t* sc = a.scratch + (int64_t)seg * 4 * a.stride_in;
  uint32_t* kb[2] = {sc, sc + 2 * a.stride_in};
  uint32_t* vb[2] = {sc + a.stride_in, sc + 3 * a.stride_in};
  for (int i = tid; i < n; i += kVgThreads) {
    const float4 p = in[i];
    const int ijk0 = (int)(floorf(p.x * inv) - (float)min_b[0]);
    const int ijk1 = (int)(floorf(p.y * inv) - (float)min_b[1]);
    const int ijk2 = (int)(floorf(p.z * inv) - (float)min_b[2]);
    kb[0][i] = morton ? (spread3_10((uint32_t)ijk0) | (spread3_10((uint32_t)ijk1) << 1) |
                         (spread3_10((uint32_t)ijk2) << 2))
                      : (uint32_t)ijk0 + (uint32_t)ijk1 * mul1 + (uint32_t)ijk2 * mul2;
    vb[0][i] = (uint32_t)i;
  }
  const uint64_t nkeys = (uint64_t)div_b[0] * (uint64_t)div_b[1] * (uint64_t)div_b[2];
  int nbits = 32;
  if (morton) {
    int b = 1;
    for (int d = 0; d < 3; ++d)
      if (div_b[d] > 1) b = max(b, 32 - __clz((uint32_t)(div_b[d] - 1)));
    nbits = 3 * b;
  } else if (nkeys <= 0xFFFFFFFFull) {
    const uint32_t maxk = (uint32_t)(nkeys - 1);
    nbits = maxk == 0 ? 1 : 32 - __clz(maxk);
  }
  __syncthreads();
  const int r = block_radix_sort(kb, vb, a.hist + (int64_t)seg * a.hist_stride, n, nbits, lds_hist, lds_wc, lds_tot);
  const uint32_t* ks = kb[r];
  const uint32_t* vs = vb[r];
  // heads -> output voxels in ascending key order
  int64_t* total = &sh_info[0];
  if (tid == 0) *total = 0;
  __syncthreads();
  for (int t0 = 0; t0 < n; t0 += kVgThreads) {
    const int i = t0 + tid;
    const bool head = i < n && (i == 0 || ks[i] != ks[i - 1]);
    const uint64_t bal = __ballot(head);
    const int wave = tid >> 6, lane = tid & 63;
    lds_hist[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    int pos = (int)*total;
    for (int w = 0; w < wave; ++w) pos += (int)lds_hist[w];
    pos += __popcll(bal & ((1ull << lane) - 1ull));
    if (head) {
      const uint32_t key = ks[i];
      float4 c = in[vs[i]];
      int j = i + 1;
      while (j < n && ks[j] == key) {
        const float4 p = in[vs[j]];
        c.x += p.x;
        c.y += p.y;
        c.z += p.z;
        c.w += p.w;
        ++j;
      }
      const float cnt = (float)(j - i);
      out[pos] = make_float4(c.x / cnt, c.y / cnt, c.z / cnt, c.w / cnt);
    }
    __syncthreads();
    if (tid == 0) {
      int add = 0;
      for (int w = 0; w < kVgWaves; ++w) add += (int)lds_hist[w];
      *total += add;
    }
    __syncthreads();
  }
  if (tid == 0) a.cnt_out[seg] = (int32_t)*total;
}

void launch_voxel_grid(hipStream_t s, const VgArgs& a) {
  if (a.nseg <= 0) return;
  hipLaunchKernelGGL(k_voxel_grid, dim3(a.nseg), dim3(kVgThreads), 0, s, a);
}

// One workgroup per job: ring-ordered concatenation of the per-ring corner picks and per-ring
// surf DS outputs (cornerCloud / surfaceCloud of featureExtraction.h).
__global__ void __launch_bounds__(256)
k_concat(int H, int W, const float4* corner_slot, const int32_t* corner_cnt, const float4* surf_ring,
         const int32_t* surf_ring_cnt, float4* corner_all, int64_t capc, int32_t* n_corner, float4* surf_all,
         int64_t caps, int32_t* n_surf) {
  extern __shared__ int32_t off[];  // [2][H+1]
  const int job = blockIdx.x, tid = threadIdx.x;
  const int32_t* cc = corner_cnt + job * H;
  const int32_t* sc = surf_ring_cnt + job * H;
  if (tid == 0) {
    int a = 0, b = 0;
    for (int r = 0; r < H; ++r) {
      off[r] = a;
      off[H + 1 + r] = b;
      a += cc[r];
      b += sc[r];
    }
    off[H] = a;
    off[2 * H + 1] = b;
    n_corner[job] = a;
    n_surf[job] = b;
  }
  __syncthreads();
  for (int r = 0; r < H; ++r) {
    const int nc = cc[r], ns = sc[r];
    const float4* cs = corner_slot + ((int64_t)job * H + r) * kCornerPerRing;
    const float4* ss = surf_ring + ((int64_t)job * H + r) * W;
    for (int i = tid; i < nc; i += 256) corner_all[job * capc + off[r] + i] = cs[i];
    for (int i = tid; i < ns; i += 256) surf_all[job * caps + off[H + 1 + r] + i] = ss[i];
  }
}

void launch_concat(hipStream_t s, int B, int H, int W, const float4* corner_slot, const int32_t* corner_cnt,
                   const float4* surf_ring, const int32_t* surf_ring_cnt, float4* corner_all, int64_t capc,
                   int32_t* n_corner, float4* surf_all, int64_t caps, int32_t* n_surf) {
  hipLaunchKernelGGL(k_concat, dim3(B), dim3(256), sizeof(int32_t) * 2 * (H + 1), s, H, W, corner_slot,
                     corner_cnt, surf_ring, surf_ring_cnt, corner_all, capc, n_corner, surf_all, caps, n_surf);
}

}  // namespace fbr
