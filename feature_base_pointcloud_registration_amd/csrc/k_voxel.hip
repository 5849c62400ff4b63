// k_voxel.hip — A9: pcl::VoxelGrid<PointXYZI>::filter as a segmented device kernel.
//
// Used for every down-sample on the path: the per-ring surf filter (featureExtraction.h:288-292,
// leaf odometrySurfLeafSize), downsampleCurrentScan (mapOptmization.h:981-993, leaves
// mappingCornerLeafSize / mappingSurfLeafSize) and the start-up map filter (:251-257).
// Semantics follow PCL 1.8 applyFilter: float min/max box, int64 overflow check (output = input),
// key = ijk0 + ijk1*div_x + ijk2*div_x*div_y with ijk = int(floor(p*inv_leaf) - float(min_b)),
// voxels emitted in ascending key order, centroid = float sum of x,y,z,intensity / count.
// PCL sorts (key, index) with the unstable std::sort, so the order of points inside one voxel —
// and hence the last bits of the centroid sum — is introsort-specific.  The kernels reproduce it
// (fbr_introsort.h) when fbr_params.exact_voxel_order = 1: std::sort's partition phase on (PCL key, index), then
// their stable radix sort of that sequence, which is std::sort's result; centroids are bit-exact.
// By default the partition phase is skipped (points summed in index order, centroids to float
// rounding, at about twice the exact mode's throughput).
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
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "fbr_common.h"
#include "fbr_introsort.h"
#include "fbr_kernels.h"

#include <algorithm>
#include <atomic>
#include <mutex>
#include <cstdlib>
#include <type_traits>

namespace fbr {

// Stable LSD radix sort of one segment by one workgroup of T threads ("wave chunks"): wave w owns
// the contiguous chunk [c0, c1) of the (key, index) array; per pass each wave builds an LDS digit
// histogram of its chunk, one digit-major / wave-minor exclusive scan gives every (digit, wave)
// its output base, and each wave scatters its chunk in index order (8..9 ballots give each lane
// its rank among equal digits in the 64-element step).  Waves in chunk order and steps in index
// order make the sort stable.  Keys and indices live in LDS when the segment fits (per-ring
// filters, u16 indices), otherwise in a per-segment global scratch (mapping DS, 1024 threads).

__device__ __forceinline__ uint32_t spread3_10(uint32_t v) {  // 10 bits -> every third bit
  v &= 0x3FFu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// ---- shared pieces of the two VoxelGrid front ends ----

// Block-wide float min / max (getMinMax3D) of per-thread partials; mm = [NW][6] LDS.
template <int T>
__device__ void vg_block_minmax(float (&mn)[3], float (&mx)[3], float* mm) {
  constexpr int NW = T / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 0; d < 3; ++d)
    for (int o = 32; o > 0; o >>= 1) {
      const float a = __shfl_xor(mn[d], o), b = __shfl_xor(mx[d], o);
      mn[d] = (a < mn[d]) ? a : mn[d];
      mx[d] = (mx[d] < b) ? b : mx[d];
    }
  if (lane == 0)
    for (int d = 0; d < 3; ++d) {
      mm[w * 6 + d] = mn[d];
      mm[w * 6 + 3 + d] = mx[d];
    }
  __syncthreads();
  for (int d = 0; d < 3; ++d) {
    mn[d] = mm[d];
    mx[d] = mm[3 + d];
    for (int ww = 1; ww < NW; ++ww) {
      const float a = mm[ww * 6 + d], b = mm[ww * 6 + 3 + d];
      mn[d] = (a < mn[d]) ? a : mn[d];
      mx[d] = (mx[d] < b) ? b : mx[d];
    }
  }
}

// getMinMax3D of segment seg (its first n points): from the producer's ring boxes when the set
// has them (k_concat; bounds are exact under any merge order), else from the points.  All threads
// get the result.
template <int T>
__device__ void vg_seg_bounds(const VgSet& S, int seg, int n, const float4* in, float (&mn)[3], float (&mx)[3],
                              float* mm) {
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    mn[d] = FLT_MAX;
    mx[d] = -FLT_MAX;
  }
  if (S.box && (int64_t)S.cnt_in[seg] <= S.cap) {  // boxes cover exactly the segment's points
    const float* bx = S.box + (int64_t)seg * S.box_stride;
    for (int k = threadIdx.x; k < S.box_n; k += T) {
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const float a = bx[(int64_t)k * kRingBox + d], b = bx[(int64_t)k * kRingBox + 3 + d];
        mn[d] = (a < mn[d]) ? a : mn[d];
        mx[d] = (mx[d] < b) ? b : mx[d];
      }
    }
  } else {
    for (int i = threadIdx.x; i < n; i += T) {
      const float4 p = in[i];
      const float v[3] = {p.x, p.y, p.z};
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        mn[d] = (v[d] < mn[d]) ? v[d] : mn[d];
        mx[d] = (mx[d] < v[d]) ? v[d] : mx[d];
      }
    }
  }
  vg_block_minmax<T>(mn, mx, mm);
}

// PCL applyFilter's grid (leaf inverse, min_b, div_b) and the key function.
struct VgGrid {
  float inv;
  int min_b[3];
  uint32_t mul1, mul2;
  bool morton, overflow;
  int nbits;
  __device__ void init(const float (&mn)[3], const float (&mx)[3], float leaf, bool want_morton) {
    inv = 1.0f / leaf;
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    overflow = dx * dy * dz > (int64_t)INT32_MAX;  // PCL: "Leaf size is too small" -> output = input
    int div_b[3];
    for (int d = 0; d < 3; ++d) {
      min_b[d] = (int)floorf(mn[d] * inv);
      const int max_b = (int)floorf(mx[d] * inv);
      div_b[d] = max_b - min_b[d] + 1;
    }
    mul1 = (uint32_t)div_b[0];
    mul2 = (uint32_t)div_b[0] * (uint32_t)div_b[1];
    morton = want_morton && div_b[0] <= 1024 && div_b[1] <= 1024 && div_b[2] <= 1024;
    nbits = 32;
    if (morton) {
      int b = 1;
      for (int d = 0; d < 3; ++d)
        if (div_b[d] > 1) b = max(b, 32 - __clz((uint32_t)(div_b[d] - 1)));
      nbits = 3 * b;
    } else {
      const uint64_t nkeys = (uint64_t)div_b[0] * (uint64_t)div_b[1] * (uint64_t)div_b[2];
      if (nkeys <= 0xFFFFFFFFull) {
        const uint32_t maxk = (uint32_t)(nkeys - 1);
        nbits = maxk == 0 ? 1 : 32 - __clz(maxk);
      }
    }
  }
  // PCL's key (the one std::sort compares), whatever the output order
  __device__ __forceinline__ uint32_t pcl_key(const float4& p) const {
    const int ijk0 = (int)(floorf(p.x * inv) - (float)min_b[0]);
    const int ijk1 = (int)(floorf(p.y * inv) - (float)min_b[1]);
    const int ijk2 = (int)(floorf(p.z * inv) - (float)min_b[2]);
    return (uint32_t)ijk0 + (uint32_t)ijk1 * mul1 + (uint32_t)ijk2 * mul2;
  }
  // the output-order key of a PCL key (its Morton code in Morton mode; ijk < div_b decodes uniquely)
  __device__ __forceinline__ uint32_t out_key(uint32_t k) const {
    if (!morton) return k;
    const uint32_t k2 = k / mul2, r = k - k2 * mul2, k1 = r / mul1, k0 = r - k1 * mul1;
    return spread3_10(k0) | (spread3_10(k1) << 1) | (spread3_10(k2) << 2);
  }
  __device__ __forceinline__ uint32_t key(const float4& p) const {
    const int ijk0 = (int)(floorf(p.x * inv) - (float)min_b[0]);
    const int ijk1 = (int)(floorf(p.y * inv) - (float)min_b[1]);
    const int ijk2 = (int)(floorf(p.z * inv) - (float)min_b[2]);
    return morton ? (spread3_10((uint32_t)ijk0) | (spread3_10((uint32_t)ijk1) << 1) | (spread3_10((uint32_t)ijk2) << 2))
                  : (uint32_t)ijk0 + (uint32_t)ijk1 * mul1 + (uint32_t)ijk2 * mul2;
  }
};

// LDS-mode buffers are accessed through address-space-3 pointers: the ping-pong selection by a
// loop-carried index otherwise leaves generic pointers, i.e. flat_* instead of ds_* accesses.
#define FBR_LDS_AS __attribute__((address_space(3)))
template <bool L, typename X>
__device__ __forceinline__ auto lds_if(X* p) {
  if constexpr (L) return (FBR_LDS_AS X*)p;
  else return p;
}

// Stable LSD radix sort of kb[0]/vb[0] (n pairs) over the low nbits key bits; returns the index
// (0/1) of the buffers holding the sorted pairs.  Ends with a barrier.
template <int T, typename V, int MAXD = 9, bool KV_LDS = true>
__device__ int vg_radix_sort(uint32_t* (&kb)[2], V* (&vb)[2], int n, int nbits, uint32_t* hist, uint32_t* wsum,
                             int dbg = 0) {
  constexpr int NW = T / 64, NB = 1 << MAXD;  // digits of <= MAXD bits; hist rows of NB counters
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int passes = dbg == 1 ? 0 : (nbits + MAXD - 1) / MAXD;
  const int dbits = passes > 0 ? (nbits + passes - 1) / passes : MAXD;
  const int nbins = 1 << dbits;
  const int chunk = (((n + NW - 1) / NW) + 63) & ~63;
  const int c0 = min(n, w * chunk), c1 = min(n, c0 + chunk);
  // Counters live at hist[w * NB + d] (lanes of one wave hit distinct banks); the exclusive scan
  // runs over them in digit-major, wave-minor order, which gives every (digit, wave) its output
  // base (waves in chunk order -> stable)
  constexpr int PER = NB * NW / T;
  int cur = 0;
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = dbits * pass;
    const uint32_t dmask = (uint32_t)nbins - 1u;
    const int tot = nbins * NW;
    const auto kin = lds_if<KV_LDS>(kb[cur]);
    const auto vin = lds_if<KV_LDS>(vb[cur]);
    const auto kout = lds_if<KV_LDS>(kb[cur ^ 1]);
    const auto vout = lds_if<KV_LDS>(vb[cur ^ 1]);
    for (int b = tid; b < tot; b += T) hist[(b % NW) * NB + b / NW] = 0u;
    __syncthreads();
    // per-wave digit counts: one add per distinct digit of a 64-step, by the lowest lane holding it
    // (ballot peer masks; per-element LDS atomics serialise on the long equal-digit runs that
    // spatially ordered keys have in their upper digits)
    for (int i0 = c0; i0 < c1; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < c1;
      const uint32_t d = valid ? (kin[i] >> shift) & dmask : 0u;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < dbits; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
      if (valid && (peers & ((1ull << lane) - 1ull)) == 0ull) hist[w * NB + d] += (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    {
      uint32_t v[PER], loc = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid * PER + k;
        v[k] = idx < tot ? hist[(idx % NW) * NB + idx / NW] : 0u;
        loc += v[k];
      }
      uint32_t inc = loc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t run = inc - loc;
      for (int ww = 0; ww < w; ++ww) run += wsum[ww];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid * PER + k;
        if (idx < tot) hist[(idx % NW) * NB + idx / NW] = run;
        run += v[k];
      }
    }
    __syncthreads();
    for (int i0 = c0; i0 < c1; i0 += 64) {
      const int i = i0 + lane;
      const bool valid = i < c1;
      const uint32_t key = valid ? kin[i] : 0u;
      const uint32_t d = (key >> shift) & dmask;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < dbits; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
      const int rank = __popcll(peers & ((1ull << lane) - 1ull));
      uint32_t* hc = &hist[w * NB + d];
      const uint32_t base = valid ? *hc : 0u;
      if (valid) {
        kout[base + rank] = key;
        vout[base + rank] = vin[i];
      }
      __builtin_amdgcn_wave_barrier();
      if (valid && rank == 0) *hc = base + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    cur ^= 1;
    __syncthreads();
  }
  return cur;
}

// Stable in-place LSD radix sort of an LDS-resident segment (n <= T * KPL pairs): every wave keeps
// its chunk (KPL 64-element steps) in registers, so a pass reads the whole chunk before the barrier
// and scatters straight into the same LDS arrays after it -- no ping-pong buffer, no global scratch.
// The ranking is vg_radix_sort's (wave chunks in order, ballot peer masks), so the sort is stable.
// 8-bit digits (hist holds (NW + 1) * 256 counters).  Ends with a barrier.  Always inlined: with
// two callers (the exact and default kernels) the compiler outlined it, and the call frame put
// 80 B per lane in scratch (spilled on every call: ~50 MB of writes per B = 1024 launch).
// kLeader (diagnostic, fbr_selftest_radix_sort only): 1 = per-wave digit counts by the lowest lane
// of each digit's ballot peer group instead of LDS atomics; 2 = that, plus round 3's wave-uniform
// early exit (`if (c0 + 64 * k >= c1) break;`) in the count and scatter loops: the exact form that
// mis-sorted in round 3.
template <int T, int KPL, int kLeader = 0>
__device__ __attribute__((always_inline)) void vg_radix_sort_inplace(FBR_LDS_AS uint32_t* keys, FBR_LDS_AS uint16_t* vals, int n, int nbits,
                                      uint32_t* hist, uint32_t* wsum) {
  constexpr int NW = T / 64, NB = 256, PER = NB * NW / T;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int passes = (nbits + 7) / 8;
  const int dbits = passes > 0 ? (nbits + passes - 1) / passes : 8;
  const uint32_t dmask = (1u << dbits) - 1u;
  const int nbins = 1 << dbits, tot = nbins * NW;
  const int chunk = (((n + NW - 1) / NW) + 63) & ~63;
  const int c0 = min(n, w * chunk), c1 = min(n, c0 + chunk);
  uint32_t kr[KPL], vr[KPL];
  for (int pass = 0; pass < passes; ++pass) {
    const int shift = dbits * pass;
#pragma unroll
    for (int k = 0; k < KPL; ++k) {
      const int i = c0 + 64 * k + lane;
      kr[k] = i < c1 ? keys[i] : 0u;
      vr[k] = i < c1 ? vals[i] : 0u;
    }
    for (int b = tid; b < tot; b += T) hist[(b % NW) * NB + b / NW] = 0u;
    __syncthreads();  // every wave holds its chunk: the scatter below may overwrite any position
    if constexpr (kLeader != 0) {
#pragma unroll
      for (int k = 0; k < KPL; ++k) {
        if constexpr (kLeader == 2)
          if (c0 + 64 * k >= c1) break;  // wave-uniform
        const bool valid = c0 + 64 * k + lane < c1;
        const uint32_t d = (kr[k] >> shift) & dmask;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < dbits; ++b) {
          const uint64_t bal = __ballot((d >> b) & 1u);
          peers &= ((d >> b) & 1u) ? bal : ~bal;
        }
        if (valid && (peers & ((1ull << lane) - 1ull)) == 0ull) hist[w * NB + d] += (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
      }
    } else {
#pragma unroll
      for (int k = 0; k < KPL; ++k)
        if (c0 + 64 * k + lane < c1) atomicAdd(&hist[w * NB + ((kr[k] >> shift) & dmask)], 1u);
    }
    __syncthreads();
    {
      uint32_t v[PER], loc = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid * PER + k;
        v[k] = idx < tot ? hist[(idx % NW) * NB + idx / NW] : 0u;
        loc += v[k];
      }
      uint32_t inc = loc;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t run = inc - loc;
      for (int ww = 0; ww < w; ++ww) run += wsum[ww];
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int idx = tid * PER + k;
        if (idx < tot) hist[(idx % NW) * NB + idx / NW] = run;
        run += v[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KPL; ++k) {
      if constexpr (kLeader == 2)
        if (c0 + 64 * k >= c1) break;  // wave-uniform: the rest of the chunk is empty
      const bool valid = c0 + 64 * k + lane < c1;
      const uint32_t d = (kr[k] >> shift) & dmask;
      uint64_t peers = __ballot(valid);
      for (int b = 0; b < dbits; ++b) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
      }
      const int rank = __popcll(peers & ((1ull << lane) - 1ull));
      uint32_t* hc = &hist[w * NB + d];
      const uint32_t base = valid ? *hc : 0u;
      if (valid) {
        keys[base + rank] = kr[k];
        vals[base + rank] = (uint16_t)vr[k];
      }
      __builtin_amdgcn_wave_barrier();
      if (valid && rank == 0) *hc = base + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
  }
}

// Stable radix sort of kb[0]/vb[0] (n pairs), then one centroid per run of equal keys in
// ascending key order: out[v] = mean of in[vals of the run].  Returns the voxel count (all threads).
template <int T, typename V, int MAXD = 9, bool KV_LDS = true>
__device__ int vg_sort_emit(uint32_t* (&kb)[2], V* (&vb)[2], int n, int nbits, uint32_t* hist, uint32_t* wsum,
                            const float4* in, float4* out, int dbg = 0, unsigned long long* t_sorted = nullptr);

// One centroid per run of equal keys of the sorted pairs ks / vs (n), in ascending key order.
// hist must hold NW KB (the per-wave point stage), and with kStage NW * 2176 B: the centroids then
// collect in a per-wave LDS ring of kEmitRing and leave as whole 128-B lines (a step completes a
// few scattered centroids, and partial-line stores cost the L2 a write each time the line is
// evicted half written).  Returns the voxel count (all threads).
constexpr int kEmitRing = 72;  // >= 7 unflushed + 65 written in one step (see the flush below)
template <int T, bool kStage = false, typename KP, typename VP>
__device__ int vg_emit(KP ks, VP vs, int n, uint32_t* hist, uint32_t* wsum, const float4* in, float4* out) {
  constexpr int NW = T / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int chunk = (((n + NW - 1) / NW) + 63) & ~63;
  const int c0 = min(n, w * chunk), c1 = min(n, c0 + chunk);
  // ---- voxels in ascending key order: heads of equal-key runs, centroid = float sum / count ----
  int nh = 0;
  for (int i0 = c0; i0 < c1; i0 += 64) {
    const int i = i0 + lane;
    nh += __popcll(__ballot(i < c1 && (i == 0 || ks[i] != ks[i - 1])));
  }
  if (lane == 0) wsum[w] = (uint32_t)nh;
  __syncthreads();
  int pos = 0;
  for (int ww = 0; ww < w; ++ww) pos += (int)wsum[ww];
  int total = pos;
  for (int ww = w; ww < NW; ++ww) total += (int)wsum[ww];
  // Runs of equal keys are summed in sorted order (the serial float sum of the reference) out of a
  // per-wave LDS stage of the current 64-step (the digit histogram is free after the sort): every
  // lane gathers its own sorted point (one parallel gather per step), a run's first lane adds the
  // following staged points up to the next key break (independent LDS reads, no load chain), and
  // a run still open at the end of the step is carried into the next step by lane 0 -- past c1 if
  // it continues into the next wave's chunk.
  float4* stg = reinterpret_cast<float4*>(hist) + w * 64;  // NW*1 KB <= (NW+1)*NB*4 B
  bool carry_open = false;
  float4 carry = make_float4(0.f, 0.f, 0.f, 0.f);
  int carry_start = 0, carry_out = 0;
  // kStage: this wave's voxels are [pos0, pos0 + nh); those below fl have been stored.  Every
  // index below the frontier (the open carry's, else pos) is written after a step, and a step
  // writes indices <= frontier + 64, so the live ring entries span < 8 + 65 <= kEmitRing.
  float4* ost = reinterpret_cast<float4*>(hist) + NW * 64 + w * kEmitRing;
  const int pos0 = pos;
  int fl = pos0 & ~7;
  auto flush = [&](int fe) {  // store ring entries [fl, fe) (wave-uniform fe)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int b = fl; b < fe; b += 64) {
      const int idx = b + lane;
      if (idx < fe && idx >= pos0) out[idx] = ost[idx % kEmitRing];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    fl = fe;
  };
  // the gathers run one step ahead (the loop is otherwise one dependent HBM/L2 round trip per step)
  float4 pnext = c0 + lane < n && c0 < c1 ? in[vs[c0 + lane]] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i0 = c0; i0 < c1 || carry_open; i0 += 64) {
    const int i = i0 + lane;
    const bool valid = i < n;
    const uint32_t key = valid ? ks[i] : 0u;
    const bool brk_i = !valid || i == 0 || ks[i - 1] != key;  // a run starts here (or no point)
    const bool head = valid && i < c1 && brk_i;
    const bool cont = carry_open && lane == 0;  // continues the carried run (brk_i is false)
    const uint64_t brk = __ballot(brk_i), hb = __ballot(head);
    const float4 p = valid ? pnext : make_float4(0.f, 0.f, 0.f, 0.f);
    pnext = i + 64 < n ? in[vs[i + 64]] : make_float4(0.f, 0.f, 0.f, 0.f);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    stg[lane] = p;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t after = lane == 63 ? 0ull : (brk >> (lane + 1)) << (lane + 1);
    const int nb = after ? __ffsll((unsigned long long)after) - 1 : 64;  // next break after this lane
    float4 c = p;
    if (cont) {
      c.x = carry.x + p.x;
      c.y = carry.y + p.y;
      c.z = carry.z + p.z;
      c.w = carry.w + p.w;
    }
    const bool starter = head || cont;
    if (starter)
      for (int k = lane + 1; k < nb; k += 4) {  // four staged reads in flight, adds in order
        float4 q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) q[u] = stg[min(k + u, 63)];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k + u < nb) {
            c.x += q[u].x;
            c.y += q[u].y;
            c.z += q[u].z;
            c.w += q[u].w;
          }
      }
    const bool spills = starter && nb == 64 && i0 + 64 < n && ks[i0 + 64] == key;
    const int start = cont ? carry_start : i;
    const int oidx = cont ? carry_out : pos + __popcll(hb & ((1ull << lane) - 1ull));
    if (starter && !spills) {
      const float cnt = (float)(i0 + nb - start);
      const float4 r = make_float4(c.x / cnt, c.y / cnt, c.z / cnt, c.w / cnt);
      if constexpr (kStage) ost[oidx % kEmitRing] = r;
      else out[oidx] = r;
    }
    const uint64_t sp = __ballot(spills);
    carry_open = sp != 0ull;
    if (carry_open) {
      const int src = __ffsll((unsigned long long)sp) - 1;
      carry = make_float4(__shfl(c.x, src), __shfl(c.y, src), __shfl(c.z, src), __shfl(c.w, src));
      carry_start = __shfl(start, src);
      carry_out = __shfl(oidx, src);
    }
    pos += __popcll(hb);
    if constexpr (kStage) {
      const int fe = (carry_open ? carry_out : pos) & ~7;
      if (fe > fl) flush(fe);
    }
  }
  if constexpr (kStage) flush(pos);
  return total;
}

template <int T, typename V, int MAXD, bool KV_LDS>
__device__ int vg_sort_emit(uint32_t* (&kb)[2], V* (&vb)[2], int n, int nbits, uint32_t* hist, uint32_t* wsum,
                            const float4* in, float4* out, int dbg, unsigned long long* t_sorted) {
  const int cur = vg_radix_sort<T, V, MAXD, KV_LDS>(kb, vb, n, nbits, hist, wsum, dbg);
  if (t_sorted && threadIdx.x == 0) *t_sorted = __builtin_amdgcn_s_memtime();
  if (dbg == 2) return 0;
  return vg_emit<T>(lds_if<KV_LDS>(kb[cur]), lds_if<KV_LDS>(vb[cur]), n, hist, wsum, in, out);
}

// Generic front end: segments of a VgArgs (per-job mapping DS, start-up map filter, fbr_voxel_grid).
template <int T, typename V, bool LDS, bool kExact>
__global__ void __launch_bounds__(T) k_voxel_grid(VgArgs A) {
  constexpr int NW = T / 64;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  int seg = blockIdx.x;
  const bool second = seg >= A.s[0].nseg;
  const VgSet S = second ? A.s[1] : A.s[0];
  if (second) seg -= A.s[0].nseg;
  uint32_t* hist = (uint32_t*)smem;  // [NW + 1][512]: per-wave digit counters + digit totals
  uint32_t* wsum = hist + (NW + 1) * 512;
  float* mm = (float*)(wsum + NW);
  int* misc = (int*)(mm + NW * 6);
  const int n = (int)min((int64_t)S.cnt_in[seg], S.cap);
  const float4* in = S.in + (int64_t)seg * S.stride_in;
  float4* out = S.out + (int64_t)seg * S.stride_out;
  if (n <= 0) {
    if (tid == 0) S.cnt_out[seg] = 0;
    return;
  }
  float mn[3], mx[3];
  vg_seg_bounds<T>(S, seg, n, in, mn, mx, mm);
  VgGrid G;
  G.init(mn, mx, S.leaf, S.morton != 0);
  if (G.overflow) {
    for (int i = tid; i < n; i += T) out[i] = in[i];
    if (tid == 0) S.cnt_out[seg] = n;
    return;
  }
  uint32_t* kb[2];
  V* vb[2];
  if constexpr (LDS) {
    unsigned char* q = smem + ((((unsigned char*)(misc + 4) - smem) + 15) & ~15);  // keeps the LDS address space
    const int cap = (int)S.cap;
    kb[0] = (uint32_t*)q;
    kb[1] = kb[0] + cap;
    vb[0] = (V*)(kb[1] + cap);
    vb[1] = vb[0] + cap;
  } else {
    uint32_t* sc = S.scratch + (int64_t)seg * kVgScratch * S.cap;
    kb[0] = sc;
    kb[1] = sc + S.cap;
    vb[0] = (V*)(sc + 2 * S.cap);
    vb[1] = (V*)(sc + 3 * S.cap);
  }
  for (int i = tid; i < n; i += T) {
    kb[0][i] = kExact ? G.pcl_key(in[i]) : G.key(in[i]);
    vb[0][i] = (V)i;
  }
  __syncthreads();
  if constexpr (kExact) {  // PCL's order inside a voxel: std::sort's partition phase, then the stable sort
    const int cap = (int)S.cap, nf = 3 * (cap / 17 + 2);
    if constexpr (LDS) {
      FBR_LDS_AS uint16_t* pl = (FBR_LDS_AS uint16_t*)kb[1];  // the free ping-pong half
      FBR_LDS_AS int* fr = (FBR_LDS_AS int*)hist;
      is_partition_phase<T>((FBR_LDS_AS uint32_t*)kb[0], (FBR_LDS_AS V*)vb[0], pl, pl + cap, n, fr, fr + nf, (int*)wsum);
    } else {
      int* fr = (int*)(S.scratch + (int64_t)seg * kVgScratch * S.cap + 4 * S.cap);
      is_partition_phase<T>(kb[0], vb[0], (int32_t*)kb[1], (int32_t*)vb[1], n, fr, fr + nf, (int*)wsum);
    }
    if (G.morton) {
      for (int i = tid; i < n; i += T) kb[0][i] = G.out_key(kb[0][i]);
      __syncthreads();
    }
  }
  const int total = vg_sort_emit<T, V, 9, LDS>(kb, vb, n, G.nbits, hist, wsum, in, out);
  if (tid == 0) S.cnt_out[seg] = total;
}

// Mapping-DS front end (downsampleCurrentScan, one 1024-thread workgroup per job cloud): segments
// of up to T * KPL points sort in place in LDS (keys u32 + u16 indices, vg_radix_sort_inplace), so
// the only global writes are the centroids; larger segments take the global-scratch ping-pong of
// k_voxel_grid.  Same semantics and output as k_voxel_grid.
#ifdef FBR_VG_STAMPS
// Diagnostic builds only: s_memtime at the phase boundaries of k_voxel_grid_ip's workgroup 0
// (start, grid set-up, keys, sort, emit), read by fbr_diag_vg_stamps.
__device__ unsigned long long fbr_vg_stamps[8];
#define FBR_VG_STAMP(k)                                                                       \
  do {                                                                                        \
    __syncthreads();                                                                          \
    if (blockIdx.x == 0 && threadIdx.x == 0) fbr_vg_stamps[k] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define FBR_VG_STAMP(k) \
  do {                  \
  } while (0)
#endif

template <int T, int KPL, bool kExact>
__global__ void __launch_bounds__(T) k_voxel_grid_ip(VgArgs A) {
  constexpr int NW = T / 64, LCAP = T * KPL;
  static_assert(NW * (64 + kEmitRing) * 16 <= (NW + 1) * 512 * 4, "vg_emit's point stage + centroid ring exceed hist");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  int seg = blockIdx.x;
  const bool second = seg >= A.s[0].nseg;
  const VgSet S = second ? A.s[1] : A.s[0];
  if (second) seg -= A.s[0].nseg;
  uint32_t* hist = (uint32_t*)smem;  // [NW + 1][512] (global path) / [NW + 1][256] (in place)
  uint32_t* wsum = hist + (NW + 1) * 512;
  float* mm = (float*)(wsum + NW);
  int* misc = (int*)(mm + NW * 6);
  FBR_VG_STAMP(0);
  const int n = (int)min((int64_t)S.cnt_in[seg], S.cap);
  const float4* in = S.in + (int64_t)seg * S.stride_in;
  float4* out = S.out + (int64_t)seg * S.stride_out;
  if (n <= 0) {
    if (tid == 0) S.cnt_out[seg] = 0;
    return;
  }
  float mn[3], mx[3];
  vg_seg_bounds<T>(S, seg, n, in, mn, mx, mm);
  VgGrid G;
  G.init(mn, mx, S.leaf, S.morton != 0);
  FBR_VG_STAMP(1);
  if (G.overflow) {
    for (int i = tid; i < n; i += T) out[i] = in[i];
    if (tid == 0) S.cnt_out[seg] = n;
    return;
  }
  int total;
  if (n <= LCAP) {
    unsigned char* q = smem + ((((unsigned char*)(misc + 4) - smem) + 15) & ~15);
    FBR_LDS_AS uint32_t* keys = (FBR_LDS_AS uint32_t*)q;
    FBR_LDS_AS uint16_t* vals = (FBR_LDS_AS uint16_t*)((FBR_LDS_AS uint32_t*)q + LCAP);
    for (int i = tid; i < n; i += T) {
      keys[i] = kExact ? G.pcl_key(in[i]) : G.key(in[i]);
      vals[i] = (uint16_t)i;
    }
    __syncthreads();
    if constexpr (kExact) {  // PCL's order inside a voxel: std::sort's partition phase, then the stable sort
      int32_t* sc = (int32_t*)(S.scratch + (int64_t)seg * kVgScratch * S.cap);  // positions (global)
      FBR_LDS_AS int* fr = (FBR_LDS_AS int*)hist;
      is_partition_phase<T>(keys, vals, sc, sc + S.cap, n, fr, fr + 3 * (LCAP / 17 + 2), (int*)wsum);
      if (G.morton) {
        for (int i = tid; i < n; i += T) keys[i] = G.out_key(keys[i]);
        __syncthreads();
      }
    }
    FBR_VG_STAMP(2);
    vg_radix_sort_inplace<T, KPL>(keys, vals, n, G.nbits, hist, wsum);
    FBR_VG_STAMP(3);
    total = vg_emit<T, true>(keys, vals, n, hist, wsum, in, out);  // hist: (NW + 1) * 2 KB
    FBR_VG_STAMP(4);
  } else {
    uint32_t* sc = S.scratch + (int64_t)seg * kVgScratch * S.cap;
    uint32_t* kb[2] = {sc, sc + S.cap};
    uint32_t* vb[2] = {sc + 2 * S.cap, sc + 3 * S.cap};
    for (int i = tid; i < n; i += T) {
      kb[0][i] = kExact ? G.pcl_key(in[i]) : G.key(in[i]);
      vb[0][i] = (uint32_t)i;
    }
    __syncthreads();
    if constexpr (kExact) {
      int* fr = (int*)(sc + 4 * S.cap);
      is_partition_phase<T>(kb[0], vb[0], (int32_t*)kb[1], (int32_t*)vb[1], n, fr, fr + 3 * ((int)S.cap / 17 + 2),
                            (int*)wsum);
      if (G.morton) {
        for (int i = tid; i < n; i += T) kb[0][i] = G.out_key(kb[0][i]);
        __syncthreads();
      }
    }
    total = vg_sort_emit<T, uint32_t, 9, false>(kb, vb, n, G.nbits, hist, wsum, in, out);
  }
  if (tid == 0) S.cnt_out[seg] = total;
}

// Few segments (single-scan calls: one corner and one surf cloud) leave all but two CUs idle in
// k_voxel_grid_ip.  Here P workgroups share a segment (block = seg * P + part): each computes the
// grid and a histogram of the keys' top bits over the whole cloud (the same in every part), keeps
// the points of its key range (the bins between the n * part / P and n * (part + 1) / P quantiles)
// in index order, sorts them in LDS and emits their voxels.  Equal keys share a bin, so every voxel
// lies in one part, and the parts' key ranges are ascending: part p's voxels go after the voxels of
// parts < p.  Each part publishes its voxel count as (gen << 32 | count) in flags[block], then reads
// the lower parts' counts (decoupled look-back: a lower block was dispatched earlier, so it runs to
// completion; the wait is bounded anyway, and gives up with a zero count rather than hang).  Same
// output as k_voxel_grid_ip (`test_split_voxel_grid_is_bit_identical`).  Default-order mode only.
template <int T, int KPL>
__global__ void __launch_bounds__(T) k_voxel_grid_split(VgArgs A, int P, unsigned long long* flags, unsigned gen) {
  constexpr int NW = T / 64, LCAP = T * KPL;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int blk = blockIdx.x, part = blk % P;
  int seg = blk / P;
  const bool second = seg >= A.s[0].nseg;
  const VgSet S = second ? A.s[1] : A.s[0];
  if (second) seg -= A.s[0].nseg;
  uint32_t* hist = (uint32_t*)smem;  // [NW + 1][256] in-place sort counters; 1024 key bins before
  uint32_t* wsum = hist + (NW + 1) * 512;
  float* mm = (float*)(wsum + NW);
  int* misc = (int*)(mm + NW * 6);
  const int n = (int)min((int64_t)S.cnt_in[seg], S.cap);
  const float4* in = S.in + (int64_t)seg * S.stride_in;
  float4* out = S.out + (int64_t)seg * S.stride_out;
  if (n <= 0) {
    if (tid == 0 && part == 0) S.cnt_out[seg] = 0;
    return;
  }
  float mn[3], mx[3];
  vg_seg_bounds<T>(S, seg, n, in, mn, mx, mm);
  VgGrid G;
  G.init(mn, mx, S.leaf, S.morton != 0);
  if (G.overflow) {  // PCL's "leaf size too small": output = input
    if (part == 0) {
      for (int i = tid; i < n; i += T) out[i] = in[i];
      if (tid == 0) S.cnt_out[seg] = n;
    }
    return;
  }
  if (n > LCAP) {  // over the LDS capacity: part 0 alone, k_voxel_grid_ip's global-scratch path
    if (part != 0) return;
    uint32_t* sc = S.scratch + (int64_t)seg * kVgScratch * S.cap;
    uint32_t* kb[2] = {sc, sc + S.cap};
    uint32_t* vb[2] = {sc + 2 * S.cap, sc + 3 * S.cap};
    for (int i = tid; i < n; i += T) {
      kb[0][i] = G.key(in[i]);
      vb[0][i] = (uint32_t)i;
    }
    __syncthreads();
    const int total = vg_sort_emit<T, uint32_t, 9, false>(kb, vb, n, G.nbits, hist, wsum, in, out);
    if (tid == 0) S.cnt_out[seg] = total;
    return;
  }
  // ---- key histogram over the top hb bits (every part computes the same) ----
  const int hb = min(10, G.nbits), sh = G.nbits - hb, nbin = 1 << hb;
  for (int b = tid; b < nbin; b += T) hist[b] = 0u;
  __syncthreads();
  // wave w owns the contiguous chunk [c0, c1) of the cloud (at most KPL steps of 64: n <= LCAP)
  // and keeps its keys in registers for the compaction below (one read of the cloud)
  const int per = (((n + NW - 1) / NW) + 63) & ~63;
  const int c0 = min(n, w * per), c1 = min(n, c0 + per);
  uint32_t kv[KPL];
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    const int i = c0 + 64 * k + lane;
    kv[k] = 0u;
    if (i < c1) {
      kv[k] = G.key(in[i]);
      atomicAdd(&hist[kv[k] >> sh], 1u);
    }
  }
  __syncthreads();
  // this part's bin range [b0, b1): the first bins whose inclusive prefix exceeds n * part / P
  // and n * (part + 1) / P (inclusive scan over the bins, one bin per thread, T >= 1024)
  {
    const uint32_t c = tid < nbin ? hist[tid] : 0u;
    uint32_t inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < w; ++k) pre += wsum[k];
    inc += pre;  // inclusive prefix of bin tid
    const uint32_t lo = (uint32_t)(((int64_t)n * part) / P), hi = (uint32_t)(((int64_t)n * (part + 1)) / P);
    // bin tid starts the range of part q when inc(tid - 1) <= n q / P < inc(tid): the bins of
    // part q are those whose exclusive prefix lies in [n q / P, n (q + 1) / P) -- every bin lands in
    // exactly one part, in order
    const uint32_t ex = inc - c;
    const bool mine = tid < nbin && c > 0 && ex >= lo && (part == P - 1 || ex < hi);
    __syncthreads();
    if (tid == 0) { misc[0] = nbin; misc[1] = -1; }
    __syncthreads();
    if (mine) atomicMin(&misc[0], tid);
    if (mine) atomicMax(&misc[1], tid);
    __syncthreads();
  }
  const int b0 = misc[0], b1 = misc[1];  // empty range: b0 = nbin, b1 = -1
  // ---- this part's points in index order: every wave counts its chunk's points, one prefix over
  // the waves, then each wave writes its chunk in order (chunks are in index order): two barriers
  // (a block-wide pass per 1024 points took two per pass) ----
  unsigned char* q = smem + ((((unsigned char*)(misc + 4) - smem) + 15) & ~15);
  FBR_LDS_AS uint32_t* keys = (FBR_LDS_AS uint32_t*)q;
  FBR_LDS_AS uint16_t* vals = (FBR_LDS_AS uint16_t*)((FBR_LDS_AS uint32_t*)q + LCAP);
  const uint64_t lt = (1ull << lane) - 1ull;
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    const int i = c0 + 64 * k + lane;
    const int b = (int)(kv[k] >> sh);
    cnt += __popcll(__ballot(i < c1 && b >= b0 && b <= b1));
  }
  if (lane == 0) wsum[w] = (uint32_t)cnt;
  __syncthreads();
  int pre = 0, nk = 0;
  for (int k = 0; k < NW; ++k) {
    if (k < w) pre += (int)wsum[k];
    nk += (int)wsum[k];
  }
#pragma unroll
  for (int k = 0; k < KPL; ++k) {
    const int i = c0 + 64 * k + lane;
    const int b = (int)(kv[k] >> sh);
    const bool keep = i < c1 && b >= b0 && b <= b1;
    const uint64_t m = __ballot(keep);
    if (keep) {
      const int pos = pre + __popcll(m & lt);
      keys[pos] = kv[k];
      vals[pos] = (uint16_t)i;
    }
    pre += __popcll(m);
  }
  __syncthreads();
  if (nk > 0) vg_radix_sort_inplace<T, KPL>(keys, vals, nk, G.nbits, hist, wsum);
  // ---- voxel count, publish, look back ----
  int heads = 0;
  for (int i = tid; i < nk; i += T) heads += (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
  for (int off = 32; off > 0; off >>= 1) heads += __shfl_xor(heads, off);
  __syncthreads();
  if (lane == 0) wsum[w] = (uint32_t)heads;
  __syncthreads();
  if (tid == 0) {
    uint32_t V = 0;
    for (int k = 0; k < NW; ++k) V += wsum[k];
    __hip_atomic_store(&flags[blk], ((unsigned long long)gen << 32) | V, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t off = 0;
    bool lost = false;
    for (int j = blk - part; j < blk; ++j) {
      unsigned long long f = 0;
      for (int spin = 0; spin < (1 << 24); ++spin) {
        f = __hip_atomic_load(&flags[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned)(f >> 32) == gen) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if ((unsigned)(f >> 32) == gen) off += (uint32_t)f;
      else lost = true;
    }
    // a lower part never published (the wait is a safety bound, it does not happen when the lower
    // blocks run): the offsets are unknown, so the segment is reported failed, never short
    if (lost && A.err) atomicOr(&A.err[seg], kVgErrLookback);
    misc[2] = (int)off;
    misc[3] = (int)V;
    misc[1] = lost ? 1 : 0;
  }
  __syncthreads();
  const int off = misc[2], V = misc[3];
  const bool lost = misc[1] != 0;
  if (nk > 0 && !lost) vg_emit<T, true>(keys, vals, nk, hist, wsum, in, out + off);
  if (tid == 0 && part == P - 1) S.cnt_out[seg] = lost ? (A.err ? 0 : -1) : off + V;
}

// Per-ring front end (featureExtraction.h:279-292): the surf candidates of (job, ring) are the
// points k of the ring's non-empty segments [sp, ep] (sp < ep, :195-200) with cloudLabel[k] <= 0,
// in index order, read straight from the projected cloud and the label mask (the label of
// index 4 may be stale across scans exactly as the reference's cloudLabel[4]).  One register
// pass feeds min/max, the keys and the compaction; the sort runs in LDS (u16 ring offsets).
template <int T, int KPT, bool kExact>
__global__ void __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(KPT <= 4 && !kExact ? 8 : 1)))
k_voxel_ring(VgRing A) {
  constexpr int NW = T / 64, MAXD = 8;  // 8-bit digits: 3 passes cover the <= 24-bit ring keys
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = blockIdx.x, job = slot / A.H;
#ifdef FBR_VR_STAMPS  // diagnostic build only (tools/vr_stamps.py): phase boundaries of wave 0
  unsigned long long ts[5] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0};
#define VR_TS(i) (ts[i] = __builtin_amdgcn_s_memtime())
#define VR_TS_PTR (&ts[3])
#else
#define VR_TS(i) ((void)0)
#define VR_TS_PTR nullptr
#endif
  uint32_t* hist = (uint32_t*)smem;
  uint32_t* wsum = hist + (NW + 1) * (1 << MAXD);
  float* mm = (float*)(wsum + NW);
  int* cnts = (int*)(mm + NW * 6);  // [KPT][NW]
  const int s = A.start_ring[slot], e = A.end_ring[slot];
  float4* out = A.out + (int64_t)slot * A.stride_out;
  if (e <= s) {
    if (tid == 0) A.cnt_out[slot] = 0;
    return;
  }
  int sp6[6], ep6[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    sp6[j] = (s * (6 - j) + e * j) / 6;
    ep6[j] = (s * (5 - j) + e * (j + 1)) / 6 - 1;
  }
  const float4* CL = A.cloud + (int64_t)job * A.HW + s;
  const int8_t* LB = A.label + (int64_t)job * A.HW;
  // segment j is [sp_j, sp_{j+1} - 1] (ep_j = sp_{j+1} - 1, ep_5 = e - 1): when all six are
  // non-empty (sp < ep) they tile [s, e - 1]
  bool all6 = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) all6 = all6 && sp6[j] < ep6[j];
  bool cd[KPT];
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  // Every label and point load issued before any is used (one round trip; clamped indices, and an
  // empty asm taking the values, or the compiler sinks each point load under its label test: a
  // chain of 2 * KPT dependent round trips).  The exact instance keeps its round-5 loads: the
  // hoisted form cost its partition phase's register allocation 25 % (voxel_ring 10.3 -> 12.8 ms per
  // B = 1024 step, profiles/r06y_voxel_ring_loads_ab.txt).
  int lbr[KPT];
  float4 pr[KPT];
  if constexpr (!kExact) {
#pragma unroll
    for (int r = 0; r < KPT; ++r) {
      const int kc = min(s + r * T + tid, e - 1);
      lbr[r] = LB[kc];
      pr[r] = CL[kc - s];
    }
#pragma unroll
    for (int r = 0; r < KPT; ++r) asm volatile("" ::"v"(lbr[r]), "v"(pr[r].x), "v"(pr[r].y), "v"(pr[r].z));
  }
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    const int k = s + r * T + tid;
    bool in = false;
    if (all6) {
      in = k <= ep6[5];
    } else {
#pragma unroll
      for (int j = 0; j < 6; ++j) in |= sp6[j] < ep6[j] && k >= sp6[j] && k <= ep6[j];
    }
    float4 p;
    if constexpr (kExact) {
      const int8_t lab = in ? LB[k] : (int8_t)1;
      p = in ? CL[k - s] : make_float4(0.f, 0.f, 0.f, 0.f);
      cd[r] = lab <= 0;
    } else {
      p = pr[r];
      cd[r] = in && lbr[r] <= 0;
    }
    if (cd[r]) {
      const float v[3] = {p.x, p.y, p.z};
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        mn[d] = (v[d] < mn[d]) ? v[d] : mn[d];
        mx[d] = (mx[d] < v[d]) ? v[d] : mx[d];
      }
    }
  }
  // compaction positions in index order: per step r, waves in order
  uint64_t bal[KPT];
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    bal[r] = __ballot(cd[r]);
    if (lane == 0) cnts[r * NW + w] = __popcll(bal[r]);
  }
  vg_block_minmax<T>(mn, mx, mm);  // (its barrier also publishes cnts)
  int n = 0, pos[KPT];
#pragma unroll
  for (int r = 0; r < KPT; ++r) {
    int before = 0, all = 0;
    for (int ww = 0; ww < NW; ++ww) {
      const int c = cnts[r * NW + ww];
      before += ww < w ? c : 0;
      all += c;
    }
    pos[r] = n + before + __popcll(bal[r] & ((1ull << lane) - 1ull));
    n += all;
  }
  if (n == 0 || A.dbg == 3) {
    if (tid == 0) A.cnt_out[slot] = 0;
    return;
  }
  VR_TS(1);
  VgGrid G;
  G.init(mn, mx, A.leaf, false);
  unsigned char* q = smem + ((((unsigned char*)(cnts + KPT * NW) - smem) + 15) & ~15);  // keeps the LDS address space
  const int cap = (int)A.cap;
  uint32_t* kb[2];   // [0]: candidate keys in index order, then run keys; sort ping-pong
  uint16_t* vb[2];   // run ids; sort ping-pong
  kb[0] = (uint32_t*)q;
  kb[1] = kb[0] + cap;
  vb[0] = (uint16_t*)(kb[1] + cap);
  vb[1] = vb[0] + cap;
  uint16_t* off = vb[1] + cap;  // [cap] ring offset of the t-th candidate
  uint16_t* rst = off + cap;    // [cap + 1] first candidate of each run, rst[R] = n
  if (G.overflow) {  // output = input, in index order
#pragma unroll
    for (int r = 0; r < KPT; ++r)
      if (cd[r]) out[pos[r]] = CL[r * T + tid];
    if (tid == 0) A.cnt_out[slot] = n;
    return;
  }
#pragma unroll
  for (int r = 0; r < KPT; ++r)
    if (cd[r]) {
      kb[0][pos[r]] = G.key(CL[r * T + tid]);  // re-read (L2): no point registers live across the barrier
      off[pos[r]] = (uint16_t)(r * T + tid);   // offset from the ring start s
    }
  __syncthreads();
  if constexpr (kExact) {
    // PCL's order inside a voxel: std::sort's partition phase on (key, offset) (fbr_introsort.h);
    // everything below treats the permuted sequence as the input order, and its stable run sort
    // completes std::sort.  Scratch: the free ping-pong half kb[1] (positions, u16), the digit
    // histogram (frame lists) and wsum.. (the workgroup's scan slots).
    FBR_LDS_AS uint16_t* pl = (FBR_LDS_AS uint16_t*)kb[1];
    FBR_LDS_AS int* fr = (FBR_LDS_AS int*)hist;
    // frames above 512 points are partitioned by the whole workgroup (the top levels of a ring)
    is_partition_phase<T, FBR_LDS_AS uint32_t*, FBR_LDS_AS uint16_t*, FBR_LDS_AS uint16_t*, FBR_LDS_AS int*, 512>(
        (FBR_LDS_AS uint32_t*)kb[0], (FBR_LDS_AS uint16_t*)off, pl, pl + cap, n, fr, fr + 3 * (cap / 17 + 2), (int*)wsum);
  }
  VR_TS(2);
  // Runs of equal keys in index order (points adjacent along the ring share voxels: ~6.6
  // candidates per run on C2, and nearly one run per voxel).  Only the runs are sorted; the
  // stable sort keeps a voxel's runs in index order, so its points are still summed in index order.
  const int chunk = (((n + NW - 1) / NW) + 63) & ~63;
  const int c0 = min(n, w * chunk), c1 = min(n, c0 + chunk);
  uint32_t rkey[KPT];
  uint64_t hb[KPT];
  int nrun = 0;
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    const int t = c0 + 64 * k + lane;
    const bool valid = t < c1;
    const uint32_t key = valid ? kb[0][t] : 0u;
    hb[k] = __ballot(valid && (t == 0 || kb[0][t - 1] != key));
    rkey[k] = key;
    nrun += __popcll(hb[k]);
  }
  if (lane == 0) wsum[w] = (uint32_t)nrun;
  __syncthreads();  // every candidate key is read before the run keys overwrite them
  int rq = 0, R = 0;
  for (int ww = 0; ww < NW; ++ww) {
    const int cw = (int)wsum[ww];
    rq += ww < w ? cw : 0;
    R += cw;
  }
#pragma unroll
  for (int k = 0; k < KPT; ++k) {
    if ((hb[k] >> lane) & 1ull) {
      const int qq = rq + __popcll(hb[k] & ((1ull << lane) - 1ull));
      kb[0][qq] = rkey[k];
      vb[0][qq] = (uint16_t)qq;
      rst[qq] = (uint16_t)(c0 + 64 * k + lane);
    }
    rq += __popcll(hb[k]);
  }
  if (tid == 0) rst[R] = (uint16_t)n;
  __syncthreads();
  const int cur = vg_radix_sort<T, uint16_t, MAXD>(kb, vb, R, G.nbits, hist, wsum, A.dbg);
  VR_TS(3);
  if (A.dbg == 2) {
    if (tid == 0) A.cnt_out[slot] = 0;
    return;
  }
  // voxels = groups of equal keys in sorted run order: voxel index of each group's first run and
  // the next run of the same voxel, scattered by run id into the free ping-pong halves
  const FBR_LDS_AS uint32_t* ks = (const FBR_LDS_AS uint32_t*)kb[cur];
  const FBR_LDS_AS uint16_t* vs = (const FBR_LDS_AS uint16_t*)vb[cur];
  FBR_LDS_AS int32_t* nxt = (FBR_LDS_AS int32_t*)kb[cur ^ 1];
  FBR_LDS_AS uint16_t* vox = (FBR_LDS_AS uint16_t*)vb[cur ^ 1];
  const int rchunk = (((R + NW - 1) / NW) + 63) & ~63;
  const int r0 = min(R, w * rchunk), r1 = min(R, r0 + rchunk);
  int nh = 0;
  for (int i0 = r0; i0 < r1; i0 += 64) {
    const int i = i0 + lane;
    nh += __popcll(__ballot(i < r1 && (i == 0 || ks[i] != ks[i - 1])));
  }
  if (lane == 0) wsum[w] = (uint32_t)nh;
  __syncthreads();
  int vpos = 0, total = 0;
  for (int ww = 0; ww < NW; ++ww) {
    const int cw = (int)wsum[ww];
    vpos += ww < w ? cw : 0;
    total += cw;
  }
  for (int i0 = r0; i0 < r1; i0 += 64) {
    const int i = i0 + lane;
    const bool valid = i < r1;
    const uint32_t key = valid ? ks[i] : 0u;
    const bool head = valid && (i == 0 || ks[i - 1] != key);
    const uint64_t bh = __ballot(head);
    if (valid) {
      const int rid = vs[i];
      vox[rid] = head ? (uint16_t)(vpos + __popcll(bh & ((1ull << lane) - 1ull))) : (uint16_t)0xFFFFu;
      nxt[rid] = (i + 1 < R && ks[i + 1] == key) ? (int32_t)vs[i + 1] : -1;
    }
    vpos += __popcll(bh);
  }
  __syncthreads();
  // one lane per voxel (at its first run, in index order): the reference's serial float sum over
  // the voxel's points in index order, four loads in flight
  for (int rid = tid; rid < R; rid += T) {
    const int v = vox[rid];
    if (v == 0xFFFF) continue;
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
    for (int qq = rid; qq >= 0; qq = nxt[qq]) {
      const int t0 = rst[qq], t1 = rst[qq + 1];
      for (int t = t0; t < t1; t += 4) {
        float4 pp[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pp[u] = CL[off[min(t + u, t1 - 1)]];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (t + u < t1) {
            if (cnt == 0) {
              c = pp[u];
            } else {
              c.x += pp[u].x;
              c.y += pp[u].y;
              c.z += pp[u].z;
              c.w += pp[u].w;
            }
            ++cnt;
          }
      }
    }
    const float fc = (float)cnt;
    out[v] = make_float4(c.x / fc, c.y / fc, c.z / fc, c.w / fc);
  }
  if (tid == 0) A.cnt_out[slot] = total;
#ifdef FBR_VR_STAMPS
  VR_TS(4);
  if (tid == 0 && A.stamps)
    for (int i = 0; i < 5; ++i) A.stamps[(int64_t)slot * 12 + i] = ts[i];
#endif
#undef VR_TS
#undef VR_TS_PTR
}

// ---- register helpers of the four-wave per-ring surf filter (k_voxel_ring_q below) ----
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t x, int m) {
  const uint32_t lo = __shfl_xor((uint32_t)x, m), hi = __shfl_xor((uint32_t)(x >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

// Ascending bitonic sort of 64 * E distinct u64 values held lane-major (element g = lane * E + e):
// compare-exchanges inside a lane for distances below E, xor lane exchanges above.  The values are
// below kF64KeyMax (a run key < 2^32 shifted by 16, or the padding kF64KeyMax), so the exchanges
// take their minima / maxima on the f64 unit (key_min / key_max, fbr_common.h).
template <int E>
__device__ __forceinline__ void wave_bitonic_u64(uint64_t (&v)[E], int lane) {
  constexpr int N = 64 * E;
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= E) {
        const int m = j / E;
        const bool lower = (lane & m) == 0;
        const bool asc = ((lane * E) & k) == 0;  // k > j >= E: the same for all e of the lane
        const bool take_min = lower == asc;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const uint64_t o = shfl_xor_u64(v[e], m);
          v[e] = take_min ? key_min(o, v[e]) : key_max(o, v[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if (e & j) continue;
          const bool asc = ((lane * E + e) & k) == 0;
          const uint64_t a = v[e], b = v[e | j];
          const uint64_t lo = key_min(a, b), hi = key_max(a, b);
          v[e] = asc ? lo : hi;
          v[e | j] = asc ? hi : lo;
        }
      }
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// Sorted run ids sid[0, R) and voxel starts vst[0, V] (vst[V] = R) from the register-sorted values.
template <int E>
__device__ int vr_sort_runs(const uint32_t* kb, int R, uint16_t* sid, uint16_t* vst, int lane) {
  uint64_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int g = lane * E + e;
    v[e] = g < R ? (((uint64_t)kb[g] << 16) | (uint64_t)g) : kF64KeyMax;
  }
  wave_bitonic_u64<E>(v, lane);
  const uint32_t lo = __shfl_up((uint32_t)v[E - 1], 1), hi = __shfl_up((uint32_t)(v[E - 1] >> 32), 1);
  const uint64_t prev_last = ((uint64_t)hi << 32) | lo;
  bool hd[E];
  int nh = 0;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int g = lane * E + e;
    const uint64_t pk = e ? (v[e - 1] >> 16) : (prev_last >> 16);
    hd[e] = g < R && (g == 0 || (v[e] >> 16) != pk);
    nh += hd[e] ? 1 : 0;
  }
  int inc = nh;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  const int V = __shfl(inc, 63);
  int vi = inc - nh;
  wave_lds_sync();  // every lane read its kb values (sid overwrites them)
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int g = lane * E + e;
    if (g < R) sid[g] = (uint16_t)(v[e] & 0xFFFFull);
    if (hd[e]) vst[vi++] = (uint16_t)g;
  }
  if (lane == 0) vst[V] = (uint16_t)R;
  wave_lds_sync();
  return V;
}

// ---- the per-ring surf filter, four waves per ring (default order) ----
// The same filter as k_voxel_ring for the index-order sums with a ring's memory round trips cut to
// about three: each of the 4 waves loads a quarter of the ring's labels and points in one go (up
// to 8 steps of 64, kept in registers for the key pass: one load per point), the run keys and
// starts are compacted with workgroup prefixes, wave 0 sorts the (key << 16 | run id) values in
// registers (R <= 512; run ids are in index order, so equal keys keep it: the stable order; above,
// the four waves rank them by counting), and every thread sums about one voxel in index order.  A
// ring holds ~1.5k candidates in ~230 runs of equal keys (C2).  (Round 4 also measured one wave
// per ring: 2.3x fewer VALU instructions than the 512-thread kernel but ~14 dependent round trips
// per ring, slower overall; removed in round 5.)
// Occupancy (round 5): the ring's waves mostly wait on their few dependent memory round trips, so
// more rings per CU pay.  Pass A keeps only x, y, z of its points (80 -> 72 VGPRs: still 6-7 waves
// per SIMD, no change), and KQ = 8 is held to 64 VGPRs (8 waves per SIMD) at the cost of 44 B of
// spills: voxel_ring 1.37 -> 1.22 ms per B = 1024 step, 106.4k -> 109.3k scans/s interleaved
// (profiles/r05af_voxel_ring_occupancy_ab.txt).  KQ = 16 (rings of 2049-4096 points) keeps its own
// allocation (the compiler's choice for this attribute pair: 118 VGPRs, 28 B of spills).  The
// allocation is sensitive to the attribute's spelling: (8) on both instances or (8, 8) here gives
// 64 VGPRs; a separate kernel per KQ or (8, 8) with another maximum for KQ = 16 missed the target
// (69 VGPRs, 7 waves) on this compiler.
template <int KQ>  // steps of 64 points per wave: 4 * 64 * KQ >= the ring capacity
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KQ <= 8 ? 8 : 1, KQ <= 8 ? 8 : 10)))
k_voxel_ring_q(VgRing A) {
  constexpr int NW = 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float mmx[NW][6];
  __shared__ int cntw[NW], runw[NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int slot = blockIdx.x, job = slot / A.H;
  const int s = A.start_ring[slot], e = A.end_ring[slot];
  float4* out = A.out + (int64_t)slot * A.stride_out;
  if (e <= s) {
    if (tid == 0) A.cnt_out[slot] = 0;
    return;
  }
  int sp6[6], ep6[6];
  bool all6 = true;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    sp6[j] = (s * (6 - j) + e * j) / 6;
    ep6[j] = (s * (5 - j) + e * (j + 1)) / 6 - 1;
    all6 = all6 && sp6[j] < ep6[j];
  }
  auto in_seg = [&](int k) {  // the non-empty segments [sp, ep] (:195-200), inside [s, e - 1]
    if (all6) return k <= ep6[5];
    bool in = false;
#pragma unroll
    for (int j = 0; j < 6; ++j) in |= sp6[j] < ep6[j] && k >= sp6[j] && k <= ep6[j];
    return in;
  };
  const float4* CL = A.cloud + (int64_t)job * A.HW + s;
  const int8_t* LB = A.label + (int64_t)job * A.HW + s;
  const int len = min(e - s, (int)A.cap);
  const uint64_t lt = (1ull << lane) - 1ull;
  // ---- pass A: this wave's quarter [q0, q1) in one round of loads, kept in registers ----
  const int qlen = (((len + NW - 1) / NW) + 63) & ~63;
  const int q0 = min(len, w * qlen), q1 = min(len, q0 + qlen);
  // Every label and point load of the wave is issued before any is used: loads of a clamped index
  // (no branch), then an empty asm that takes all the values.  Without it the compiler sank each
  // point load under its label test, a chain of 2 * KQ dependent round trips per wave.
  float4 pt[KQ];
  bool cd[KQ];
  int lb[KQ];
#pragma unroll
  for (int u = 0; u < KQ; ++u) {
    const int ic = min(q0 + 64 * u + lane, len - 1);
    lb[u] = LB[ic];
    pt[u] = CL[ic];
  }
#pragma unroll
  for (int u = 0; u < KQ; ++u) asm volatile("" ::"v"(lb[u]), "v"(pt[u].x), "v"(pt[u].y), "v"(pt[u].z));
#pragma unroll
  for (int u = 0; u < KQ; ++u) cd[u] = q0 + 64 * u + lane < q1 && lb[u] <= 0;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  int nw = 0;
#pragma unroll
  for (int u = 0; u < KQ; ++u) {
    cd[u] = cd[u] && in_seg(s + q0 + 64 * u + lane);
    if (cd[u]) {
      const float v[3] = {pt[u].x, pt[u].y, pt[u].z};
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        mn[d] = (v[d] < mn[d]) ? v[d] : mn[d];
        mx[d] = (mx[d] < v[d]) ? v[d] : mx[d];
      }
    }
    nw += __popcll(__ballot(cd[u]));
  }
#pragma unroll
  for (int d = 0; d < 3; ++d)
    for (int o = 32; o > 0; o >>= 1) {
      const float a = __shfl_xor(mn[d], o), b = __shfl_xor(mx[d], o);
      mn[d] = (a < mn[d]) ? a : mn[d];
      mx[d] = (mx[d] < b) ? b : mx[d];
    }
  if (lane == 0) {
    for (int d = 0; d < 3; ++d) {
      mmx[w][d] = mn[d];
      mmx[w][3 + d] = mx[d];
    }
    cntw[w] = nw;
  }
  __syncthreads();
  int n = 0, base = 0;
#pragma unroll
  for (int ww = 0; ww < NW; ++ww) {
    base += ww < w ? cntw[ww] : 0;
    n += cntw[ww];
  }
  if (n == 0) {
    if (tid == 0) A.cnt_out[slot] = 0;
    return;
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    mn[d] = mmx[0][d];
    mx[d] = mmx[0][3 + d];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) {
      mn[d] = (mmx[ww][d] < mn[d]) ? mmx[ww][d] : mn[d];
      mx[d] = (mx[d] < mmx[ww][3 + d]) ? mmx[ww][3 + d] : mx[d];
    }
  }
  VgGrid G;
  G.init(mn, mx, A.leaf, false);
  const int cap = (int)A.cap;
  uint32_t* kb = (uint32_t*)smem;             // [cap + 1] candidate keys, then run keys; then sid / vst (u16)
  uint16_t* off = (uint16_t*)(kb + cap + 1);  // [cap] ring offset of the t-th candidate
  uint16_t* rst = off + cap;                  // [cap + 1] first candidate of each run
  // ---- pass B: keys in index order (or, on PCL's overflow, the candidates themselves) ----
#pragma unroll
  for (int u = 0; u < KQ; ++u) {
    const uint64_t b = __ballot(cd[u]);
    const int pos = base + __popcll(b & lt);
    if (cd[u]) {
      if (G.overflow) {  // PCL: "Leaf size is too small" -> output = input, in index order
        out[pos] = CL[q0 + 64 * u + lane];  // re-read: only x, y, z stay live from pass A
      } else {
        kb[pos] = G.key(pt[u]);
        off[pos] = (uint16_t)(q0 + 64 * u + lane);
      }
    }
    base += __popcll(b);
  }
  if (G.overflow) {
    if (tid == 0) A.cnt_out[slot] = n;
    return;
  }
  __syncthreads();
  // ---- pass C: run heads (keys read before the barrier, run keys written after it) ----
  const int tq = (((n + NW - 1) / NW) + 63) & ~63;
  const int t0w = min(n, w * tq), t1w = min(n, t0w + tq);
  constexpr int KR = KQ;  // n <= len: each wave's share of candidates fits KR steps as well
  uint32_t rk[KR];
  uint64_t hb[KR];
  int nr = 0;
#pragma unroll
  for (int u = 0; u < KR; ++u) {
    const int t = t0w + 64 * u + lane;
    const bool valid = t < t1w;
    const uint32_t key = valid ? kb[t] : 0u;
    const uint32_t prev = (valid && t > 0) ? kb[t - 1] : 0u;
    rk[u] = key;
    hb[u] = __ballot(valid && (t == 0 || key != prev));
    nr += __popcll(hb[u]);
  }
  if (lane == 0) runw[w] = nr;
  __syncthreads();
  int R = 0, rq = 0;
#pragma unroll
  for (int ww = 0; ww < NW; ++ww) {
    rq += ww < w ? runw[ww] : 0;
    R += runw[ww];
  }
#pragma unroll
  for (int u = 0; u < KR; ++u) {
    if ((hb[u] >> lane) & 1ull) {
      const int r = rq + __popcll(hb[u] & lt);
      kb[r] = rk[u];
      rst[r] = (uint16_t)(t0w + 64 * u + lane);
    }
    rq += __popcll(hb[u]);
  }
  if (tid == 0) rst[R] = (uint16_t)n;
  __syncthreads();
  // ---- sort the runs (stable by run id), voxel starts ----
  uint16_t* sid = (uint16_t*)kb;  // [R]
  uint16_t* vst = sid + cap + 1;  // [V + 1]
  __shared__ int vcount;
  if (R <= 512) {
    if (w == 0) {
      const int V = R <= 256 ? vr_sort_runs<4>(kb, R, sid, vst, lane) : vr_sort_runs<8>(kb, R, sid, vst, lane);
      if (lane == 0) vcount = V;
    }
  } else {
    // rank by counting over all 4 waves into the output slot, then wave 0 marks the voxels
    uint64_t* scr = reinterpret_cast<uint64_t*>(out);
    for (int r = tid; r < R; r += 256) {
      const uint32_t key = kb[r];
      int rank = 0;
      for (int j = 0; j < R; ++j) {
        const uint32_t kj = kb[j];
        rank += (kj < key || (kj == key && j < r)) ? 1 : 0;
      }
      scr[rank] = ((uint64_t)key << 16) | (uint64_t)r;
    }
    __syncthreads();  // (also orders the global scratch writes before the reads below)
    if (w == 0) {
      int V = 0;
      for (int g0 = 0; g0 < R; g0 += 64) {
        const int g = g0 + lane;
        const uint64_t x = g < R ? scr[g] : ~0ull;
        const uint64_t px = (g > 0 && g < R) ? scr[g - 1] : ~0ull;
        const bool hd = g < R && (g == 0 || (x >> 16) != (px >> 16));
        const uint64_t b = __ballot(hd);
        wave_lds_sync();
        if (g < R) sid[g] = (uint16_t)(x & 0xFFFFull);
        if (hd) vst[V + __popcll(b & lt)] = (uint16_t)g;
        V += __popcll(b);
      }
      if (lane == 0) {
        vst[V] = (uint16_t)R;
        vcount = V;
      }
    }
  }
  __syncthreads();  // (the scratch reads above precede the emit's stores to the same slot)
  const int V = vcount;
  // ---- one thread per voxel: the float sum of its points in index order (runs in id order) ----
  for (int vv = tid; vv < V; vv += 256) {
    const int g0 = vst[vv], g1 = vst[vv + 1];
    float4 c = make_float4(0.f, 0.f, 0.f, 0.f);
    int cnt = 0;
    for (int g = g0; g < g1; ++g) {
      const int rid = sid[g];
      const int ta = rst[rid], tb = rst[rid + 1];
      for (int t = ta; t < tb; t += 8) {  // a run's points, 8 gathers in flight
        float4 pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = CL[off[min(t + u, tb - 1)]];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (t + u < tb) {
            if (cnt == 0) {
              c = pp[u];
            } else {
              c.x += pp[u].x;
              c.y += pp[u].y;
              c.z += pp[u].z;
              c.w += pp[u].w;
            }
            ++cnt;
          }
      }
    }
    const float fc = (float)cnt;
    out[vv] = make_float4(c.x / fc, c.y / fc, c.z / fc, c.w / fc);
  }
  if (tid == 0) A.cnt_out[slot] = V;
}

// The per-ring filter of the default order: four waves per ring, except launches of at most 256
// rings (single scans), where the 512-thread kernel finishes a ring sooner (C2 single scan: 19.8 vs
// 34.3 us, profiles/r04u_latency_scan_timeline.txt) and the chip has room for the extra threads.
bool vr_four_waves(int nseg) { return nseg > 256; }

size_t voxel_ring_lds_bytes(const VgRing& a, int threads, int kpt) {
  const int nw = threads / 64;
  size_t b = sizeof(uint32_t) * ((size_t)(nw + 1) * 256 + nw) + sizeof(float) * nw * 6 + sizeof(int) * kpt * nw;
  b = (b + 15) & ~(size_t)15;
  // keys / run ids ping-pong + candidate offsets + run starts
  return b + (size_t)a.cap * 2 * (sizeof(uint32_t) + sizeof(uint16_t)) + (size_t)(2 * a.cap + 1) * sizeof(uint16_t) + 16;
}

void launch_voxel_ring(hipStream_t s, const VgRing& a) {
  const int nseg = a.B * a.H;
  if (nseg <= 0) return;
  // 512 threads, KPT = ceil(W / 512) points per thread (instances up to W = 4096)
  const int kpt = (int)((a.cap + 511) / 512);
  auto go = [&](auto ex) {
    constexpr bool E = decltype(ex)::value;
    if (kpt <= 2)
      fbr_launch((k_voxel_ring<512, 2, E>), dim3(nseg), dim3(512), voxel_ring_lds_bytes(a, 512, 2), s, a);
    else if (kpt <= 4)
      fbr_launch((k_voxel_ring<512, 4, E>), dim3(nseg), dim3(512), voxel_ring_lds_bytes(a, 512, 4), s, a);
    else
      fbr_launch((k_voxel_ring<512, 8, E>), dim3(nseg), dim3(512), voxel_ring_lds_bytes(a, 512, 8), s, a);
  };
  if (a.exact) {
    go(std::true_type{});
  } else if ((a.kernel < 0 ? vr_four_waves(nseg) : a.kernel == 2) && a.dbg == 0 && a.cap <= 4096) {
    const size_t lds = (((size_t)a.cap + 1) * 4 + (size_t)a.cap * 2 + ((size_t)a.cap + 1) * 2 + 15) & ~(size_t)15;
    if (a.cap <= 4 * 64 * 8) fbr_launch(k_voxel_ring_q<8>, dim3(nseg), dim3(256), lds, s, a);
    else fbr_launch(k_voxel_ring_q<16>, dim3(nseg), dim3(256), lds, s, a);
  } else {
    go(std::false_type{});
  }
}

// In-place LDS sort of the mapping-DS segments (FBR_VG_INPLACE=0: the global-scratch kernel).
bool vg_inplace() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_VG_INPLACE");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

size_t voxel_lds_bytes(const VgArgs& a, int threads, bool lds_mode) {
  const int nw = threads / 64;
  size_t b = sizeof(uint32_t) * ((size_t)(nw + 1) * 512 + nw) + sizeof(float) * nw * 6 + sizeof(int) * 4;
  b = (b + 15) & ~(size_t)15;
  if (lds_mode) {
    int64_t cap = 0;
    for (int k = 0; k < 2; ++k)
      if (a.s[k].nseg > 0) cap = std::max<int64_t>(cap, a.s[k].cap);
    b += (size_t)cap * 2 * (sizeof(uint32_t) + sizeof(uint16_t)) + 16;
  }
  return b;
}

constexpr int kVgIpKpl = 18;  // k_voxel_grid_ip: segments up to 1024 * 18 points sort in LDS
constexpr int kVgSplitSlots = 16;   // k_voxel_grid_split: segments x parts per launch
constexpr int kVgSplitRing = 1024;  // flag regions: a launch's own region (concurrent launches)
constexpr int kVgSplitMaxDevices = 64;
int vg_split() {
  static const int v = [] {
    const char* e = std::getenv("FBR_VG_SPLIT");
    const int p = e ? std::atoi(e) : 8;
    return p < 2 ? 1 : std::min(p, 8);
  }();
  return v;
}

void launch_voxel_grid(hipStream_t s, const VgArgs& a) {
  const int nseg = a.s[0].nseg + a.s[1].nseg;
  if (nseg <= 0) return;
  int64_t cap = 0;
  for (int k = 0; k < 2; ++k)
    if (a.s[k].nseg > 0) cap = std::max<int64_t>(cap, a.s[k].cap);
  const bool exact = a.s[0].exact || a.s[1].exact;  // both sets share the context's mode
  // few segments (single-scan calls): P workgroups per segment (FBR_VG_SPLIT = P, default 8: C2 latency
  // -10 us against 4, profiles/r05w_latency_knob_sweep.txt; 1 off)
  const int P = vg_split();
  if (!exact && P > 1 && cap > kVgLdsCap && vg_inplace() && nseg * P <= kVgSplitSlots) {
    // look-back flags of the current device (agent-scope atomics must stay on the device that runs
    // the kernel: contexts on several GPUs in one process each get their own)
    static std::mutex mu;
    static unsigned long long* dev_flags[kVgSplitMaxDevices] = {};
    static bool dev_failed[kVgSplitMaxDevices] = {};
    int dev = -1;
    unsigned long long* flags = nullptr;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kVgSplitMaxDevices) {
      std::lock_guard<std::mutex> lk(mu);
      if (!dev_flags[dev] && !dev_failed[dev]) {
        unsigned long long* f = nullptr;
        const size_t bytes = sizeof(unsigned long long) * kVgSplitSlots * kVgSplitRing;
        if (hipMalloc(&f, bytes) == hipSuccess && hipMemset(f, 0, bytes) == hipSuccess) dev_flags[dev] = f;
        else dev_failed[dev] = true;  // the one-workgroup kernel below serves this device
      }
      flags = dev_flags[dev];
    }
    static std::atomic<unsigned> gen{0};
    if (flags) {
      const unsigned g = gen.fetch_add(1) + 1;  // never 0 (the zeroed flags)
      const size_t lds = voxel_lds_bytes(a, 1024, false) + (size_t)1024 * kVgIpKpl * (sizeof(uint32_t) + sizeof(uint16_t));
      fbr_launch((k_voxel_grid_split<1024, kVgIpKpl>), dim3(nseg * P), dim3(1024), lds, s, a, P,
                 flags + (size_t)(g % kVgSplitRing) * kVgSplitSlots, g);
      return;
    }
  }
  auto go = [&](auto ex) {
    constexpr bool E = decltype(ex)::value;
    if (cap <= kVgLdsCap) {
      fbr_launch((k_voxel_grid<256, uint16_t, true, E>), dim3(nseg), dim3(256), voxel_lds_bytes(a, 256, true), s, a);
    } else if (vg_inplace()) {
      const size_t lds =
          voxel_lds_bytes(a, 1024, false) + (size_t)1024 * kVgIpKpl * (sizeof(uint32_t) + sizeof(uint16_t));
      fbr_launch((k_voxel_grid_ip<1024, kVgIpKpl, E>), dim3(nseg), dim3(1024), lds, s, a);
    } else {
      fbr_launch((k_voxel_grid<1024, uint32_t, false, E>), dim3(nseg), dim3(1024), voxel_lds_bytes(a, 1024, false),
                 s, a);
    }
  };
  if (exact) go(std::true_type{});
  else go(std::false_type{});
}

// Ring-ordered concatenation of the per-ring corner picks and per-ring surf DS outputs
// (cornerCloud / surfaceCloud of featureExtraction.h).  One wave per (job, ring), 4 rings per
// workgroup: the wave sums the counts of the rings before its own (lanes over rings, a shuffle
// reduction) and copies its ring's corner picks and surf DS points to their offsets; the last
// ring's wave writes the job totals.
__global__ void __launch_bounds__(256)
k_concat(int H, int W, const float4* corner_slot, const int32_t* corner_cnt, const float4* surf_ring,
         const int32_t* surf_ring_cnt, float4* corner_all, int64_t capc, int32_t* n_corner, float4* surf_all,
         int64_t caps, int32_t* n_surf, float* ring_box) {
  const int lane = threadIdx.x & 63, rpj = (H + 3) / 4;
  const int job = blockIdx.x / rpj, r = (blockIdx.x % rpj) * 4 + (threadIdx.x >> 6);
  if (r >= H) return;
  const int32_t* cc = corner_cnt + job * H;
  const int32_t* sc = surf_ring_cnt + job * H;
  int oc = 0, os = 0;
  for (int k = lane; k < r; k += 64) {
    oc += cc[k];
    os += sc[k];
  }
  for (int o = 32; o > 0; o >>= 1) {
    oc += __shfl_xor(oc, o);
    os += __shfl_xor(os, o);
  }
  const int nc = cc[r], ns = sc[r];
  if (r == H - 1 && lane == 0) {
    n_corner[job] = oc + nc;
    n_surf[job] = os + ns;
  }
  const float4* cs = corner_slot + ((int64_t)job * H + r) * kCornerPerRing;
  const float4* ss = surf_ring + ((int64_t)job * H + r) * W;
  float bx[2][6];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      bx[c][d] = FLT_MAX;
      bx[c][3 + d] = -FLT_MAX;
    }
  auto grow = [&](float (&b)[6], const float4& p) {
    const float v[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      b[d] = (v[d] < b[d]) ? v[d] : b[d];
      b[3 + d] = (b[3 + d] < v[d]) ? v[d] : b[3 + d];
    }
  };
  for (int i = lane; i < nc; i += 64) {
    const float4 p = cs[i];
    corner_all[job * capc + oc + i] = p;
    grow(bx[0], p);
  }
  for (int i = lane; i < ns; i += 64) {
    const float4 p = ss[i];
    surf_all[job * caps + os + i] = p;
    grow(bx[1], p);
  }
  if (!ring_box) return;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int d = 0; d < 3; ++d)
      for (int o = 32; o > 0; o >>= 1) {
        const float a = __shfl_xor(bx[c][d], o), b = __shfl_xor(bx[c][3 + d], o);
        bx[c][d] = (a < bx[c][d]) ? a : bx[c][d];
        bx[c][3 + d] = (bx[c][3 + d] < b) ? b : bx[c][3 + d];
      }
  if (lane < kRingBox) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kRingBox; ++k)
      if (lane == k) v = bx[k / 6][k % 6];
    ring_box[((int64_t)job * H + r) * kRingBox + lane] = v;
  }
}

void launch_concat(hipStream_t s, int B, int H, int W, const float4* corner_slot, const int32_t* corner_cnt,
                   const float4* surf_ring, const int32_t* surf_ring_cnt, float4* corner_all, int64_t capc,
                   int32_t* n_corner, float4* surf_all, int64_t caps, int32_t* n_surf, float* ring_box) {
  if (B <= 0 || H <= 0) return;
  fbr_launch(k_concat, dim3(B * ((H + 3) / 4)), dim3(256), 0, s, H, W, corner_slot, corner_cnt, surf_ring,
                     surf_ring_cnt, corner_all, capc, n_corner, surf_all, caps, n_surf, ring_box);
}


// ---- radix sort selftests (fbr_selftest_radix_sort): one workgroup sorts one array with the
// product's configurations of the wave-chunk sorts ----
// variant 0: vg_radix_sort<512, u16, 8, LDS> (per-ring filter), 1: vg_radix_sort<256, u16, 9, LDS>
// (per-segment LDS kernel), 2: vg_radix_sort<1024, u32, 9, global> (global-scratch kernel),
// 3: vg_radix_sort_inplace<1024, 18> (mapping DS), 4: the same with ballot-leader digit counts,
// 5: round 3's rejected form (ballot-leader counts + wave-uniform early exits).
template <int T, typename V, int MAXD, bool KV_LDS>
__global__ void __launch_bounds__(T) k_selftest_radix(uint32_t* keys, uint32_t* vals, uint32_t* scratch, int n, int nbits) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = T / 64;
  uint32_t* hist = (uint32_t*)smem;
  uint32_t* wsum = hist + (NW + 1) * 512;
  unsigned char* q = (unsigned char*)(wsum + NW);
  q = smem + (((q - smem) + 15) & ~15);
  uint32_t* kb[2];
  V* vb[2];
  if constexpr (KV_LDS) {
    kb[0] = (uint32_t*)q;
    kb[1] = kb[0] + n;
    vb[0] = (V*)(kb[1] + n);
    vb[1] = vb[0] + n;
  } else {
    kb[0] = scratch;
    kb[1] = scratch + n;
    vb[0] = (V*)(scratch + 2 * n);
    vb[1] = (V*)(scratch + 3 * n);
  }
  for (int i = threadIdx.x; i < n; i += T) {
    kb[0][i] = keys[i];
    vb[0][i] = (V)i;
  }
  __syncthreads();
  const int cur = vg_radix_sort<T, V, MAXD, KV_LDS>(kb, vb, n, nbits, hist, wsum);
  for (int i = threadIdx.x; i < n; i += T) {
    keys[i] = kb[cur][i];
    vals[i] = (uint32_t)vb[cur][i];
  }
}

template <int kLeader>
__global__ void __launch_bounds__(1024) k_selftest_radix_ip(uint32_t* keys, uint32_t* vals, int n, int nbits) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int NW = 16, LCAP = 1024 * kVgIpKpl;
  uint32_t* hist = (uint32_t*)smem;
  uint32_t* wsum = hist + (NW + 1) * 512;
  unsigned char* q = (unsigned char*)(wsum + NW);
  q = smem + (((q - smem) + 15) & ~15);
  FBR_LDS_AS uint32_t* k = (FBR_LDS_AS uint32_t*)q;
  FBR_LDS_AS uint16_t* v = (FBR_LDS_AS uint16_t*)((FBR_LDS_AS uint32_t*)q + LCAP);
  for (int i = threadIdx.x; i < n; i += 1024) {
    k[i] = keys[i];
    v[i] = (uint16_t)i;
  }
  __syncthreads();
  vg_radix_sort_inplace<1024, kVgIpKpl, kLeader>(k, v, n, nbits, hist, wsum);
  for (int i = threadIdx.x; i < n; i += 1024) {
    keys[i] = k[i];
    vals[i] = v[i];
  }
}

}  // namespace fbr

// Diagnostic entry point (tests/test_gpu_parity.py): sort n keys (low nbits significant) with one of
// the product's radix sort configurations; keys_inout gets the sorted keys, perm the source index of
// each sorted position.
extern "C" int fbr_selftest_radix_sort(int64_t n, int nbits, int variant, uint32_t* keys_inout, uint32_t* perm) {
  using namespace fbr;
  const int64_t lcap[6] = {4096, 4096, 1 << 20, 1024 * kVgIpKpl, 1024 * kVgIpKpl, 1024 * kVgIpKpl};
  if (n < 0 || variant < 0 || variant > 5 || n > lcap[variant] || nbits < 1 || nbits > 32 || (n && (!keys_inout || !perm)))
    return FBR_ERR_INVALID_ARG;
  if (n == 0) return FBR_OK;
  uint32_t *dk = nullptr, *dv = nullptr, *ds = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&dk, 4 * n) != hipSuccess || hipMalloc(&dv, 4 * n) != hipSuccess || hipMalloc(&ds, 16 * n) != hipSuccess ||
      hipMemcpy(dk, keys_inout, 4 * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    const int nn = (int)n;
    auto hdr = [](int T) { return (((size_t)(T / 64 + 1) * 512 + T / 64) * 4 + 15) & ~(size_t)15; };
    switch (variant) {
      case 0:
        hipLaunchKernelGGL((k_selftest_radix<512, uint16_t, 8, true>), dim3(1), dim3(512), hdr(512) + (size_t)n * 12, 0,
                           dk, dv, ds, nn, nbits);
        break;
      case 1:
        hipLaunchKernelGGL((k_selftest_radix<256, uint16_t, 9, true>), dim3(1), dim3(256), hdr(256) + (size_t)n * 12, 0,
                           dk, dv, ds, nn, nbits);
        break;
      case 2:
        hipLaunchKernelGGL((k_selftest_radix<1024, uint32_t, 9, false>), dim3(1), dim3(1024), hdr(1024), 0, dk, dv, ds,
                           nn, nbits);
        break;
      default: {
        const size_t lds = hdr(1024) + (size_t)1024 * kVgIpKpl * 6;
        if (variant == 3) hipLaunchKernelGGL(k_selftest_radix_ip<0>, dim3(1), dim3(1024), lds, 0, dk, dv, nn, nbits);
        else if (variant == 4) hipLaunchKernelGGL(k_selftest_radix_ip<1>, dim3(1), dim3(1024), lds, 0, dk, dv, nn, nbits);
        else hipLaunchKernelGGL(k_selftest_radix_ip<2>, dim3(1), dim3(1024), lds, 0, dk, dv, nn, nbits);
      }
    }
    if (hipGetLastError() != hipSuccess || hipMemcpy(keys_inout, dk, 4 * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(perm, dv, 4 * n, hipMemcpyDeviceToHost) != hipSuccess)
      rc = FBR_ERR_HIP;
  }
  for (void* q : {(void*)dk, (void*)dv, (void*)ds}) (void)hipFree(q);
  return rc;
}

namespace fbr {

// ---------------------------------------------------------------------------------------------
// Device-wide VoxelGrid of one large cloud (the start-up map filter, the keyframe local map,
// fbr_voxel_grid): the per-segment kernel above gives a whole workgroup to a segment, which leaves
// the chip idle for a single cloud of 10^5-10^7 points.  Same semantics (PCL box, overflow
// fallback, key, float centroids in ascending key order); the (key, index) sort is rocprim's
// stable LSD radix sort, so points inside a voxel are summed in index order exactly as in the
// segmented kernel.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t f2ord(float f) {  // order-preserving float -> uint
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u); }

__global__ void __launch_bounds__(256) k_vgl_minmax(const float4* __restrict__ in, int64_t n, uint32_t* mm) {
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float4 p = in[i];
    const float v[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int d = 0; d < 3; ++d) {  // getMinMax3D's comparisons (NaN never replaces)
      mn[d] = (v[d] < mn[d]) ? v[d] : mn[d];
      mx[d] = (mx[d] < v[d]) ? v[d] : mx[d];
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    for (int o = 32; o > 0; o >>= 1) {
      const float a = __shfl_xor(mn[d], o), b = __shfl_xor(mx[d], o);
      mn[d] = (a < mn[d]) ? a : mn[d];
      mx[d] = (mx[d] < b) ? b : mx[d];
    }
    if ((threadIdx.x & 63) == 0) {
      atomicMin(&mm[d], f2ord(mn[d]));
      atomicMax(&mm[3 + d], f2ord(mx[d]));
    }
  }
}

struct VglState {
  VgGrid G;
  int32_t nvox;
};

__global__ void k_vgl_grid(const uint32_t* mm, float leaf, int morton, VglState* st) {
  float mn[3], mx[3];
  for (int d = 0; d < 3; ++d) {
    mn[d] = ord2f(mm[d]);
    mx[d] = ord2f(mm[3 + d]);
  }
  st->G.init(mn, mx, leaf, morton != 0);
}

__global__ void __launch_bounds__(256)
k_vgl_keys(const float4* __restrict__ in, int64_t n, const VglState* __restrict__ st, int exact, uint32_t* keys,
           uint32_t* vals) {
  const VgGrid G = st->G;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    keys[i] = G.overflow ? 0u : (exact ? G.pcl_key(in[i]) : G.key(in[i]));
    vals[i] = (uint32_t)i;
  }
}

// std::sort's partition phase over the whole cloud (fbr_introsort.h) by one workgroup: PCL's
// order inside the voxels for the stable device-wide radix sort that follows.  n / 17 + 2 frames
// per list in fa / fb.
__global__ void __launch_bounds__(1024)
k_vgl_isort(uint32_t* keys, uint32_t* vals, int32_t* posL, int32_t* posR, int* fa, int* fb, int n) {
  __shared__ int sh[64];
  is_partition_phase<1024>(keys, vals, posL, posR, n, fa, fb, sh);
}

__global__ void __launch_bounds__(256) k_vgl_outkeys(uint32_t* keys, int64_t n, const VglState* __restrict__ st) {
  const VgGrid G = st->G;
  if (!G.morton || G.overflow) return;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    keys[i] = G.out_key(keys[i]);
}

__global__ void __launch_bounds__(256) k_vgl_heads(const uint32_t* __restrict__ keys, int64_t n, uint32_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void __launch_bounds__(256)
k_vgl_emit(const float4* __restrict__ in, int64_t n, const VglState* __restrict__ st, const uint32_t* __restrict__ keys,
           const uint32_t* __restrict__ vals, const uint32_t* __restrict__ vox, float4* __restrict__ out,
           int32_t* __restrict__ nout) {
  const bool overflow = st->G.overflow;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    if (overflow) {  // PCL: "Leaf size is too small" -> output = input
      out[i] = in[i];
      if (i == 0) *nout = (int32_t)n;
      continue;
    }
    if (!(i == 0 || keys[i] != keys[i - 1])) continue;
    const uint32_t key = keys[i];
    float4 c = in[vals[i]];
    int64_t j = i + 1;
    while (j < n && keys[j] == key) {
      const float4 p = in[vals[j]];
      c.x += p.x;
      c.y += p.y;
      c.z += p.z;
      c.w += p.w;
      ++j;
    }
    const float cnt = (float)(j - i);
    out[vox[i]] = make_float4(c.x / cnt, c.y / cnt, c.z / cnt, c.w / cnt);
    if (j == n) *nout = (int32_t)vox[i] + 1;
  }
}

int voxel_grid_large(hipStream_t s, DevArena& ar, const float4* in, int64_t n, float leaf, int morton, int exact,
                     float4* out, int32_t* d_nout) {
  if (n <= 0) return hipMemsetAsync(d_nout, 0, sizeof(int32_t), s) == hipSuccess ? FBR_OK : FBR_ERR_HIP;
  if (n > (int64_t)INT32_MAX) return FBR_ERR_CAPACITY;
  const size_t N = (size_t)n;
  size_t tb_sort = 0, tb_scan = 0;
  uint32_t* null32 = nullptr;
  if (rocprim::radix_sort_pairs(nullptr, tb_sort, null32, null32, null32, null32, N, 0, 32, s) != hipSuccess ||
      rocprim::exclusive_scan(nullptr, tb_scan, null32, null32, 0u, N, rocprim::plus<uint32_t>(), s) != hipSuccess)
    return FBR_ERR_HIP;
  const size_t tb = std::max<size_t>(std::max(tb_sort, tb_scan), 16);
  if (arena_reserve(ar, arena_bytes(6 * sizeof(uint32_t)) + arena_bytes(sizeof(VglState)) + 6 * arena_bytes(4 * N) +
                            arena_bytes(tb), s) != hipSuccess)
    return FBR_ERR_HIP;
  uint32_t* mm = arena_take<uint32_t>(ar, 6 * sizeof(uint32_t));
  VglState* st = arena_take<VglState>(ar, sizeof(VglState));
  uint32_t* k0 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* k1 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* v0 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* v1 = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* head = arena_take<uint32_t>(ar, 4 * N);
  uint32_t* vox = arena_take<uint32_t>(ar, 4 * N);
  void* tmp = arena_take<void>(ar, tb);
  if (!mm || !st || !k0 || !k1 || !v0 || !v1 || !head || !vox || !tmp) return FBR_ERR_HIP;  // arena sizing slip
  int rc = FBR_OK;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess) rc = FBR_ERR_HIP;
    return rc == FBR_OK;
  };
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
  // min / max accumulators: ordered-uint encodings of +inf-like (all ones) and -inf-like (0)
  if (ok(hipMemsetD32Async((hipDeviceptr_t)mm, 0xFFFFFFFFu, 3, s)) && ok(hipMemsetD32Async((hipDeviceptr_t)(mm + 3), 0u, 3, s))) {
    fbr_launch(k_vgl_minmax, dim3(grid), dim3(256), 0, s, in, n, mm);
    fbr_launch(k_vgl_grid, dim3(1), dim3(1), 0, s, mm, leaf, morton, st);
    fbr_launch(k_vgl_keys, dim3(grid), dim3(256), 0, s, in, n, st, exact, k0, v0);
    if (exact) {  // scratch: head / vox (positions) and k1 / v1 (frame lists), all free until the sort
      fbr_launch(k_vgl_isort, dim3(1), dim3(1024), 0, s, k0, v0, (int32_t*)head, (int32_t*)vox, (int*)k1, (int*)v1,
                 (int)n);
      fbr_launch(k_vgl_outkeys, dim3(grid), dim3(256), 0, s, k0, n, st);
    }
    if (ok(rocprim::radix_sort_pairs(tmp, tb_sort, k0, k1, v0, v1, N, 0, 32, s))) {
      fbr_launch(k_vgl_heads, dim3(grid), dim3(256), 0, s, k1, n, head);
      // head flags -> voxel index (out of place)
      if (ok(rocprim::exclusive_scan(tmp, tb_scan, head, vox, 0u, N, rocprim::plus<uint32_t>(), s)))
        fbr_launch(k_vgl_emit, dim3(grid), dim3(256), 0, s, in, n, st, k1, v1, vox, out, d_nout);
    }
  }
  return rc;
}

}  // namespace fbr

#ifdef FBR_VG_STAMPS
extern "C" int fbr_diag_vg_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(fbr::fbr_vg_stamps), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -1;
}
#endif
