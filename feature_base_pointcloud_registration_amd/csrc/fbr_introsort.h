// fbr_introsort.h — the point order inside a voxel of pcl::VoxelGrid, on the device.
//
// PCL's applyFilter (voxel_grid.cpp) sorts the index vector {idx, cloud_point_index} with
// std::sort, comparing idx only, and sums each voxel's points in the resulting order
// (featureExtraction.h:288-292, mapOptmization.h:251-257, 981-993).  std::sort is unstable, so
// that order -- and with it the last bits of every centroid -- is libstdc++'s introsort's.
//
// libstdc++ (stl_algo.h; unchanged since GCC 4.8, the reference's toolchains included):
//   __introsort_loop(first, last, depth = 2 * floor(log2 n)):
//     while (last - first > 16) {
//       if (depth == 0) { partial_sort(first, last, last); return; }        // heap sort
//       --depth;
//       __move_median_to_first(first, first + 1, mid, last - 1);
//       cut = __unguarded_partition(first + 1, last, first);
//       __introsort_loop(cut, last, depth); last = cut;
//     }
//   __final_insertion_sort(first, last): an insertion sort, i.e. STABLE on its input.
// So std::sort's result is the stable sort (by key) of the array the partition phase leaves, and
// that phase is what this header reproduces:
//   * frames (sub-ranges) of one recursion level are disjoint, so they are processed level by
//     level, in parallel (the order of disjoint frames does not change the array);
//   * __unguarded_partition(lo, hi, pivot p) in closed form: the k-th element from the left that
//     is not < p (a "left stopper" g_k) is swapped with the k-th element from the right that is
//     not > p (r_k) for as long as g_k < r_k; with K such swaps the cut is min(g_K, r_{K-1}) (the
//     swapped elements stop the scans).  g_k / r_k are ballot-ranked (one wave per small frame) or
//     block-scan-ranked (the whole workgroup on frames larger than kIsBig);
//   * median-of-3 and the depth-exhausted heap sort run on one lane, as serial code.
// A stable radix sort of the result by key (the kernels' existing sorts) then gives std::sort's
// order exactly; tests/test_voxel_order.py checks it against the host std::sort (oracle), and the
// VoxelGrid tests compare the centroids bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace fbr {

#define FBR_IS_LDS __attribute__((address_space(3)))

struct IsFrame {
  int first, last, depth;
};

__host__ __device__ inline int is_lg(int n) {
  int r = -1;
  while (n) {
    n >>= 1;
    ++r;
  }
  return r;
}

// Visibility of this wave's LDS / global writes to its other lanes (and to later workgroup
// barriers): workgroup-scope release / acquire around a wave barrier.
__device__ __forceinline__ void is_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <typename KP, typename VP>
__device__ __forceinline__ void is_swap(KP k, VP v, int a, int b) {
  const auto ka = k[a];
  k[a] = k[b];
  k[b] = ka;
  const auto va = v[a];
  v[a] = v[b];
  v[b] = va;
}

// __move_median_to_first(result, a, b, c) (one lane)
template <typename KP, typename VP>
__device__ void is_median_to_first(KP k, VP v, int result, int a, int b, int c) {
  if (k[a] < k[b]) {
    if (k[b] < k[c]) is_swap(k, v, result, b);
    else if (k[a] < k[c]) is_swap(k, v, result, c);
    else is_swap(k, v, result, a);
  } else if (k[a] < k[c]) {
    is_swap(k, v, result, a);
  } else if (k[b] < k[c]) {
    is_swap(k, v, result, c);
  } else {
    is_swap(k, v, result, b);
  }
}

// std::partial_sort(first, last, last) = __make_heap + __sort_heap (stl_heap.h), one lane.
template <typename KP, typename VP>
__device__ void is_adjust_heap(KP k, VP v, int first, int hole, int len, uint32_t vk, uint32_t vv) {
  const int top = hole;
  int second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (k[first + second] < k[first + second - 1]) second--;
    k[first + hole] = k[first + second];
    v[first + hole] = v[first + second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    k[first + hole] = k[first + second - 1];
    v[first + hole] = v[first + second - 1];
    hole = second - 1;
  }
  int parent = (hole - 1) / 2;  // __push_heap
  while (hole > top && k[first + parent] < vk) {
    k[first + hole] = k[first + parent];
    v[first + hole] = v[first + parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  k[first + hole] = vk;
  v[first + hole] = vv;
}

template <typename KP, typename VP>
__device__ void is_heap_sort(KP k, VP v, int first, int last) {
  const int len = last - first;
  if (len >= 2) {
    int parent = (len - 2) / 2;
    while (true) {
      is_adjust_heap(k, v, first, parent, len, (uint32_t)k[first + parent], (uint32_t)v[first + parent]);
      if (parent == 0) break;
      parent--;
    }
  }
  while (last - first > 1) {
    --last;
    const uint32_t vk = k[last], vv = v[last];  // __pop_heap(first, last, last)
    k[last] = k[first];
    v[last] = v[first];
    is_adjust_heap(k, v, first, 0, last - first, vk, vv);
  }
}

// The same partial_sort on a range of at most 64 elements held in one wave's registers (lane a + j
// holds element j, key / val), by the whole wave in lockstep: every index of the heap walk is
// wave-uniform, so an element is read with v_readlane (an SGPR) and written by the one lane that
// holds it -- the identical sequence of comparisons and moves as is_heap_sort's single lane over
// LDS, without an LDS round trip per step (round 6: depth-exhausted frames were ~40k cycles each).
__device__ __forceinline__ void is_reg_heap_sort(uint32_t& key, uint32_t& val, int a, int len, int lane) {
  auto K = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)key, a + i); };
  auto V = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)val, a + i); };
  auto set = [&](int i, uint32_t kk, uint32_t vv) {
    if (lane == a + i) {
      key = kk;
      val = vv;
    }
  };
  auto adjust = [&](int hole, int n, uint32_t vk, uint32_t vv) {
    const int top = hole;
    int second = hole;
    while (second < (n - 1) / 2) {
      second = 2 * (second + 1);
      if (K(second) < K(second - 1)) second--;
      set(hole, K(second), V(second));
      hole = second;
    }
    if ((n & 1) == 0 && second == (n - 2) / 2) {
      second = 2 * (second + 1);
      set(hole, K(second - 1), V(second - 1));
      hole = second - 1;
    }
    int parent = (hole - 1) / 2;  // __push_heap
    while (hole > top && K(parent) < vk) {
      set(hole, K(parent), V(parent));
      hole = parent;
      parent = (hole - 1) / 2;
    }
    set(hole, vk, vv);
  };
  if (len >= 2) {
    int parent = (len - 2) / 2;
    while (true) {
      adjust(parent, len, K(parent), V(parent));
      if (parent == 0) break;
      parent--;
    }
  }
  int last = len;
  while (last > 1) {
    --last;
    const uint32_t vk = K(last), vv = V(last);  // __pop_heap(first, last, last)
    set(last, K(0), V(0));
    adjust(0, last, vk, vv);
  }
}

// __unguarded_partition(lo, hi, pivot value p) by one wave; posL / posR: scratch indexed [lo, hi).
// Returns the cut.  Ends with a wave sync.
template <typename KP, typename VP, typename PP>
__device__ int is_wave_partition(KP k, VP v, PP posL, PP posR, int lo, int hi, uint32_t p, int lane) {
  const uint64_t below = (1ull << lane) - 1ull;
  // the left and right stopper scans in one loop (independent: their LDS reads overlap)
  int cL = 0, cR = 0;
  for (int o = 0; o < hi - lo; o += 64) {
    const int i = lo + o + lane, t = hi - 1 - o - lane;
    const bool isL = i < hi && !(k[i] < p);
    const bool isR = t >= lo && !(p < k[t]);
    const uint64_t bl = __ballot(isL), br = __ballot(isR);
    if (isL) posL[lo + cL + __popcll(bl & below)] = i;
    if (isR) posR[lo + cR + __popcll(br & below)] = t;
    cL += __popcll(bl);
    cR += __popcll(br);
  }
  is_wave_sync();
  const int mn = min(cL, cR);
  int K = 0;  // swaps: the k with g_k < r_k form a prefix (g increases, r decreases)
  for (int k0 = 0; k0 < mn; k0 += 64) {
    const int kk = k0 + lane;
    const uint64_t bo = __ballot(kk < mn && (int)posL[lo + kk] < (int)posR[lo + kk]);
    K += __popcll(bo);
    if (bo != ~0ull) break;
  }
  for (int kk = lane; kk < K; kk += 64) is_swap(k, v, (int)posL[lo + kk], (int)posR[lo + kk]);
  int cut = K < cL ? (int)posL[lo + K] : INT_MAX;
  if (K > 0) cut = min(cut, (int)posR[lo + K - 1]);
  is_wave_sync();
  return min(cut, hi);
}

// The same by the whole workgroup (T threads) on a large frame; sh: LDS ints, >= 2 * T / 64 + 4.
// Returns the cut to every thread.  Starts and ends with a barrier.
template <int T, typename KP, typename VP, typename PP>
__device__ int is_block_partition(KP k, VP v, PP posL, PP posR, int lo, int hi, uint32_t p, int* sh) {
  constexpr int NW = T / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m = hi - lo, per = (m + T - 1) / T;
  const int b0 = lo + min(m, tid * per), b1 = lo + min(m, (tid + 1) * per);
  int nl = 0, nr = 0;
  for (int i = b0; i < b1; ++i) {
    const uint32_t x = k[i];
    nl += !(x < p);
    nr += !(p < x);
  }
  // exclusive prefix of (nl, nr) over the threads in order
  int il = nl, ir = nr;
  for (int o = 1; o < 64; o <<= 1) {
    const int a = __shfl_up(il, o), b = __shfl_up(ir, o);
    if (lane >= o) {
      il += a;
      ir += b;
    }
  }
  __syncthreads();
  if (lane == 63) {
    sh[w] = il;
    sh[NW + w] = ir;
  }
  __syncthreads();
  int bl = 0, br = 0, cL = 0, cR = 0;
  for (int ww = 0; ww < NW; ++ww) {
    bl += ww < w ? sh[ww] : 0;
    br += ww < w ? sh[NW + ww] : 0;
    cL += sh[ww];
    cR += sh[NW + ww];
  }
  int ol = bl + il - nl, orr = br + ir - nr;  // this thread's first left / right stopper ranks
  for (int i = b0; i < b1; ++i) {
    const uint32_t x = k[i];
    if (!(x < p)) posL[lo + ol++] = i;
    if (!(p < x)) posR[lo + (cR - 1 - orr++)] = i;  // rank from the right
  }
  if (tid == 0) sh[2 * NW] = 0;
  __syncthreads();
  // K = #{k < min(cL, cR): g_k < r_k} (a prefix: g increases, r decreases), counted by every
  // thread over a stride of k and summed (round 6; one lane's binary search was ~11 dependent LDS
  // reads on the critical path of every large frame)
  {
    const int mn = min(cL, cR);
    int cnt = 0;
    for (int k0 = 0; k0 < mn; k0 += T) {
      const int kk = k0 + tid;
      cnt += __popcll(__ballot(kk < mn && (int)posL[lo + kk] < (int)posR[lo + kk]));
    }
    if (lane == 0 && cnt) atomicAdd(&sh[2 * NW], cnt);
  }
  __syncthreads();
  const int K = sh[2 * NW];
  int cut = K < cL ? (int)posL[lo + K] : INT_MAX;
  if (K > 0) cut = min(cut, (int)posR[lo + K - 1]);
  cut = min(cut, hi);
  for (int kk = tid; kk < K; kk += T) is_swap(k, v, (int)posL[lo + kk], (int)posR[lo + kk]);
  __syncthreads();
  return cut;
}

// A frame of at most 64 elements and its whole subtree of the introsort recursion, by one wave
// with the elements in registers (lane j holds element first + j): median-of-3 and the partition's
// swaps are lane exchanges, the stoppers' ranks ballots; the k-th left / right stopper positions
// go through the frame's own slots of posL / posR (rank -> lane).  The sub-frames are kept on a
// wave-uniform stack (children of one frame are disjoint, so their order is immaterial).  A
// depth-exhausted sub-frame is written back and heap-sorted by lane 0 (rare).  Ends with a wave
// sync after the write-back.
template <typename KP, typename VP, typename PP>
__device__ void is_wave_small(KP k, VP v, PP posL, PP posR, int first, int last, int depth, int lane) {
  const int m = last - first;
  uint32_t key = lane < m ? (uint32_t)k[first + lane] : 0xFFFFFFFFu;
  uint32_t val = lane < m ? (uint32_t)v[first + lane] : 0u;
  // the stack of pending sub-frames lives in the lanes' registers (slot j in lane j), so the
  // dynamically indexed entries are lane exchanges instead of scratch memory
  int st_a = 0, st_b = m, st_d = depth;
  int sp = 1;
  const uint64_t below = (1ull << lane) - 1ull, above = lane == 63 ? 0ull : ~0ull << (lane + 1);
  while (sp > 0) {
    --sp;
    const int a = __shfl(st_a, sp), b = __shfl(st_b, sp);
    int d = __shfl(st_d, sp);
    if (b - a <= 16) continue;
    if (d == 0) {  // partial_sort(a, b, b) on the registers
      is_reg_heap_sort(key, val, a, b - a, lane);
      continue;
    }
    --d;
    // __move_median_to_first(a, a + 1, mid, b - 1): exchange lane a with the median's lane
    const int mid = a + (b - a) / 2;
    const uint32_t x = __shfl(key, a + 1), y = __shfl(key, mid), z = __shfl(key, b - 1);
    int c;
    if (x < y) c = (y < z) ? mid : ((x < z) ? b - 1 : a + 1);
    else c = (x < z) ? a + 1 : ((y < z) ? b - 1 : mid);
    {
      const int src = lane == a ? c : (lane == c ? a : lane);
      key = __shfl(key, src);
      val = __shfl(val, src);
    }
    const uint32_t p = __shfl(key, a);
    // __unguarded_partition(a + 1, b, pivot p) in closed form
    const bool in = lane > a && lane < b;
    const bool isL = in && !(key < p), isR = in && !(p < key);
    const uint64_t bl = __ballot(isL), br = __ballot(isR);
    const int cL = __popcll(bl), cR = __popcll(br);
    const int rL = __popcll(bl & below), rR = __popcll(br & above);  // rank from the left / right
    if (isL) posL[first + rL] = lane;  // g_k
    if (isR) posR[first + rR] = lane;  // r_k
    is_wave_sync();
    const int mn = min(cL, cR);
    const int rk = isL && rL < mn ? (int)posR[first + rL] : -1;  // r_k of this left stopper
    const int K = __popcll(__ballot(isL && rL < mn && lane < rk));
    int partner = lane;
    if (isL && rL < K) partner = rk;
    if (isR && rR < K) partner = (int)posL[first + rR];
    int cut = K < cL ? (int)posL[first + K] : 64;
    if (K > 0) cut = min(cut, (int)posR[first + K - 1]);
    cut = min(cut, b);
    is_wave_sync();  // the rank slots are rewritten by the next frame
    key = __shfl(key, partner);
    val = __shfl(val, partner);
    if (lane == sp) {
      st_a = a;
      st_b = cut;
      st_d = d;
    } else if (lane == sp + 1) {
      st_a = cut;
      st_b = b;
      st_d = d;
    }
    sp += 2;
  }
  if (lane < m) {
    k[first + lane] = key;
    v[first + lane] = val;
  }
  is_wave_sync();
}

template <typename FP>
__device__ __forceinline__ void is_push(FP f, int i, int first, int last, int depth) {
  f[3 * i] = first;
  f[3 * i + 1] = last;
  f[3 * i + 2] = depth;
}

constexpr int kIsBig = 2048;  // default: frames larger than this are partitioned by the whole workgroup

// The partition phase of std::sort on (k, v)[0, n) by one workgroup of T threads.  posL / posR:
// n-entry scratch; fa / fb: int frame lists {first, last, depth} of >= n / 17 + 2 entries each
// (3 ints per frame); sh: LDS ints (>= 2 * T / 64 + 8).  Starts and ends with a barrier.  A stable
// sort by key of the result is std::sort's.
// Each level's frames are pushed into the next list in two groups: the frames the whole workgroup
// partitions (larger than BIG, depth left) from the front, every other frame from the back, so no
// thread scans the whole list for the large ones (round 6: the per-ring key sequences are close to
// median-of-3's bad case, ~16 levels of one or two large frames and many small ones,
// tools/ring_partition_depth.py).  Depth-exhausted frames of at most 64 elements are heap-sorted in
// one wave's registers.
template <int T, typename KP, typename VP, typename PP, typename FP, int BIG = kIsBig>
__device__ __attribute__((always_inline)) void is_partition_phase(KP k, VP v, PP posL, PP posR, int n, FP fa, FP fb, int* sh) {
  constexpr int NW = T / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int* cnt = sh + 2 * NW + 2;  // [0] large frames of the current list, [1] others, [2] / [3] the same for the next
  const int capf = n / 17 + 2;  // frames per list; the others are stored from the back
  auto large = [](int first, int last, int depth) { return last - first > BIG && depth > 0; };
  __syncthreads();
  if (tid == 0) {
    cnt[0] = cnt[1] = 0;
    if (n > 16) {
      const int d = 2 * is_lg(n);
      if (large(0, n, d)) {
        is_push(fa, 0, 0, n, d);
        cnt[0] = 1;
      } else {
        is_push(fa, capf - 1, 0, n, d);
        cnt[1] = 1;
      }
    }
  }
  __syncthreads();
  // a child frame of more than 16 elements into the next list (one lane)
  auto push = [&](FP f, int first, int last, int depth) {
    if (last - first <= 16) return;
    if (large(first, last, depth)) is_push(f, atomicAdd(&cnt[2], 1), first, last, depth);
    else is_push(f, capf - 1 - atomicAdd(&cnt[3], 1), first, last, depth);
  };
  while (true) {
    const int nbig = cnt[0], nsmall = cnt[1];
    if (nbig + nsmall == 0) break;
    __syncthreads();
    if (tid == 0) cnt[2] = cnt[3] = 0;
    __syncthreads();
    // large frames: one at a time, every thread
    for (int f = 0; f < nbig; ++f) {
      const IsFrame F{fa[3 * f], fa[3 * f + 1], fa[3 * f + 2]};
      if (tid == 0) is_median_to_first(k, v, F.first, F.first + 1, F.first + (F.last - F.first) / 2, F.last - 1);
      __syncthreads();
      const uint32_t p = k[F.first];
      const int cut = is_block_partition<T>(k, v, posL, posR, F.first + 1, F.last, p, sh);
      if (tid == 0) {
        push(fb, F.first, cut, F.depth - 1);
        push(fb, cut, F.last, F.depth - 1);
      }
    }
    // the others: one wave each, wave w takes frames w, w + NW, ... (every wave runs the same
    // number of rounds: no wave leaves the loop early)
    for (int base = 0; base < nsmall; base += NW) {
      const int f = capf - 1 - (base + w);
      if (base + w >= nsmall) continue;  // wave-uniform
      const IsFrame F{fa[3 * f], fa[3 * f + 1], fa[3 * f + 2]};
      if (F.depth == 0) {  // partial_sort(first, last, last)
        const int m = F.last - F.first;
        if (m <= 64) {
          uint32_t key = lane < m ? (uint32_t)k[F.first + lane] : 0u, val = lane < m ? (uint32_t)v[F.first + lane] : 0u;
          is_reg_heap_sort(key, val, 0, m, lane);
          if (lane < m) {
            k[F.first + lane] = key;
            v[F.first + lane] = val;
          }
        } else if (lane == 0) {
          is_heap_sort(k, v, F.first, F.last);
        }
        is_wave_sync();
        continue;
      }
      if (F.last - F.first <= 64) {  // the frame's whole subtree in registers
        is_wave_small(k, v, posL, posR, F.first, F.last, F.depth, lane);
        continue;
      }
      if (lane == 0) is_median_to_first(k, v, F.first, F.first + 1, F.first + (F.last - F.first) / 2, F.last - 1);
      is_wave_sync();
      const uint32_t p = k[F.first];
      const int cut = is_wave_partition(k, v, posL, posR, F.first + 1, F.last, p, lane);
      if (lane == 0) {
        push(fb, F.first, cut, F.depth - 1);
        push(fb, cut, F.last, F.depth - 1);
      }
    }
    __syncthreads();
    if (tid == 0) {
      cnt[0] = cnt[2];
      cnt[1] = cnt[3];
    }
    FP t = fa;
    fa = fb;
    fb = t;
    __syncthreads();
  }
  (void)w;
}

}  // namespace fbr
