// k_features.hip — A6-A8: calculateSmoothness, markOccludedPoints, extractFeatures per ring.
//
// Reference: /root/reference/src/featureExtraction.h:109-131 (curvature), :134-176 (occlusion and
// parallel-beam marks), :178-294 (6 segments per ring: std::sort, 20 corners, surf picks with
// +-5 neighbour suppression, surf candidates label <= 0).
//
// One wave (64 lanes) owns one (job, ring).  Rings are independent: every read or write of
// ring i stays inside [startRingIndex-12, endRingIndex+11), so the wave stages that window of the
// flattened arrays in LDS.  The only cross-ring object is the stale
// cloudSmoothness[4] slot (never recomputed, :113) and cloudNeighborPicked[0..4]; they live in
// StreamState and are carried only in stream mode.
//
// Every per-index flag (occlusion marks, column gaps > 10, cloudNeighborPicked, cloudLabel,
// curvature above/below the thresholds) is a bit in 64-bit words over the window, produced by wave
// ballots; marks and suppression become shifted ORs.
//   * curvature: the reference's left-to-right f32 sum, no FMA.
//   * occlusion: the sequential loop only ever writes 1s, so cloudNeighborPicked is the OR of the
//     marks covering each index: picked = C | OR_{d=0..5} A>>d | OR_{d=1..6} B<<d.
//   * sort: per segment, an LDS bitonic sort of (curvature bits, position) keys — std::sort's order
//     whenever the segment has no tied (or NaN) curvature; a segment with ties runs the exact
//     libstdc++ introsort emulation (fbr_sort.h) on one lane instead.
//   * picks: the corner walk (descending, ep first, 20 per segment) and the surf walk (ascending,
//     ep last) are greedy: a candidate is taken iff no earlier-visited taken candidate suppresses
//     it.  Suppression reach (+-5 indices, stopped by a column gap > 10) depends only on
//     pointColInd and is symmetric, so the walk is a greedy independent set in visit-priority
//     order.  The wave resolves it in rounds on wave-uniform bitmasks: a candidate becomes "taken"
//     once every higher-priority conflicting candidate is "not taken", and "not taken" once one of
//     them is taken — final decisions, identical to the sequential walk.  The corner cap keeps the
//     first 20 taken in visit order.  The segment holding the stale slot keeps the sequential walk
//     (its stale index may duplicate a member).
// Outputs: label (the feature mask) and per-ring corner slots in visit order; the per-ring surf
// candidates (label <= 0, index order) are read from the mask by the per-ring VoxelGrid.
#include "fbr_common.h"
#include "fbr_kernels.h"
#include "fbr_sort.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace fbr {

// Synchronisation of code that one wave runs on its own (the single-wave kernel, or wave 0 of the
// multi-wave kernel while the helper waves wait at the next workgroup barrier): a workgroup-scope
// fence (every earlier LDS / global access of the wave has completed) and a wave barrier (no code
// motion across it).  For a one-wave workgroup this is what __syncthreads amounts to.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

namespace {
constexpr uint64_t kPadKey = kF64KeyMax;  // above every (curvature bits << 16 | position) key
constexpr int kSurfWindow = 64;  // batch surf walk: members resolved left of ep (FeatArgs::surf_full)
constexpr int kWin = 256 + 16;  // phase-2 window: 4 chunks + 8 on each side
constexpr int kWinBytes = kWin * (sizeof(float) + sizeof(int16_t));  // 1632 B per wave (16-B multiple)
}  // namespace

// Window bit-words (index i of the window <-> bit i&63 of word i>>6).
struct Bits {
  uint64_t* w;
  __device__ __forceinline__ bool get(int i) const { return (w[i >> 6] >> (i & 63)) & 1ull; }
  __device__ __forceinline__ void set_serial(int i) const { w[i >> 6] |= 1ull << (i & 63); }
};

struct FeatLds {
  int wlo, L, nw;
  float* gcurv;       // [Lcap] the ring window's curvature, in the ring's global scratch slot
  float* scurv;       // [segcap + 16] LDS copy of the current segment's [sp-6, ep+7) curvature
  int sbase;          // window index of scurv[0]
  Bits gap;           // |col[i+1]-col[i]| > 10
  Bits picked, labpos, labneg, edgec, surfc;
  Bits occa, occb, occc;
  uint32_t* cm;       // [segcap] conflict masks
  unsigned char* rb;  // region B: phase-2 range/col windows, then the taken-corner lists
  uint64_t* tmask;    // [WMAX] taken mask copy for the cap scan
  // sorted path (stale-slot segment, relevant ties): per-ring global scratch slot (but sorder / rankc)
  uint64_t* keys;     // [kseg]
  SmoothEntry* seg;   // [segcap] serial-path entries
  SmoothEntry* tmp;   // [segcap] materialisation scratch
  uint16_t* sorder;   // [segcap] member index at each sorted position (LDS region B)
  uint16_t* rankc;    // [segcap] corner visit rank of each member (LDS region B)
  SortFrame* sstack;  // [kSortStack] introsort emulation stack (tie segments, lane 0)
};

// 64 window bits [lo, lo+64) of a bit array; bits at negative window indices read as 1 (the
// suppression loops stop there) and bits past the array as 0.
__device__ __forceinline__ uint64_t bits64(const Bits& b, int lo, int nw) {
  const int w = lo >> 6, sh = lo & 63;  // arithmetic shift: floor for negative lo
  const uint64_t a = (w >= 0 && w < nw) ? b.w[w] : (w < 0 ? ~0ull : 0ull);
  const uint64_t c = (w + 1 >= 0 && w + 1 < nw) ? b.w[w + 1] : (w + 1 < 0 ? ~0ull : 0ull);
  return sh ? ((a >> sh) | (c << (64 - sh))) : a;
}

// Forward / backward suppression reach of window index li (<= 5 each): consecutive indices
// without a column gap > 10 (:230-240 / :262-274), from the gap bit words.
__device__ __forceinline__ int reach_fwd(const FeatLds& S, int li) {
  const uint64_t x = bits64(S.gap, li, S.nw);      // bit d = gap at li+d
  return __builtin_ctzll(x | 0x20ull);              // zeros before the first gap, capped at 5
}
__device__ __forceinline__ int reach_bwd(const FeatLds& S, int li) {
  const uint64_t x = bits64(S.gap, li - 64, S.nw);  // bit 63-d = gap at li-1-d
  return __builtin_clzll(x | (1ull << 58));        // capped at 5
}

// Bits [off, off+64) of the 192-bit value w0 | w1 << 64 | w2 << 128 (0 <= off < 128).
__device__ __forceinline__ uint64_t win64(uint64_t w0, uint64_t w1, uint64_t w2, int off) {
  if (off < 64) return off ? ((w0 >> off) | (w1 << (64 - off))) : w0;
  off -= 64;
  return off ? ((w1 >> off) | (w2 << (64 - off))) : w1;
}

// Mark cloudNeighborPicked over [li-bwd, li+fwd] (the suppression loops :227-240 / :259-274).
__device__ __forceinline__ void or_range(const Bits& b, int lo, int hi) {
  const int w0 = lo >> 6, w1 = hi >> 6;
  const uint64_t m0 = ~0ull << (lo & 63);
  const uint64_t m1 = (hi & 63) == 63 ? ~0ull : ((1ull << ((hi & 63) + 1)) - 1ull);
  if (w0 == w1) {
    atomicOr((unsigned long long*)&b.w[w0], (unsigned long long)(m0 & m1));
  } else {
    atomicOr((unsigned long long*)&b.w[w0], (unsigned long long)m0);
    atomicOr((unsigned long long*)&b.w[w1], (unsigned long long)m1);
  }
}

// cloudCurvature at window index li: the segment's LDS copy, or the global slot outside it (the
// stale cloudSmoothness[4] index may point anywhere in the ring window).
__device__ __forceinline__ float curv_at(const FeatLds& S, int li, int slen) {
  const int k = li - S.sbase;
  return (k >= 0 && k < slen) ? S.scurv[k] : S.gcurv[li];
}

// Sequential walks (the reference loops verbatim) over S.seg[0..m] (seg[m] = the unsorted ep entry).
__device__ __forceinline__ void serial_walks(const FeatLds& S, int slen, const SmoothEntry* ent, const FeatArgs& a, int job, int m,
                             const float4* CL, float4* corner_out, int& corner_cnt) {
  int largestPickedNum = 0;
  for (int k = m; k >= 0; k--) {  // corners, k = ep .. sp (:208-242)
    const int ind = ent[k].ind;
    const int li = ind - S.wlo;
    if (li < 0 || li + 5 >= S.L) { atomicOr(&a.err[job], 4); return; }
    if (!S.picked.get(li) && curv_at(S, li, slen) > a.edge_thr) {
      largestPickedNum++;
      if (largestPickedNum <= kCornerPerSeg) {
        S.labpos.set_serial(li);
        corner_out[corner_cnt++] = CL[ind];
      } else {
        break;
      }
      S.picked.set_serial(li);
      const int f = reach_fwd(S, li), b = reach_bwd(S, li);  // index -1 (col[-1]) is scratch
      for (int l = 1; l <= f; ++l) S.picked.set_serial(li + l);
      for (int l = 1; l <= b; ++l) S.picked.set_serial(li - l);
    }
  }
  for (int k = 0; k <= m; k++) {  // surf, k = sp .. ep (:245-276)
    const int ind = ent[k].ind;
    const int li = ind - S.wlo;
    if (li < 0 || li + 5 >= S.L) { atomicOr(&a.err[job], 4); return; }
    if (!S.picked.get(li) && curv_at(S, li, slen) < a.surf_thr) {
      S.labneg.set_serial(li);
      S.picked.set_serial(li);
      const int f = reach_fwd(S, li), b = reach_bwd(S, li);
      for (int l = 1; l <= f; ++l) S.picked.set_serial(li + l);
      for (int l = 1; l <= b; ++l) S.picked.set_serial(li - l);
    }
  }
}

// 10 neighbour bits of member (64*w + lane) from the wave-uniform masks of words w-1, w, w+1:
// bit 5+d for d in [-5,-1], bit 4+d for d in [1,5] (the cm encoding).
__device__ __forceinline__ uint32_t win10(uint64_t a, uint64_t b, uint64_t c, int lane) {
  const int start = 59 + lane;  // bit (64 + lane - 5) of the 192-bit concatenation a | b<<64 | c<<128
  uint64_t x;
  if (start < 64) {
    x = (a >> start) | (b << (64 - start));
  } else {
    const int s2 = start - 64;
    x = (b >> s2) | (s2 ? (c << (64 - s2)) : 0ull);
  }
  const uint32_t w11 = (uint32_t)(x & 0x7FFull);
  return (w11 & 0x1Fu) | ((w11 >> 6) << 5);
}

// Greedy rounds.  cmbits(u) = 10-bit mask of the higher-priority conflicting members of u.
// und: candidate members on entry; on exit tak = the members the sequential walk takes.
// frz (optional): frozen members -- candidates outside the resolved window, kept undecided: they
// block the members they outrank and are never decided themselves; the rounds then stop when a
// round decides nothing (members whose outcome depends on a frozen one stay in und).
template <int WMAX, typename CmF>
__device__ __forceinline__ void greedy_rounds(int m, int lane, uint64_t (&und)[WMAX], uint64_t (&tak)[WMAX], CmF cmbits,
                              const FeatArgs& a, int job, const uint64_t* frz = nullptr) {
  const int nwm = (m >> 6) + 1;
  uint32_t cmr[WMAX];
#pragma unroll
  for (int w = 0; w < WMAX; ++w) cmr[w] = (w < nwm && 64 * w + lane <= m) ? cmbits(64 * w + lane) : 0u;
  for (int round = 0;; ++round) {
    bool any = false, progress = false;
#pragma unroll
    for (int w = 0; w < WMAX; ++w) {
      const uint64_t live = frz ? und[w] & ~frz[w] : und[w];
      if (w < nwm && live != 0ull) {  // words whose candidates are all decided are skipped
        bool nt = false, tk = false;
        const bool mine = (live >> lane) & 1ull;
        if (mine) {
          const uint32_t wt = win10(w > 0 ? tak[w - 1] : 0ull, tak[w], w + 1 < WMAX ? tak[w + 1] : 0ull, lane);
          const uint32_t wu = win10(w > 0 ? und[w - 1] : 0ull, und[w], w + 1 < WMAX ? und[w + 1] : 0ull, lane);
          if (wt & cmr[w]) nt = true;
          else if (!(wu & cmr[w])) tk = true;
        }
        const uint64_t bt = __ballot(tk);
        tak[w] |= bt;
        // members suppressed by a member taken just now are decided in the same round (a
        // monotone-priority run then resolves 6 members per round instead of 3)
        if (bt != 0ull && mine && !tk && !nt) {
          const uint32_t wt = win10(w > 0 ? tak[w - 1] : 0ull, tak[w], w + 1 < WMAX ? tak[w + 1] : 0ull, lane);
          nt = (wt & cmr[w]) != 0u;
        }
        const uint64_t bn = __ballot(nt);
        und[w] &= ~(bt | bn);
        progress |= (bt | bn) != 0ull;
        any |= (frz ? und[w] & ~frz[w] : und[w]) != 0ull;
      }
    }
    if (!any || (frz && !progress)) break;
    if (round > 4 * (m + 2)) {  // unreachable: each round decides the best-ranked undecided
      if (lane == 0) atomicOr(&a.err[job], 8);
      break;
    }
  }
}

// libstdc++ 11 std::sort on a segment with tied curvatures, wave-parallel.  The final
// __insertion_sort / __unguarded_insertion_sort pass is stable, so std::sort's result is the
// stable sort of the array as the introsort partition phase leaves it.  That phase is reproduced
// exactly: __unguarded_partition(lo, hi, pivot) swaps the k-th element (from the left) that is
// not < pivot with the k-th element (from the right) that is not > pivot while the former lies
// left of the latter, and returns min(g_K, r_{K-1}) for the first k = K where that fails
// (swapped elements stop the scans).  Checked against std::sort on tie-heavy arrays
// (tests/test_oracle_pinning.py).  Depth exhaustion falls back to the serial heap sort.
__device__ __forceinline__ int wave_partition(SmoothEntry* a, int lo, int hi, float p, uint16_t* posL, uint16_t* posR,
                                              int lane) {
  int cntL = 0;
  for (int b = lo; b < hi; b += 64) {
    const int i = b + lane;
    const bool isL = i < hi && !(a[i].v < p);
    const uint64_t bl = __ballot(isL);
    if (isL) posL[cntL + __popcll(bl & ((1ull << lane) - 1ull))] = (uint16_t)i;
    cntL += __popcll(bl);
  }
  int cntR = 0;
  for (int t = hi - 1; t >= lo; t -= 64) {
    const int i = t - lane;
    const bool isR = i >= lo && !(p < a[i].v);
    const uint64_t br = __ballot(isR);
    if (isR) posR[cntR + __popcll(br & ((1ull << lane) - 1ull))] = (uint16_t)i;
    cntR += __popcll(br);
  }
  wsync();
  const int mn = min(cntL, cntR);
  int K1 = 0;  // swaps performed = number of k with g_k < r_k (a prefix of k)
  for (int k0 = 0; k0 < mn; k0 += 64) {
    const int k = k0 + lane;
    const uint64_t bo = __ballot(k < mn && posL[k] < posR[k]);
    K1 += __popcll(bo);
    if (bo != ~0ull) break;
  }
  for (int k = lane; k < K1; k += 64) {
    const int x = posL[k], y = posR[k];
    const SmoothEntry t = a[x];
    a[x] = a[y];
    a[y] = t;
  }
  int cut = K1 < cntL ? posL[K1] : INT_MAX;
  if (K1 > 0) cut = min(cut, posR[K1 - 1]);
  wsync();
  return min(cut, hi);
}

__device__ __forceinline__ void wave_introsort_partitions(SmoothEntry* a, int n, SortFrame* stack, uint16_t* posL,
                                                          uint16_t* posR, int lane) {
  int sp = 0;
  stack[sp++] = SortFrame{0, n, 2 * sm_lg(n)};  // every lane writes / reads the same frames
  while (sp > 0) {
    const SortFrame f = stack[--sp];
    int first = f.first, last = f.last, depth = f.depth;
    while (last - first > 16) {
      if (depth == 0) {  // std::partial_sort(first, last, last)
        if (lane == 0) sm_heap_sort(a, first, last);
        wsync();
        break;
      }
      --depth;
      const int mid = first + (last - first) / 2;
      if (lane == 0) sm_move_median_to_first(a, first, first + 1, mid, last - 1);
      wsync();
      const int cut = wave_partition(a, first + 1, last, a[first].v, posL, posR, lane);
      if (sp < kSortStack) stack[sp++] = SortFrame{cut, last, depth};
      last = cut;
    }
  }
  wsync();
}

// Bitonic sort of kpow (power of two, <= 128 * QP) 64-bit keys held in registers: element
// e = 64 * r + lane sits in register r of its lane, so a compare-exchange at distance j2 < 64 is a
// lane shuffle and one at j2 >= 64 is between two registers of the same lane.  keys[] is read
// once and written once (it was a global-scratch network with a wave sync per stage).  The keys
// are below 2^48, so the exchanges run on the f64 unit (key_min / key_max, fbr_common.h).
template <int QP>
__device__ __forceinline__ void bitonic_sort_keys(uint64_t* keys, int kpow, int lane) {
  constexpr int KPL = 2 * QP;
  uint64_t k[KPL];
#pragma unroll
  for (int r = 0; r < KPL; ++r) k[r] = 64 * r + lane < kpow ? keys[64 * r + lane] : kPadKey;
  for (int k2 = 2; k2 <= kpow; k2 <<= 1) {
    for (int j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
      if (j2 >= 64) {  // register distance jr (a compile-time index per case)
        auto step = [&](auto JR) __attribute__((always_inline)) {
          constexpr int jr = decltype(JR)::value;
#pragma unroll
          for (int r = 0; r < KPL; ++r) {
            if constexpr (jr < KPL) {
              if ((r & jr) == 0 && r + jr < KPL) {
                const int e = 64 * r + lane;
                const bool up = (e & k2) == 0;
                const uint64_t x = k[r], y = k[(r + jr) % KPL];
                const uint64_t mn = key_min(x, y), mx = key_max(x, y);
                k[r] = up ? mn : mx;
                k[(r + jr) % KPL] = up ? mx : mn;
              }
            }
          }
        };
        switch (j2 >> 6) {
          case 1: step(std::integral_constant<int, 1>{}); break;
          case 2: step(std::integral_constant<int, 2>{}); break;
          case 4: step(std::integral_constant<int, 4>{}); break;
          case 8: step(std::integral_constant<int, 8>{}); break;
          default: break;
        }
      } else {
        const bool lower = (lane & j2) == 0;
#pragma unroll
        for (int r = 0; r < KPL; ++r) {
          const int e = 64 * r + lane;
          const bool up = (e & k2) == 0;
          const uint64_t x = k[r];
          const uint32_t ylo = __shfl_xor((uint32_t)x, j2), yhi = __shfl_xor((uint32_t)(x >> 32), j2);
          const uint64_t y = ((uint64_t)yhi << 32) | ylo;
          const uint64_t mn = key_min(x, y), mx = key_max(x, y);
          k[r] = (lower == up) ? mn : mx;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < KPL; ++r)
    if (64 * r + lane < kpow) keys[64 * r + lane] = k[r];
  wsync();
}

// The stale-slot segment's walks (the reference loops of serial_walks) with the wave's lanes as
// the picked-word window: lane i holds picked word w_lo + i, so a test is one readlane of a
// wave-uniform word and a suppression range is one masked OR per lane.  Every entry's window
// index, candidate tests and suppression reach are computed lane-parallel first (info[k]); the
// walks then visit the entries in order on wave-uniform values, record the taken corners and
// write the picked / label words back.  Returns false (nothing written) when an entry lies
// outside the ring window or the window spans more than 64 words; the caller then runs
// serial_walks (which reports the error, as the reference's out-of-range access has no answer).
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ bool stale_walks_fast(const FeatLds& S, int slen, const SmoothEntry* ent, const FeatArgs& a, int m,
                                 const float4* CL, float4* corner_out, int& corner_cnt, uint32_t* info,
                                 int32_t* tlist, int lane) {
  int lo_li = INT_MAX, hi_li = INT_MIN;
  bool bad = false;
  for (int k0 = 0; k0 <= m; k0 += 64) {
    const int k = k0 + lane;
    if (k <= m) {
      const int li = ent[k].ind - S.wlo;
      uint32_t v = 0u;
      if (li >= 0 && li + 5 < S.L) {
        const float cv = curv_at(S, li, slen);
        const int f = reach_fwd(S, li), b = reach_bwd(S, li);
        v = (uint32_t)li | ((uint32_t)f << 16) | ((uint32_t)b << 19) | ((cv > a.edge_thr) ? 1u << 22 : 0u) |
            ((cv < a.surf_thr) ? 1u << 23 : 0u);
        lo_li = min(lo_li, li - b);
        hi_li = max(hi_li, li + f);
      } else {
        bad = true;
      }
      info[k] = v;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo_li = min(lo_li, __shfl_xor(lo_li, o));
    hi_li = max(hi_li, __shfl_xor(hi_li, o));
  }
  wsync();
  if (__any(bad) || lo_li < 0) return false;
  const int w_lo = lo_li >> 6;
  if ((hi_li >> 6) - w_lo >= 64) return false;
  const int myw = w_lo + lane;
  uint64_t pv = myw < S.nw ? S.picked.w[myw] : 0ull;
  auto is_picked = [&](int li) __attribute__((always_inline)) {
    return (readlane64(pv, (li >> 6) - w_lo) >> (li & 63)) & 1ull;
  };
  auto mark = [&](int lo, int hi) __attribute__((always_inline)) {  // picked over [lo, hi]
    const int w0 = (lo >> 6) - w_lo, w1 = (hi >> 6) - w_lo;
    uint64_t mm = (lane >= w0 && lane <= w1) ? ~0ull : 0ull;
    if (lane == w0) mm &= ~0ull << (lo & 63);
    if (lane == w1) mm &= (hi & 63) == 63 ? ~0ull : ((1ull << ((hi & 63) + 1)) - 1ull);
    pv |= mm;
  };
  // corners: k = ep .. sp (:208-242); the walks visit only the entries that pass the curvature
  // test (a ballot per 64 entries: the others are no-ops in the reference loops)
  int taken = 0;
  bool stop = false;
  for (int c0 = (m >> 6) << 6; c0 >= 0 && !stop; c0 -= 64) {
    const uint32_t vv = c0 + lane <= m ? info[c0 + lane] : 0u;
    uint64_t cand = __ballot((vv >> 22) & 1u);
    while (cand) {
      const int l = 63 - __builtin_clzll(cand);  // descending entries
      cand &= ~(1ull << l);
      const uint32_t v = __builtin_amdgcn_readlane(vv, l);
      const int li = (int)(v & 0xFFFFu);
      if (is_picked(li)) continue;
      if (++taken > kCornerPerSeg) {
        stop = true;
        break;
      }
      if (lane == 0) {
        tlist[taken - 1] = li + S.wlo;
        atomicOr((unsigned long long*)&S.labpos.w[li >> 6], 1ull << (li & 63));
      }
      mark(li - (int)((v >> 19) & 7u), li + (int)((v >> 16) & 7u));
    }
  }
  const int nc = min(taken, kCornerPerSeg);
  // surf: k = sp .. ep (:245-276); the picked-surf labels collect in the lanes' window words
  uint64_t lv = 0ull;
  for (int c0 = 0; c0 <= m; c0 += 64) {
    const uint32_t vv = c0 + lane <= m ? info[c0 + lane] : 0u;
    uint64_t cand = __ballot((vv >> 23) & 1u);
    while (cand) {
      const int l = __builtin_ctzll(cand);  // ascending entries
      cand &= cand - 1ull;
      const uint32_t v = __builtin_amdgcn_readlane(vv, l);
      const int li = (int)(v & 0xFFFFu);
      if (is_picked(li)) continue;
      lv |= lane == (li >> 6) - w_lo ? 1ull << (li & 63) : 0ull;
      mark(li - (int)((v >> 19) & 7u), li + (int)((v >> 16) & 7u));
    }
  }
  if (lv) atomicOr((unsigned long long*)&S.labneg.w[myw], (unsigned long long)lv);
  if (myw < S.nw) S.picked.w[myw] = pv;
  wsync();
  for (int t = lane; t < nc; t += 64) corner_out[corner_cnt + t] = CL[tlist[t]];
  corner_cnt += nc;
  wsync();
  return true;
}

// Diagnostic build only (-DFBR_FEAT_STAMPS, tools/feat_stamps.py): per-phase s_memtime cycle sums
// per ring into FeatArgs::stamps.  The shipped library is compiled without it.
#ifdef FBR_FEAT_STAMPS
#define FBR_STAMP(i)                                               \
  do {                                                             \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
    stamp_acc[i] += t_ - stamp_last;                               \
    stamp_last = t_;                                               \
  } while (0)
#else
#define FBR_STAMP(i) \
  do {               \
  } while (0)
#endif

// WMAX: 64-bit words of segment-member masks (members <= 64*WMAX); QP: bitonic pairs per lane
// (segment sort <= 128*QP keys).  <6,4> covers Horizon_SCAN <= 2048, <12,8> up to 4096.
// NWV: waves per ring.  NWV = 1 for large launches (every SIMD holds many ring waves, so one wave
// per ring hides its LDS latency behind the others).  With few rings per SIMD (single scans,
// small batches) a ring's critical path is one wave's latency chain, so NWV > 1 spreads the
// lane-parallel passes (flags and curvature, the conflict masks of each segment, the outputs)
// over NWV waves, while wave 0 alone runs the walks (ballot masks, greedy rounds, the sorted
// path) between workgroup barriers.
template <int WMAX, int QP, int NWV>
__global__ void __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NWV > 1 ? 2 : 4)))
k_features(FeatArgs a) {
  constexpr int NT = 64 * NWV;
#ifdef FBR_FEAT_STAMPS
  unsigned long long stamp_acc[12] = {0}, stamp_last = __builtin_amdgcn_s_memtime();
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = a.H, W = a.W;
  // Ring 0 of every job first: its segment 0 holds the stale cloudSmoothness[4] slot and runs the
  // serial walk, the longest wave of the launch; dispatching those waves first hides them behind
  // the other rings instead of leaving the last jobs' ones in the tail.
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int job = b < a.B ? b : (b - a.B) / (H - 1);
  const int ring = b < a.B ? 0 : 1 + (b - a.B) % (H - 1);
  const int64_t HW = (int64_t)H * W;
  const int n = a.nvalid[job];
  const int s = a.start_ring[job * H + ring], e = a.end_ring[job * H + ring];
  const int cb = s - 4, ca = e + 6;  // this ring's points [cb, ca)
  const int slot = job * H + ring;
  if (ca <= cb) {
    if (tid == 0) a.corner_cnt[slot] = 0;
    return;
  }
  FeatLds S;
  S.wlo = max(s - 12, 0);
  const int whi = min(e + 11, n);
  S.L = whi - S.wlo;
  S.nw = (S.L + 63) >> 6;
  const int Lcap = a.lcap, segcap = a.segcap, nwcap = a.nwcap, kseg = a.kseg;
  if (S.L > Lcap) {
    if (tid == 0) atomicOr(&a.err[job], 1);
    return;
  }
  unsigned char* p = smem;
  S.scurv = (float*)p;               p += sizeof(float) * ((segcap + 19) & ~3);  // 16-B multiple: the
                                                                                 // bit words below are 64-bit
  uint64_t* words = (uint64_t*)p;    p += sizeof(uint64_t) * 9 * nwcap;  // 9 bit arrays of nwcap words
  S.gap.w = words;
  S.picked.w = words + 1 * nwcap;
  S.labpos.w = words + 2 * nwcap;
  S.labneg.w = words + 3 * nwcap;
  S.edgec.w = words + 4 * nwcap;
  S.surfc.w = words + 5 * nwcap;
  S.occa.w = words + 6 * nwcap;
  S.occb.w = words + 7 * nwcap;
  S.occc.w = words + 8 * nwcap;
  S.tmask = (uint64_t*)p;            p += sizeof(uint64_t) * 16;
  S.sstack = (SortFrame*)p;          p += sizeof(SortFrame) * kSortStack;
  S.cm = (uint32_t*)p;               p += sizeof(uint32_t) * segcap;
  S.rb = smem + (((p - smem) + 15) & ~15);  // offset arithmetic: keeps the LDS address space (ds_*, not flat_*)
  {
    unsigned char* g = a.gscratch + (int64_t)slot * a.gslot_bytes;
    S.keys = (uint64_t*)g;           g += sizeof(uint64_t) * kseg;
    S.seg = (SmoothEntry*)g;         g += sizeof(SmoothEntry) * segcap;
    S.tmp = (SmoothEntry*)g;         g += sizeof(SmoothEntry) * segcap;
    g += 2 * sizeof(uint16_t) * segcap;  // (sorder / rankc: in region B below)
    unsigned char* g0 = a.gscratch + (int64_t)slot * a.gslot_bytes;
    S.gcurv = (float*)(g0 + (((g - g0) + 15) & ~(int64_t)15));
  }
  // the sorted path's member order and ranks in LDS region B (free from the tie sort's end to the
  // corner cap scan, the only readers; the cm loop reads ~10 ranks per member)
  S.sorder = (uint16_t*)S.rb;
  S.rankc = S.sorder + segcap;
  S.sbase = 0;

  const float* R = a.range + job * HW;
  const int32_t* C = a.col + job * HW;
  const float4* CL = a.cloud + job * HW;
  StreamState* st = a.stream + job;
  for (int w = tid; w < 9 * nwcap; w += NT) words[w] = 0ull;
  __syncthreads();
  FBR_STAMP(0);
  // ---- phase 2: occlusion marks, column gaps, curvature, threshold bits (chunk c = 64 indices) ----
  // range / col are staged per group of 4 chunks: window [256g - 8, 256g + 264) in region B (a
  // window per wave); with one wave the next group's window is loaded into registers while this
  // group is processed, with several the waves take the groups in turn
  float* rw = (float*)(S.rb + wv * kWinBytes);
  int16_t* cw = (int16_t*)(rw + kWin);
  constexpr int kWq = (kWin + 63) / 64;
  float rv[kWq];
  int cv[kWq];
  auto load_window = [&](int c) __attribute__((always_inline)) {
    const int wb = 64 * c - 8;
#pragma unroll
    for (int q = 0; q < kWq; ++q) {
      const int t = 64 * q + lane, idx = wb + t;
      const bool in = t < kWin && idx >= 0 && idx < S.L;
      rv[q] = in ? R[S.wlo + idx] : 0.0f;
      cv[q] = in ? C[S.wlo + idx] : 0;
    }
  };
  auto store_window = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < kWq; ++q) {
      const int t = 64 * q + lane;
      if (t < kWin) {
        rw[t] = rv[q];
        cw[t] = (int16_t)cv[q];
      }
    }
  };
  auto chunk = [&](int c) __attribute__((always_inline)) {
    const int i = 64 * c + lane;
    const int j = S.wlo + i;
    const int wo = 64 * (c & ~3) - 8;  // window origin of this chunk's group
    // Branch-free: every window read is in bounds (t in [8, 264), margins of 8), values past the
    // ring are masked by the conditions; the arithmetic is the reference's, in its order.
    const int t = i - wo;
    const float rm5 = rw[t - 5], rm4 = rw[t - 4], rm3 = rw[t - 3], rm2 = rw[t - 2], rm1 = rw[t - 1], r0 = rw[t];
    const float rp1 = rw[t + 1], rp2 = rw[t + 2], rp3 = rw[t + 3], rp4 = rw[t + 4], rp5 = rw[t + 5];
    const int c0 = cw[t], c1 = cw[t + 1];
    const bool inL = i < S.L, has1 = i + 1 < S.L;
    const int columnDiff = abs(c1 - c0);
    const bool gp = !(inL & has1) | (columnDiff > 10);
    const bool occ = inL & has1 & (j >= 5) & (j < n - 6) & (i >= 1);  // markOccludedPoints (:140-175)
    const bool near = columnDiff < 10;
    const bool a1 = (double)(r0 - rp1) > 0.3;  // depth1 - depth2
    const bool fa = occ & near & a1;
    const bool fb = occ & near & !a1 & ((double)(rp1 - r0) > 0.3);
    const float diff1 = fabsf(rm1 - r0), diff2 = fabsf(rp1 - r0);
    const bool fc = occ & ((double)diff1 > 0.02 * (double)r0) & ((double)diff2 > 0.02 * (double)r0);
    const bool smooth_ok = inL & (j >= 5) & (j < n - 5) & (i >= 5) & (i + 5 < S.L);  // calculateSmoothness (:113-122)
    const float d = rm5 + rm4 + rm3 + rm2 + rm1 - r0 * 10.0f + rp1 + rp2 + rp3 + rp4 + rp5;
    const float curv = smooth_ok ? d * d : 0.0f;
    if (inL) S.gcurv[i] = curv;  // indices outside [5, n-5) keep the zero-initialised scratch value
    const uint64_t ba = __ballot(fa), bb = __ballot(fb), bc = __ballot(fc), bg = __ballot(gp);
    const uint64_t be = __ballot(i < S.L && curv > a.edge_thr);
    const uint64_t bs = __ballot(i < S.L && curv < a.surf_thr);
    if (lane == 0) {
      S.occa.w[c] = ba;
      S.occb.w[c] = bb;
      S.occc.w[c] = bc;
      S.gap.w[c] = bg;
      S.edgec.w[c] = be;
      S.surfc.w[c] = bs;
    }
  };
  if constexpr (NWV == 1) {
    load_window(0);
    for (int c = 0; c < S.nw; ++c) {
      if ((c & 3) == 0) {
        wsync();
        store_window();
        wsync();
        if (c + 4 < S.nw) load_window(c + 4);
      }
      chunk(c);
    }
  } else {
    const int G = (S.nw + 3) >> 2;  // groups of 4 chunks, dealt round-robin; uniform trip count
    for (int g0 = 0; g0 < G; g0 += NWV) {
      const int g = g0 + wv;
      if (g < G) {
        load_window(4 * g);
        store_window();
      }
      __syncthreads();
      if (g < G)
        for (int c = 4 * g; c < min(4 * g + 4, S.nw); ++c) chunk(c);
      __syncthreads();
    }
  }
  __syncthreads();
  // cloudNeighborPicked: reset over [5, n-5) (:124) then the marks; indices < 5 keep stream state
  for (int c = tid; c < S.nw; c += NT) {
    const uint64_t A = S.occa.w[c], An = c + 1 < S.nw ? S.occa.w[c + 1] : 0ull;
    const uint64_t B = S.occb.w[c], Bp = c > 0 ? S.occb.w[c - 1] : 0ull;
    uint64_t mk = S.occc.w[c] | A;
#pragma unroll
    for (int d = 1; d <= 5; ++d) mk |= (A >> d) | (An << (64 - d));
#pragma unroll
    for (int d = 1; d <= 6; ++d) mk |= (B << d) | (Bp >> (64 - d));
    if (c == 0 && S.wlo == 0)
      for (int k = 0; k < 5 && k < S.L; ++k)
        if (st->picked04[k]) mk |= 1ull << k;
    S.picked.w[c] = mk;
  }
  __syncthreads();
  FBR_STAMP(1);

  // ---- extractFeatures (:188-285) ----
  int corner_cnt = 0;
  float4* corner_out = a.corner_slot + (int64_t)slot * kCornerPerRing;
  // The next non-empty segment's curvature window is loaded into registers during this segment's
  // surf walk and written to LDS after it (windows up to 64 * kCq entries; longer ones, the first
  // segment and the segment after a stale-slot one are staged on the spot).
  constexpr int kCq = WMAX;  // 384 entries for W <= 2048
  float cpf[kCq];
  int pf_seg = -1, pf_next = -1, pf_len = 0;
  auto prefetch_curv = [&](int j0) __attribute__((always_inline)) {
    pf_next = -1;
    for (int jj = j0; jj < 6; ++jj) {
      const int psp = (s * (6 - jj) + e * jj) / 6, pep = (s * (5 - jj) + e * (jj + 1)) / 6 - 1;
      if (psp >= pep) continue;
      const int pb = max(psp - S.wlo - 6, 0), pl = min(pep - S.wlo + 7, S.L) - pb;
      if (pl > 64 * kCq || pep - psp + 1 > segcap) return;
#pragma unroll
      for (int q = 0; q < kCq; ++q) cpf[q] = S.gcurv[pb + min(64 * q + lane, pl - 1)];  // clamped: no branch
      pf_next = jj;
      pf_len = pl;
      return;
    }
  };
  int lastj = -1;  // the ring's last non-empty segment
  for (int j = 0; j < 6; j++)
    if ((s * (6 - j) + e * j) / 6 < (s * (5 - j) + e * (j + 1)) / 6 - 1) lastj = j;
  for (int j = 0; j < 6; j++) {
    const int sp = (s * (6 - j) + e * j) / 6;
    const int ep = (s * (5 - j) + e * (j + 1)) / 6 - 1;
    if (sp >= ep) continue;
    const int m = ep - sp;
    if (m + 1 > segcap || m > kseg) {
      if (tid == 0) atomicOr(&a.err[job], 2);
      return;
    }
    // stage this segment's curvature window [sp-6, ep+7) in LDS (members +-5 plus ep)
    S.sbase = max(sp - S.wlo - 6, 0);
    const int slen = min(ep - S.wlo + 7, S.L) - S.sbase;
    if (pf_seg != j)
      for (int t = tid; t < slen; t += NT) S.scurv[t] = S.gcurv[S.sbase + t];
    __syncthreads();
#ifdef FBR_FEAT_SKIP_STALE
    const bool has_stale = false;  // diagnostic ablation only
#else
    const bool has_stale = (sp <= 4 && 4 < ep);
#endif
    // Visit priority.  The greedy walks depend only on the relative priority of conflicting
    // neighbours, and the corner cap / output order only on the order of the taken corners, so
    // without ties among those no sort is needed: priorities come from curvature comparisons
    // (corner walk: ep first, then descending; surf walk: the reverse).  The stale-slot segment
    // and segments with a relevant tie (their order is introsort's) take the sorted path.
    auto sorted_order = [&]() __attribute__((always_inline)) {
      // -- sort [sp, ep) by (curvature bits, position) --
      int kpow = 1;
      while (kpow < m) kpow <<= 1;
      for (int t = lane; t < kpow; t += 64) {
        uint64_t key = kPadKey;
        if (t < m) {
          const int pos = sp + t;
          const float v = (pos == 4) ? st->smooth4_value : S.scurv[pos - S.wlo - S.sbase];
          key = ((uint64_t)__float_as_uint(v) << 16) | (uint64_t)t;
        }
        S.keys[t] = key;
      }
      wsync();
      bitonic_sort_keys<QP>(S.keys, kpow, lane);
      bool tflag = false, nflag = false;
      for (int t = lane; t < m; t += 64) {
        const uint32_t vb = (uint32_t)(S.keys[t] >> 16);
        nflag |= vb > 0x7f800000u;  // NaN
        if (t + 1 < m) tflag |= (uint32_t)(S.keys[t + 1] >> 16) == vb;
      }
      const bool nan = __any(nflag);
      const bool tie = __any(tflag) || nan;
      FBR_STAMP(2);
      if (tie) {
        // equal curvatures: their order is introsort's; materialise std::sort's result in S.seg
        // (the partition phase on an LDS copy in region B, 8 B x segcap, whose lists are dead here,
        // with the partition positions as u16 in cm: no global round trip per partition step)
        SmoothEntry* A = nan ? S.seg : (SmoothEntry*)S.rb;
        for (int t = lane; t < m; t += 64) {
          const int pos = sp + t;
          A[t] = (pos == 4) ? SmoothEntry{st->smooth4_value, st->smooth4_ind} : SmoothEntry{S.scurv[pos - S.wlo - S.sbase], pos};
        }
        wsync();
        if (nan) {
          if (lane == 0) std_sort_emul(S.seg, m, S.sstack);
          wsync();
        } else {
          wave_introsort_partitions(A, m, S.sstack, (uint16_t*)S.cm, (uint16_t*)S.cm + segcap, lane);
          for (int t = lane; t < kpow; t += 64)
            S.keys[t] = t < m ? (((uint64_t)__float_as_uint(A[t].v) << 16) | (uint64_t)t) : kPadKey;
          wsync();
          bitonic_sort_keys<QP>(S.keys, kpow, lane);  // stable sort of the partitioned array
          for (int k = lane; k < m; k += 64) S.seg[k] = A[S.keys[k] & 0xFFFFu];
          wsync();
        }
      } else if (has_stale) {
        for (int k = lane; k < m; k += 64) {
          const int pos = sp + (int)(S.keys[k] & 0xFFFFu);
          S.seg[k] = (pos == 4) ? SmoothEntry{st->smooth4_value, st->smooth4_ind} : SmoothEntry{S.scurv[pos - S.wlo - S.sbase], pos};
        }
        wsync();
      }
      if (has_stale) {
        if (lane == 0) {
          S.seg[m] = SmoothEntry{S.scurv[ep - S.wlo - S.sbase], ep};  // cloudSmoothness[ep] is never sorted (:203)
          st->smooth4_value = S.seg[4 - sp].v;            // the entry left at position 4 is the next
          st->smooth4_ind = S.seg[4 - sp].ind;            // scan's stale slot
        }
        wsync();
      }
      if (!has_stale) {
        // members u in [0, m] (index sp+u): sorted order, visit ranks, conflict masks
        for (int k = lane; k <= m; k += 64) {
          const int u = (k == m) ? m : (tie ? S.seg[k].ind - sp : (int)(S.keys[k] & 0xFFFFu));
          S.sorder[k] = (uint16_t)u;
          S.rankc[u] = (uint16_t)(k == m ? 0 : m - k);  // corner visit order: ep, then descending
        }
        wsync();
        for (int u = lane; u <= m; u += 64) {
          const int li = sp + u - S.wlo;
          const int f = reach_fwd(S, li), b = reach_bwd(S, li);
          const int ru = S.rankc[u];
          uint32_t nb = 0, hc = 0;
          int rn[10];
#pragma unroll
          for (int d = 1; d <= 5; ++d) {  // independent LDS reads, then the masks
            rn[4 + d] = (d <= f && u + d <= m) ? (int)S.rankc[u + d] : INT_MAX;
            rn[5 - d] = (d <= b && u - d >= 0) ? (int)S.rankc[u - d] : INT_MAX;
          }
#pragma unroll
          for (int d = 1; d <= 5; ++d) {
            if (d <= f && u + d <= m) nb |= 1u << (4 + d);
            if (d <= b && u - d >= 0) nb |= 1u << (5 - d);
            if (rn[4 + d] < ru) hc |= 1u << (4 + d);
            if (rn[5 - d] < ru) hc |= 1u << (5 - d);
          }
          S.cm[u] = hc | (nb << 10) | ((uint32_t)f << 20) | ((uint32_t)b << 24);
        }
        wsync();
      }
    };
    float* tlv = (float*)S.rb;                         // direct path: taken corners (value, member)
    uint16_t* tlu = (uint16_t*)(tlv + segcap);
    uint16_t* vis = tlu + segcap;                      // taken corners in visit order
    // Conflict masks of member u from curvature comparisons (the direct path): returns whether a
    // conflicting neighbour has the same curvature (its order would be introsort's).
    auto cm_member = [&](int u) __attribute__((always_inline)) -> bool {
      const int li = sp - S.wlo + u;
      const int f = reach_fwd(S, li), b = reach_bwd(S, li);
      float cv[11];
#pragma unroll
      for (int d = 0; d < 11; ++d) cv[d] = S.scurv[max(li + d - 5, 0) - S.sbase];
      const float vu = cv[5];
      // neighbour bits (bit 4+d forward, 5-d backward) as ranges: forward d <= min(f, m-u),
      // backward d <= min(b, u); ep (member m) outranks every neighbour
      const int lf = min(f, m - u), lb = min(b, u);
      const uint32_t nbf = ((1u << lf) - 1u) << 5, nbb = ((1u << lb) - 1u) << (5 - lb);
      const uint32_t epb = (m - u >= 1 && m - u <= 5) ? 1u << (4 + m - u) : 0u;
      uint32_t gt = 0, eq = 0;
#pragma unroll
      for (int d = 1; d <= 5; ++d) {
        gt |= (cv[5 + d] > vu ? 1u : 0u) << (4 + d);
        eq |= (!(cv[5 + d] < vu || cv[5 + d] > vu) ? 1u : 0u) << (4 + d);  // equal or NaN
        gt |= (cv[5 - d] > vu ? 1u : 0u) << (5 - d);
        eq |= (!(cv[5 - d] < vu || cv[5 - d] > vu) ? 1u : 0u) << (5 - d);
      }
      const uint32_t notep = u != m ? ~0u : 0u;
      const uint32_t nb = nbf | nbb;
      const uint32_t hc = ((gt | epb) & nbf) | (gt & nbb & notep);
      S.cm[u] = hc | (nb << 10) | ((uint32_t)f << 20) | ((uint32_t)b << 24);
      return ((eq & ~epb & nbf) | (eq & nbb & notep)) != 0u;
    };
    const bool seg_full = a.surf_full || (a.carry && sp <= 9);  // the whole surf walk is observable
    const bool cm_sparse = !seg_full && !has_stale;
    bool direct = !has_stale;
#ifdef FBR_FEAT_SKIP_CM
    if (direct) {
      for (int u = tid; u <= m; u += NT) S.cm[u] = 0u;
      __syncthreads();
    }
    if (false) {
#else
    if (direct) {
#endif
      bool tf = false;
      // Batch jobs need cm only for the corner candidates and the surf window [m - 63, m] (none
      // for the surf walk of the ring's last segment): the members are listed in region B (free
      // until the corner walk) and only those are computed; the rest follow in the rare case the
      // surf window falls back to the whole walk (cm_rest below).
      int nlist = m + 1;
      if (cm_sparse) {
        uint16_t* list = (uint16_t*)S.rb;
        if (wv == 0) {
          int cnt = 0;
          const int wlo_u = j == lastj ? m + 1 : max(0, m - (kSurfWindow - 1));
          for (int k0 = 0; k0 <= m; k0 += 64) {
            const int u = k0 + lane;
            bool need = false;
            if (u <= m) {
              const int li = sp + u - S.wlo;
              need = u >= wlo_u || (!S.picked.get(li) && S.edgec.get(li));
            }
            const uint64_t bm = __ballot(need);
            if (need) list[cnt + __popcll(bm & ((1ull << lane) - 1ull))] = (uint16_t)u;
            cnt += __popcll(bm);
          }
          if (lane == 0) S.tmask[15] = (uint64_t)cnt;
        }
        if constexpr (NWV == 1) wsync();
        else __syncthreads();
        nlist = (int)S.tmask[15];
      }
      for (int k0 = 64 * wv; k0 < nlist; k0 += NT) {
        if (cm_sparse) {
          const int k = k0 + lane;
          if (k < nlist) tf |= cm_member(((const uint16_t*)S.rb)[k]);
        } else {
          const int u = k0 + lane;
          if (u <= m) tf |= cm_member(u);
        }
      }
      if constexpr (NWV == 1) {
        direct = !__any(tf);
        wsync();
      } else {
        __syncthreads();
        direct = !__syncthreads_or(tf);
      }
      FBR_STAMP(10);
    }
    if (wv == 0) {  // the walks: wave 0 alone (helper waves wait at the segment's closing barrier)
    if (!direct) sorted_order();
    FBR_STAMP(3);
    if (has_stale) {
      SmoothEntry* ent = (SmoothEntry*)S.rb;  // the walk's entries in LDS (region B is free here)
      for (int k = lane; k <= m; k += 64) ent[k] = S.seg[k];
      wsync();
      // cm is unused on this path: it holds the entries' walk info; the taken-corner list goes
      // after the entries in region B
      if (!stale_walks_fast(S, slen, ent, a, m, CL, corner_out, corner_cnt, S.cm,
                               (int32_t*)(ent + segcap), lane)) {
        if (lane == 0) serial_walks(S, slen, ent, a, job, m, CL, corner_out, corner_cnt);
        corner_cnt = __shfl(corner_cnt, 0);
        wsync();
      }
    } else {
      // -- corner walk --
      uint64_t und[WMAX], tak[WMAX];
      auto corner_walk = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int w = 0; w < WMAX; ++w) {
          const int u = 64 * w + lane;
          bool cand = false;
          if (u <= m) {
            const int li = sp + u - S.wlo;
            cand = !S.picked.get(li) && S.edgec.get(li);
          }
          und[w] = __ballot(cand);
          tak[w] = 0ull;
        }
#ifndef FBR_FEAT_SKIP_CORNER
        greedy_rounds(m, lane, und, tak, [&](int u) { return S.cm[u] & 1023u; }, a, job);
#endif
      };
      corner_walk();
      FBR_STAMP(4);
      int T = 0;
      if (direct) {  // visit order of the taken corners: ep first, then descending curvature
#pragma unroll
        for (int w = 0; w < WMAX; ++w) {
          if ((tak[w] >> lane) & 1ull) {
            const int q = T + __popcll(tak[w] & ((1ull << lane) - 1ull));
            const int u = 64 * w + lane;
            tlu[q] = (uint16_t)u;
            tlv[q] = S.scurv[sp + u - S.wlo - S.sbase];
          }
          T += __popcll(tak[w]);
        }
        wsync();
        bool tf = false;
        for (int c = lane; c < T; c += 64) {
          const int u = tlu[c];
          const float vu = tlv[c];
          int rank = 0;
          for (int c2 = 0; c2 < T; ++c2) {
            const int u2 = tlu[c2];
            const float v2 = tlv[c2];
            if (u2 == m) rank += (u != m);
            else if (u != m && c2 != c) {
              if (v2 > vu) ++rank;
              else if (!(v2 < vu)) tf = true;
            }
          }
          vis[rank] = (uint16_t)u;
        }
        if (__any(tf)) {  // tied taken corners: their order is introsort's
          direct = false;
          wsync();
          sorted_order();
          corner_walk();
        }
        wsync();
        FBR_STAMP(11);
      }
      if (lane < WMAX) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < WMAX; ++w)
          if (w == lane) t = tak[w];
        S.tmask[lane] = t;
      }
      wsync();
      // the first kCornerPerSeg taken corners in visit order are kept (the walk breaks there)
      const int R = direct ? T : m + 1;
      int taken = 0;
      for (int r0 = 0; r0 < R && taken < kCornerPerSeg; r0 += 64) {
        const int rr = r0 + lane;
        int u = -1;
        if (rr < R) u = direct ? (int)vis[rr] : (int)S.sorder[rr == 0 ? m : m - rr];
        const bool acc = u >= 0 && ((S.tmask[u >> 6] >> (u & 63)) & 1ull);
        const uint64_t mk = __ballot(acc);
        const int pos = taken + __popcll(mk & ((1ull << lane) - 1ull));
        if (acc && pos < kCornerPerSeg) {
          corner_out[corner_cnt + pos] = CL[sp + u];
          const int li = sp + u - S.wlo;
          const uint32_t c = S.cm[u];
          atomicOr((unsigned long long*)&S.labpos.w[li >> 6], 1ull << (li & 63));
          or_range(S.picked, li - (int)((c >> 24) & 15u), li + (int)((c >> 20) & 15u));
        }
        taken += __popcll(mk);
      }
      corner_cnt += min(taken, kCornerPerSeg);
      wsync();
      FBR_STAMP(5);
      if constexpr (NWV == 1) prefetch_curv(j + 1);  // scurv is not read again in this segment
      // -- surf walk: ascending, ep last -> higher priority = not higher corner priority --
      // Batch jobs (a.surf_full == 0) need only the walk's picks within reach of ep (they suppress
      // the next segment's first members); the last segment of a ring needs none.  The members of
      // the window [ulo, m] are resolved with the candidates just left of it frozen (undecided);
      // if a member within reach of ep stays undecided (its chain of higher-priority conflicts
      // leaves the window), the whole walk runs.
      const bool bnd = !seg_full;
      const int ulo = bnd ? max(0, m - (kSurfWindow - 1)) : 0;
      auto surf_cand = [&](bool window) __attribute__((always_inline)) {
#pragma unroll
        for (int w = 0; w < WMAX; ++w) {
          const int u = 64 * w + lane;
          bool cand = false;
          if (u <= m && (!window || u >= ulo - 5)) {
            const int li = sp + u - S.wlo;
            cand = !S.picked.get(li) && S.surfc.get(li);
          }
          und[w] = __ballot(cand);
          tak[w] = 0ull;
        }
      };
      auto surf_cm = [&](int u) {
        const uint32_t c = S.cm[u];
        return ((c >> 10) & 1023u) & ~(c & 1023u);
      };
      if (bnd && j == lastj) {  // the ring's last segment: no surf pick of it is observable
#pragma unroll
        for (int w = 0; w < WMAX; ++w) tak[w] = 0ull;
      } else {
        surf_cand(bnd && ulo > 0);
#ifndef FBR_FEAT_SKIP_SURF
        if (bnd && ulo > 0) {
          uint64_t frz[WMAX];
#pragma unroll
          for (int w = 0; w < WMAX; ++w) {
            const int u = 64 * w + lane;
            frz[w] = und[w] & __ballot(u < ulo);
          }
          greedy_rounds(m, lane, und, tak, surf_cm, a, job, frz);
          // every candidate within reach of ep decided?
          bool open = false;
#pragma unroll
          for (int w = 0; w < WMAX; ++w) {
            const int u = 64 * w + lane;
            open |= u >= m - 4 && u <= m && ((und[w] >> lane) & 1ull) && !((frz[w] >> lane) & 1ull);
          }
          if (__any(open)) {
            if (direct) {  // cm was computed for the listed members only: all of them now
              bool tf2 = false;
              for (int u = lane; u <= m; u += 64) tf2 |= cm_member(u);
              wsync();
              if (__any(tf2)) sorted_order();  // a relevant tie: introsort's order for the whole walk
            }
            surf_cand(false);
            greedy_rounds(m, lane, und, tak, surf_cm, a, job);
          }
        } else {
          greedy_rounds(m, lane, und, tak, surf_cm, a, job);
        }
#endif
      }
      FBR_STAMP(6);
#pragma unroll
      for (int w = 0; w < WMAX; ++w) {
        const int u = 64 * w + lane;
        if (u <= m && ((tak[w] >> lane) & 1ull)) {
          const int li = sp + u - S.wlo;
          const uint32_t c = S.cm[u];
          atomicOr((unsigned long long*)&S.labneg.w[li >> 6], 1ull << (li & 63));
          or_range(S.picked, li - (int)((c >> 24) & 15u), li + (int)((c >> 20) & 15u));
        }
      }
      pf_seg = pf_next;
      if (pf_seg >= 0) {
#pragma unroll
        for (int q = 0; q < kCq; ++q)
          if (64 * q + lane < pf_len) S.scurv[64 * q + lane] = cpf[q];
      }
      wsync();
    }
    FBR_STAMP(7);
    // surf candidates (label <= 0 in [sp, ep], :279-284) are selected by the per-ring VoxelGrid
    // straight from the label mask (k_voxel.hip, k_voxel_ring)
    FBR_STAMP(8);
    }  // wave 0
    if constexpr (NWV > 1) __syncthreads();
  }
  // ---- outputs ----
  if constexpr (NWV > 1) __syncthreads();
  int8_t* LB = a.label + job * HW;
  for (int k = max(cb, 0) + tid; k < ca; k += NT) {
    const int li = k - S.wlo;
    const int8_t lab = S.labpos.get(li) ? 1 : (S.labneg.get(li) ? -1 : 0);
    if (k >= 5 && k < n - 5) LB[k] = lab;      // cloudLabel reset range (:126)
    else if (k < 5 && (lab != 0 || a.fresh)) LB[k] = lab;  // stale slots keep earlier values
  }
  if (cb <= 0 && tid < 5 && tid < S.L) st->picked04[tid] = S.picked.get(tid) ? 1 : 0;
  if (tid == 0) a.corner_cnt[slot] = corner_cnt;
#ifdef FBR_FEAT_STAMPS
  FBR_STAMP(9);
  if (tid == 0 && a.stamps)
    for (int i = 0; i < 12; ++i) a.stamps[(int64_t)slot * 12 + i] = stamp_acc[i];
#endif
}

size_t features_lds_bytes(const FeatArgs& a, int nwv) {
  const size_t region_b = std::max<size_t>((size_t)nwv * kWinBytes, (size_t)8 * a.segcap + sizeof(int32_t) * kCornerPerSeg);
  return (size_t)((a.segcap + 19) & ~3) * sizeof(float) + (size_t)9 * a.nwcap * sizeof(uint64_t) + sizeof(uint64_t) * 16 +
         sizeof(SortFrame) * kSortStack + sizeof(uint32_t) * a.segcap + 16 + region_b;
}

size_t features_gslot_bytes(const FeatArgs& a) {
  const size_t b = sizeof(uint64_t) * a.kseg + 2 * sizeof(SmoothEntry) * a.segcap + 2 * sizeof(uint16_t) * a.segcap +
                   16 + sizeof(float) * a.lcap;  // + the ring window's curvature
  return (b + 255) & ~(size_t)255;
}

// Waves per ring: FBR_FEAT_WAVES (1, 2 or 4) or, by default, 4 while a launch has at most 2048
// rings (<= 2 rings per SIMD: single scans, small sub-batches), 1 above.
int feature_waves(int rings) {
  static const int forced = [] {
    const char* e = std::getenv("FBR_FEAT_WAVES");
    const int v = e ? std::atoi(e) : 0;
    return v >= 4 ? 4 : v >= 2 ? 2 : v == 1 ? 1 : 0;
  }();
  if (forced) return forced;
  return rings <= 2048 ? 4 : 1;
}

void launch_features(hipStream_t s, const FeatArgs& a) {
  const int nwv = feature_waves(a.B * a.H);
  const dim3 grid(a.B * a.H);
  if (nwv == 1 && a.segcap <= 5 * 64 && a.kseg <= 4 * 128) {
    // Horizon_SCAN <= 1872 (C1 / C2): five mask words, twelve SGPRs of und / tak / frz less
    fbr_launch((k_features<5, 4, 1>), grid, dim3(64), features_lds_bytes(a, 1), s, a);
  } else if (a.segcap <= 6 * 64 && a.kseg <= 4 * 128) {
    if (nwv == 4)
      fbr_launch((k_features<6, 4, 4>), grid, dim3(256), features_lds_bytes(a, 4), s, a);
    else if (nwv == 2)
      fbr_launch((k_features<6, 4, 2>), grid, dim3(128), features_lds_bytes(a, 2), s, a);
    else
      fbr_launch((k_features<6, 4, 1>), grid, dim3(64), features_lds_bytes(a, 1), s, a);
  } else {
    if (nwv > 1)
      fbr_launch((k_features<12, 8, 4>), grid, dim3(256), features_lds_bytes(a, 4), s, a);
    else
      fbr_launch((k_features<12, 8, 1>), grid, dim3(64), features_lds_bytes(a, 1), s, a);
  }
}

}  // namespace fbr
