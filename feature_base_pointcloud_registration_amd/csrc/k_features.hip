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
//   - curvature: the reference's left-to-right f32 sum, no FMA;
//   - occlusion: the sequential loop only ever writes 1s, so each cell's final value is the OR of
//     the marks that cover it — computed in parallel;
//   - sort: parallel stable rank sort (equal to std::sort when no two curvatures tie and none is
//     NaN); segments with ties fall back to the exact libstdc++ introsort emulation (fbr_sort.h);
//   - picks: the greedy corner/surf walks are inherently ordered; lane 0 walks the sorted segment
//     with early exit once the sorted curvature crosses the threshold (exact: the remaining
//     entries fail the same test).
// Outputs: label (the feature mask), per-ring corner slots in visit order, per-ring surf
// candidates (label <= 0, index order) for the per-ring VoxelGrid (k_voxel.hip).
#include "fbr_common.h"
#include "fbr_kernels.h"
#include "fbr_sort.h"

namespace fbr {

namespace {
constexpr uint8_t kPicked = 1;
constexpr uint8_t kLabPos = 2;   // label == 1
constexpr uint8_t kLabNeg = 4;   // label == -1
constexpr uint8_t kOccA = 8;     // depth1 - depth2 > 0.3 at j (marks j-5..j)
constexpr uint8_t kOccB = 16;    // depth2 - depth1 > 0.3 at j (marks j+1..j+6)
constexpr uint8_t kOccC = 32;    // parallel beam at j
constexpr int kColM2 = 1 << 30;  // pointColInd[-2]: glibc chunk-size word (large)
}  // namespace

struct FeatLds {
  int wlo, L;
  float* r;        // ranges, later reused by nothing
  int16_t* col;    // column index
  float* curv;
  uint8_t* fl;     // picked / label / occlusion bits
  SmoothEntry* seg;
  SmoothEntry* srt;
};

__device__ __forceinline__ int col_at(const FeatLds& S, int k) {
  if (k == -1) return 0;
  if (k == -2) return kColM2;
  return S.col[k - S.wlo];
}

// Neighbour suppression after a pick (featureExtraction.h:227-240 / 259-274).
__device__ __forceinline__ void suppress(const FeatLds& S, int ind) {
  for (int l = 1; l <= 5; l++) {
    int cd = abs(col_at(S, ind + l) - col_at(S, ind + l - 1));
    if (cd > 10) break;
    S.fl[ind + l - S.wlo] |= kPicked;
  }
  for (int l = -1; l >= -5; l--) {
    int cd = abs(col_at(S, ind + l) - col_at(S, ind + l + 1));
    if (cd > 10) break;
    int k = ind + l;
    if (k >= 0) S.fl[k - S.wlo] |= kPicked;  // k == -1: write lands outside the array (scratch)
  }
}

__global__ void __launch_bounds__(64)
k_features(FeatArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int H = a.H, W = a.W;
  const int job = blockIdx.x / H, ring = blockIdx.x % H, lane = threadIdx.x;
  const int64_t HW = (int64_t)H * W;
  const int n = a.nvalid[job];
  const int s = a.start_ring[job * H + ring], e = a.end_ring[job * H + ring];
  const int cb = s - 4, ca = e + 6;  // this ring's points [cb, ca)
  const int slot = job * H + ring;
  if (ca <= cb) {
    if (lane == 0) {
      a.corner_cnt[slot] = 0;
      a.cand_cnt[slot] = 0;
    }
    return;
  }
  FeatLds S;
  S.wlo = max(s - 12, 0);
  const int whi = min(e + 11, n);
  S.L = whi - S.wlo;
  const int Lcap = a.lcap;
  unsigned char* p = smem;
  S.r = (float*)p;                 p += sizeof(float) * Lcap;
  S.curv = (float*)p;              p += sizeof(float) * Lcap;
  S.seg = (SmoothEntry*)p;         p += sizeof(SmoothEntry) * a.segcap;
  S.srt = (SmoothEntry*)p;         p += sizeof(SmoothEntry) * a.segcap;
  S.col = (int16_t*)p;             p += sizeof(int16_t) * Lcap;
  S.fl = (uint8_t*)p;
  if (S.L > Lcap) {
    if (lane == 0) atomicOr(&a.err[job], 1);
    return;
  }
  const float* R = a.range + job * HW;
  const int32_t* C = a.col + job * HW;
  const float4* CL = a.cloud + job * HW;
  StreamState* st = a.stream + job;
  for (int i = lane; i < S.L; i += 64) {
    S.r[i] = R[S.wlo + i];
    S.col[i] = (int16_t)C[S.wlo + i];
    S.fl[i] = 0;
    S.curv[i] = 0.0f;
  }
  __syncthreads();
  // ---- markOccludedPoints conditions per j in [5, n-6) (featureExtraction.h:140-175) ----
  for (int i = lane; i < S.L; i += 64) {
    const int j = S.wlo + i;
    if (j < 5 || j >= n - 6 || i == 0 || i + 1 >= S.L) continue;
    uint8_t f = 0;
    const float depth1 = S.r[i], depth2 = S.r[i + 1];
    const int columnDiff = abs((int)S.col[i + 1] - (int)S.col[i]);
    if (columnDiff < 10) {
      if ((double)(depth1 - depth2) > 0.3) f |= kOccA;
      else if ((double)(depth2 - depth1) > 0.3) f |= kOccB;
    }
    const float diff1 = fabsf(S.r[i - 1] - S.r[i]);
    const float diff2 = fabsf(S.r[i + 1] - S.r[i]);
    if ((double)diff1 > 0.02 * (double)S.r[i] && (double)diff2 > 0.02 * (double)S.r[i]) f |= kOccC;
    S.fl[i] = f;
  }
  __syncthreads();
  // ---- cloudNeighborPicked after smoothness reset + occlusion marks; curvature ----
  for (int i = lane; i < S.L; i += 64) {
    const int k = S.wlo + i;
    bool picked = (k < 5) && st->picked04[k] != 0;
    for (int j = k; j <= k + 5 && !picked; ++j)
      if (j - S.wlo < S.L && (S.fl[j - S.wlo] & kOccA)) picked = true;
    for (int j = k - 6; j <= k - 1 && !picked; ++j)
      if (j >= S.wlo && (S.fl[j - S.wlo] & kOccB)) picked = true;
    if (S.fl[i] & kOccC) picked = true;
    // Only this lane writes byte i and the occlusion bits other lanes read are left unchanged.
    if (picked) S.fl[i] |= kPicked;
    if (k >= 5 && k < n - 5 && i >= 5 && i + 5 < S.L) {  // calculateSmoothness (:113-122), f32 left-to-right
      float d = S.r[i - 5] + S.r[i - 4] + S.r[i - 3] + S.r[i - 2] + S.r[i - 1] - S.r[i] * 10.0f + S.r[i + 1] +
                S.r[i + 2] + S.r[i + 3] + S.r[i + 4] + S.r[i + 5];
      S.curv[i] = d * d;
    }
  }
  __syncthreads();

  // ---- extractFeatures (:188-285) ----
  const float edgeThr = a.edge_thr, surfThr = a.surf_thr;
  int corner_cnt = 0, cand_cnt = 0;
  float4* corner_out = a.corner_slot + (int64_t)slot * kCornerPerRing;
  float4* cand_out = a.cand + (int64_t)slot * W;
  for (int j = 0; j < 6; j++) {
    const int sp = (s * (6 - j) + e * j) / 6;
    const int ep = (s * (5 - j) + e * (j + 1)) / 6 - 1;
    if (sp >= ep) continue;
    const int m = ep - sp;
    if (m + 1 > a.segcap) {
      if (lane == 0) atomicOr(&a.err[job], 2);
      return;
    }
    const bool has_stale = (sp <= 4 && 4 < ep);
    for (int t = lane; t <= m; t += 64) {
      const int pos = sp + t;
      SmoothEntry en;
      if (pos == 4) { en.v = st->smooth4_value; en.ind = st->smooth4_ind; }
      else { en.v = S.curv[pos - S.wlo]; en.ind = pos; }
      S.seg[t] = en;
    }
    __syncthreads();
    // parallel stable rank sort of seg[0..m)
    bool tie = false, nan = false;
    for (int t = lane; t < m; t += 64) {
      const float v = S.seg[t].v;
      int rank = 0;
      for (int u = 0; u < m; ++u) {
        const float w = S.seg[u].v;
        rank += (w < v) || (w == v && u < t);
        tie |= (w == v) && (u != t);
      }
      nan |= (v != v);
      S.srt[min(rank, m - 1)] = S.seg[t];
    }
    const bool any_tie = __any(tie || nan);
    const bool any_nan = __any(nan);
    __syncthreads();
    if (lane == 0) {
      if (any_tie) {
        for (int t = 0; t < m; ++t) S.srt[t] = S.seg[t];
        std_sort_emul(S.srt, m);
      }
      S.srt[m] = S.seg[m];  // cloudSmoothness[ep] is never sorted (:203)
      if (has_stale) {      // the slot left at position 4 is the next scan's stale entry
        st->smooth4_value = S.srt[4 - sp].v;
        st->smooth4_ind = S.srt[4 - sp].ind;
      }
      const bool fast = !has_stale && !any_nan;
      // corner picks, k = ep .. sp (:208-242)
      int largestPickedNum = 0;
      for (int k = m; k >= 0; k--) {
        const SmoothEntry en = S.srt[k];
        if (fast && k < m && !(en.v > edgeThr)) break;
        const int ind = en.ind;
        const int li = ind - S.wlo;
        if (li < 0 || li + 5 >= S.L) { atomicOr(&a.err[job], 4); break; }
        if ((S.fl[li] & kPicked) == 0 && S.curv[li] > edgeThr) {
          largestPickedNum++;
          if (largestPickedNum <= kCornerPerSeg) {
            S.fl[li] |= kLabPos;
            corner_out[corner_cnt++] = CL[ind];
          } else {
            break;
          }
          S.fl[li] |= kPicked;
          suppress(S, ind);
        }
      }
      // surf picks, k = sp .. ep (:245-276); ep handled last
      for (int k = 0; k <= m; k++) {
        if (k < m && fast && !(S.srt[k].v < surfThr)) k = m;  // rest of the sorted part fails
        const SmoothEntry en = S.srt[k];
        const int ind = en.ind;
        const int li = ind - S.wlo;
        if (li < 0 || li + 5 >= S.L) { atomicOr(&a.err[job], 4); break; }
        if ((S.fl[li] & kPicked) == 0 && S.curv[li] < surfThr) {
          S.fl[li] = (uint8_t)((S.fl[li] & ~kLabPos) | kLabNeg | kPicked);
          suppress(S, ind);
        }
      }
    }
    __syncthreads();
    // surf candidates: label[k] <= 0 for k in [sp, ep] (:279-284), index order
    for (int t0 = 0; t0 <= m; t0 += 64) {
      const int t = t0 + lane;
      const bool c = t <= m && !(S.fl[sp + t - S.wlo] & kLabPos);
      const uint64_t mk = __ballot(c);
      if (c) cand_out[cand_cnt + __popcll(mk & ((1ull << lane) - 1ull))] = CL[sp + t];
      cand_cnt += __popcll(mk);
    }
    __syncthreads();
  }
  corner_cnt = __shfl(corner_cnt, 0);
  // ---- outputs ----
  int8_t* LB = a.label + job * HW;
  for (int k = max(cb, 0) + lane; k < ca; k += 64) {
    const uint8_t f = S.fl[k - S.wlo];
    const int8_t lab = (f & kLabPos) ? 1 : ((f & kLabNeg) ? -1 : 0);
    if (k >= 5 && k < n - 5) LB[k] = lab;      // cloudLabel reset range (:126)
    else if (k < 5 && lab != 0) LB[k] = lab;   // stale slots keep earlier values
  }
  if (cb <= 0 && lane < 5 && lane < S.L) st->picked04[lane] = (int8_t)(S.fl[lane - S.wlo] & kPicked);
  if (lane == 0) {
    a.corner_cnt[slot] = corner_cnt;
    a.cand_cnt[slot] = cand_cnt;
  }
}

void launch_features(hipStream_t s, const FeatArgs& a) {
  size_t lds = (size_t)a.lcap * (4 + 4 + 2 + 1) + (size_t)a.segcap * 2 * sizeof(SmoothEntry) + 64;
  hipLaunchKernelGGL(k_features, dim3(a.B * a.H), dim3(64), lds, s, a);
}

}  // namespace fbr
