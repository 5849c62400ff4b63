// fbr_gn.h — device side of the Gauss-Newton correspondence search (A13-A15), shared by
// k_register.hip (init, residual, solve, finalize) and the k_knn_*.hip translation units, which
// instantiate the kNN kernels per cell radius R and fused flag (the instantiations compile in
// parallel; one file holding all of them took ~8 minutes).  See k_register.hip for the design
// notes and reference citations (mapOptmization.h:1002-1243, :1403-1442).
#pragma once
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "fbr_common.h"
#include "fbr_imu.h"
#include "fbr_kernels.h"
#include "fbr_solvers.h"

namespace fbr {

namespace {
constexpr int kResThreads = 256;
constexpr int kSolveThreads = 128;  // k_gn_solve: wave 0 sums + solves, wave 1 the iteration-0 degeneracy
constexpr int kPartial = 32;  // doubles per item partial: 21 AtA upper + 6 AtB + count
}
// The 5 nearest as sorted 64-bit keys (float bits of d2) << 32 | map index: d2 >= +0, so the
// unsigned key order is exactly FLANN's (d2, index) order.  A key is built from a scanned point
// without any instruction (hi = the distance register, lo = the w bit pattern).  Empty slots hold
// kKnnEmpty = (bits(1.0f), 0): a point is only inserted with d2 < 1.0 (:1027, :1154).
constexpr unsigned long long kKnnEmpty = (unsigned long long)0x3f800000u << 32;
constexpr float kBelowOne = 0.99999994f;  // nextafterf(1.0f, 0.0f)

struct Knn5 {
  unsigned long long k[5];
};

__device__ __forceinline__ float knn_d(unsigned long long k) { return __int_as_float((int)(k >> 32)); }
__device__ __forceinline__ int knn_id(unsigned long long k) { return (int)(unsigned)k; }

// The sorted insertion of a key into the 5-NN list as v_min_f64 / v_max_f64 over the keys read as
// doubles: a key's high word is the
// bits of a float d2 >= +0 (at most +inf = 0x7f800000 for a point outside the crop box), so every
// key is a non-negative finite double (a subnormal when d2 = 0; the kernels keep f64 denormals,
// amdhsa_float_denorm_mode_16_64 3) and double order is the key's unsigned order.  9 v_min_f64 /
// v_max_f64 instead of 5 64-bit compares, 20 selects and the wait states between them.  Written as
// inline asm: the compiler's fmin / fmax quiet-NaN canonicalisation of the loop-carried keys would
// add a v_max_f64 per slot.
// The slots do not chain: with k sorted, the new k[t] is min(k[t], max(k[t-1], x)) (x below k[t-1]
// shifts k[t-1] up, else x or k[t] stays), so every slot is two operations deep, visited from the top
// so each max reads the old k[t-1].
__device__ __forceinline__ void knn_insert_f64(Knn5& r, unsigned long long xk) {
  const double x = __longlong_as_double((long long)xk);
  double k[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) k[t] = __longlong_as_double((long long)r.k[t]);
#pragma unroll
  for (int t = 4; t > 0; --t) {
    double m;
    asm("v_max_f64 %0, %1, %2" : "=v"(m) : "v"(k[t - 1]), "v"(x));
    asm("v_min_f64 %0, %0, %1" : "+v"(k[t]) : "v"(m));
  }
  asm("v_min_f64 %0, %0, %1" : "+v"(k[0]) : "v"(x));
#pragma unroll
  for (int t = 0; t < 5; ++t) r.k[t] = (unsigned long long)__double_as_longlong(k[t]);
}
// Branch-free sorted insertion with selects: the "less than slot t" flags are monotone over t, so
// every slot takes its own key, its left neighbour's, or the new one (5 compares + 20 selects).
__device__ __forceinline__ void knn_insert_sel(Knn5& r, unsigned long long x) {
  bool lt[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) lt[t] = x < r.k[t];
#pragma unroll
  for (int t = 4; t > 0; --t) r.k[t] = lt[t - 1] ? r.k[t - 1] : (lt[t] ? x : r.k[t]);  // lt[t-1] implies lt[t]
  r.k[0] = lt[0] ? x : r.k[0];
}
// Which form a kernel uses (round 5, profiles/r05aj_*, r05ak_knn_f64_insert_ab.txt): the f64 form
// for the 1 m (C2) and 0.25 m cells, where it took gn_knn 2.29 -> 2.00 ms per B = 1024 step
// (flat dispatch VALU 1.745e8 -> 1.342e8) and C2 109.5k -> 112-113k scans/s; the selects for the
// 0.5 m cells (C3, C5), whose per-row kernel at 85 -> 90 VGPRs lost 2.5 % on C3 with the f64 form
// (C5 gained 1.5 %).  FBR_KNN_F64_R2=1 builds the f64 form there too.
#ifndef FBR_KNN_F64_R2
#define FBR_KNN_F64_R2 0
#endif
template <int R>
__device__ __forceinline__ void knn_insert(Knn5& r, unsigned long long x) {
  if constexpr (R != 2 || FBR_KNN_F64_R2) knn_insert_f64(r, x);
  else knn_insert_sel(r, x);
}

// pcl::CropBox's inclusive test (p outside [bmin, bmax] on some axis) as one compare: for finite
// floats b - x > 0 exactly when x < b (the difference of distinct floats is never rounded to 0,
// denormals are kept), so "outside" is the largest of the six excesses being positive; 6 subtractions
// and 2 three-way maxima instead of 6 compares whose masks the compiler combined in 16-bit registers.
__device__ __forceinline__ bool crop_out(const float4& p, float bx0, float by0, float bz0, float bx1, float by1,
                                         float bz1) {
  const float ex = fmaxf(fmaxf(bx0 - p.x, p.x - bx1), fmaxf(by0 - p.y, p.y - by1));
  return fmaxf(ex, fmaxf(bz0 - p.z, p.z - bz1)) > 0.0f;
}

// Lower bound of |q - p| along one axis for a point p in the cell at offset o from q's cell
// (cells are [k*c, (k+1)*c) with c a power of two, so every edge is exact).  Rounding is
// monotone, so fl(edge - q) <= |fl(q - p)| and the bound composed in the distance's own
// operation order never exceeds the distance computed for any point of that cell.
__device__ __forceinline__ float axis_lb(float q, float fcell, int o, float c) {
  if (o == 0) return 0.0f;
  if (o > 0) return (fcell + (float)o) * c - q;
  return q - (fcell + (float)(o + 1)) * c;
}

__device__ __forceinline__ int rank_offset(int k, int s) { return k == 0 ? 0 : ((k & 1) ? s * ((k + 1) >> 1) : -s * (k >> 1)); }

// Sparse grids (k_grid.hip): the chunk of (z, y, x / kChunkX), or -1.  The table is at most half
// full, so a free slot ends every probe sequence.
__device__ __forceinline__ int chunk_find(const MapGrid& m, int z, int y, int xc) {
  const unsigned long long key = chunk_key(z, y, xc);
  uint32_t h = chunk_hash(key) & m.g.hmask;
  for (uint32_t probe = 0; probe <= m.g.hmask; ++probe) {
    const unsigned long long k = m.hkeys[h];
    if (k == key) return m.hvals[h];
    if (k == kChunkEmpty) break;
    h = (h + 1) & m.g.hmask;
  }
  return -1;
}

// Point range [b, e) of the cells x0..x1 (x1 - x0 < 2 * kChunkX) of row (y, z).  The two chunks
// are adjacent in the (z, y, x) sort, so their points form one contiguous range.
template <bool kSparse>
__device__ __forceinline__ bool row_range(const MapGrid& m, int y, int z, int x0, int x1, int& b, int& e) {
  if constexpr (!kSparse) {
    const int rowbase = (z * m.g.dims[1] + y) * m.g.dims[0];
    b = m.cell_start[rowbase + x0];
    e = m.cell_start[rowbase + x1 + 1];
    return true;
  } else {
    const int ca = x0 / kChunkX, cb = x1 / kChunkX;
    const int ia = chunk_find(m, z, y, ca);
    const int ib = cb == ca ? ia : chunk_find(m, z, y, cb);
    if (ia < 0 && ib < 0) return false;
    constexpr int S = kChunkX + 1;
    b = ia >= 0 ? m.cell_start[ia * S + (x0 - ca * kChunkX)] : m.cell_start[ib * S];
    e = ib >= 0 ? m.cell_start[ib * S + (x1 - cb * kChunkX) + 1] : m.cell_start[ia * S + kChunkX];
    return true;
  }
}

#ifdef FBR_KNN_STATS
// Diagnostic builds only (tools/knn_stats.py): [queries, rows considered, rows scanned, points
// scanned, points inserted, accepted queries, corner queries, wave iterations of the point loop,
// warm-started queries, queries whose neighbours equal the previous iteration's], accumulated into
// GnArgs::knn_stats (one device buffer for every kNN translation unit); then, for the flat walk,
// [flat queries, points within the static cut], a histogram of that count per flat query (bins
// 0..31, 32..63, >= 64) at [12, 46), [points scanned, wave trips] at [46, 48)
#define FBR_KS(i, v) ks[i] += (v)
#else
#define FBR_KS(i, v) \
  do {               \
  } while (0)
#endif

// Exact kNN-5 among map points inside the crop box with d2 < 1.0, ordered by (d2, map index):
// the neighbour set FLANN's exact search returns on the cropped cloud whenever the reference
// keeps the correspondence (pointSearchSqDis[4] < 1.0, :1027/:1154).  R = cells per side covering
// radius 1 (compile time: the row loop is fully unrolled).  Cell rows (y,z) are visited in
// near-side-first rank order; a row, and the cells of a row, are skipped once their lower-bound
// distance exceeds the current 5th distance or reaches 1.0.  Rows entirely inside the crop box
// skip the per-point box test.
// `bound` is an upper bound of the 5th-neighbour distance known before the search (the largest
// distance to the previous iteration's 5 neighbours, 5 distinct candidates of the same crop box):
// cells whose lower bound exceeds it cannot hold any of the 5 nearest, ties included, so they are
// pruned from the start instead of only once 5 points have been inserted.
// kFlat: the rows are pruned once up front with `bound` (the warm start, tight from iteration 1
// on) and their point ranges queued in LDS (`rows`, stride kResThreads); one loop then walks a
// lane's queued points across rows.  A wave then runs for its longest lane's total instead of the
// sum over rows of each row's longest lane (lanes of a wave scan different rows: the per-row loop
// kept ~30 % of the lanes busy).  Pruning with a larger cut only scans more cells, and the 5-NN
// list is a function of the scanned set, so both forms give the same neighbours.
// LPQ > 1 (wide mode, small launches): LPQ lanes share a query and lane `sub` scans the points of
// absolute map index = sub (mod LPQ) (knn5_merge combines the lists).  A lane prunes with its own
// 5th distance, which is never below the merged one (its list holds the 5 nearest of a subset),
// so every point of the merged 5 nearest is still scanned by its lane.
template <int R, int RX, bool kFlat = false, bool kSparse = false, int LPQ = 1>
__device__ void knn5_grid(const MapGrid& m, float qx, float qy, float qz, const float* bmin, const float* bmax,
                          float bound, Knn5& r, unsigned* ks, int2* rows = nullptr, int sub = 0) {
  constexpr int K = 2 * R + 1;  // rows per side in y and z; RX = cells per side along x
#pragma unroll
  for (int t = 0; t < 5; ++t) r.k[t] = kKnnEmpty;
  const float inv = m.g.inv_cell, c = 1.0f / inv, invx = m.g.inv_x, cxs = 1.0f / invx;
  const float sx = qx * invx, sy = qy * inv, sz = qz * inv;
  const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
  if (!(fabsf(fx) < 1e7f && fabsf(fy) < 1e7f && fabsf(fz) < 1e7f)) return;
  const int cx = (int)fx - (int)m.g.origin[0], cy = (int)fy - (int)m.g.origin[1], cz = (int)fz - (int)m.g.origin[2];
  const int X = m.g.dims[0], Y = m.g.dims[1], Z = m.g.dims[2];
  if (cx < -RX || cy < -R || cz < -R || cx >= X + RX || cy >= Y + R || cz >= Z + R) return;
  const int sgy = (sy - fy) >= 0.5f ? 1 : -1, sgz = (sz - fz) >= 0.5f ? 1 : -1;
  // squared per-axis lower bounds: y/z by visit rank, x by offset (negative / positive side)
  float ly2[K], lz2[K], lxm2[RX + 1], lxp2[RX + 1];
  int oyk[K], ozk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    // flat queue: rows in one fixed order for every lane (the queued set does not depend on it), so
    // lanes of a wave that share rows walk them in step
    oyk[k] = kFlat ? k - R : rank_offset(k, sgy);
    ozk[k] = kFlat ? k - R : rank_offset(k, sgz);
    const float ly = axis_lb(qy, fy, oyk[k], c), lz = axis_lb(qz, fz, ozk[k], c);
    ly2[k] = ly * ly;
    lz2[k] = lz * lz;
  }
#pragma unroll
  for (int o = 1; o <= RX; ++o) {
    const float a = axis_lb(qx, fx, -o, cxs), b = axis_lb(qx, fx, o, cxs);
    lxm2[o] = a * a;
    lxp2[o] = b * b;
  }
  // the crop box in registers (per job: wave-uniform)
  const float bx0 = bmin[0], by0 = bmin[1], bz0 = bmin[2], bx1 = bmax[0], by1 = bmax[1], bz1 = bmax[2];
  const float xlo = (fx - (float)RX) * cxs, xhi = (fx + (float)(RX + 1)) * cxs;  // row x extent (max)
  const bool xin = xlo >= bx0 && xhi <= bx1;
  int nrow = 0;  // kFlat: rows queued
  int total = 0;  // kFlat: points queued
#pragma unroll
  for (int ksum = 0; ksum <= 2 * (K - 1); ++ksum) {
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const int kz = ksum - ky;
      if (kz < 0 || kz >= K) continue;  // compile time
      const int y = cy + oyk[ky], z = cz + ozk[kz];
      FBR_KS(1, 1);
      float lb = 0.0f;
      lb += ly2[ky];
      lb += lz2[kz];
      // "lb <= cut and lb < 1.0" as one compare: the largest float below 1.0 caps the cut
      const float cut = fminf(fminf(knn_d(r.k[4]), bound), kBelowOne);
      if (y < 0 || y >= Y || z < 0 || z >= Z || lb > cut) continue;
      int xa = 0, xb = 0;
      bool go_a = true, go_b = true;
#pragma unroll
      for (int o = 1; o <= RX; ++o) {
        float ta = 0.0f, tb = 0.0f;
        ta += lxm2[o]; ta += ly2[ky]; ta += lz2[kz];
        tb += lxp2[o]; tb += ly2[ky]; tb += lz2[kz];
        go_a = go_a && !(ta > cut);
        go_b = go_b && !(tb > cut);
        if (go_a) xa = -o;
        if (go_b) xb = o;
      }
      const int x0 = max(cx + xa, 0), x1 = min(cx + xb, X - 1);
      if (x0 > x1) continue;
      int b, e;
      if (!row_range<kSparse>(m, y, z, x0, x1, b, e)) continue;
      FBR_KS(2, 1);
      FBR_KS(3, e - b);
      // the whole row inside the crop box (pcl::CropBox, inclusive) -> no per-point test
      const float ylo = (fy + (float)oyk[ky]) * c, zlo = (fz + (float)ozk[kz]) * c;
      const bool inside = xin & (ylo >= by0) & (ylo + c <= by1) & (zlo >= bz0) & (zlo + c <= bz1);
      if constexpr (kFlat) {
        if (e > b) rows[nrow++ * kResThreads] = make_int2(b, inside ? (int)((unsigned)e | 0x80000000u) : e);
        total += e - b;
        continue;
      }
      // one point load in flight within the row (the row's last point re-requests itself)
      const int i0 = LPQ == 1 ? b : b + ((sub - b) & (LPQ - 1));
      float4 p = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(m.pts) + (uint32_t)(i0 < e ? i0 : b) * 16u);
      for (int i = i0; i < e; i += LPQ) {
        const int nx = i + LPQ < e ? i + LPQ : i;
        const float4 pn = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(m.pts) + (uint32_t)nx * 16u);
        float dist = 0.0f, diff;
        diff = qx - p.x; dist += diff * diff;                            // flann::L2_Simple
        diff = qy - p.y; dist += diff * diff;
        diff = qz - p.z; dist += diff * diff;
        // pcl::CropBox (inclusive) as one mask: a point outside gets d2 = +inf (never inserted);
        // rows inside the box skip the test
        unsigned hi = (unsigned)__float_as_int(dist);
        if (!inside && crop_out(p, bx0, by0, bz0, bx1, by1, bz1)) hi = 0x7f800000u;
        FBR_KS(4, __int_as_float((int)hi) < knn_d(r.k[4]) ? 1 : 0);
#ifdef FBR_KNN_STATS
        if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) ks[7] += 1;  // one per wave iteration
#endif
        knn_insert<R>(r, ((unsigned long long)hi << 32) | (unsigned)__float_as_int(p.w));
        p = pn;
      }
    }
  }
  if constexpr (kFlat) {
    // counted walk: one trip per queued point (the lane's total), the row advance a short branch
    // (a while loop that tests for the next row first: +16 % per dispatch, r04ae).  The row offset
    // is a 32-bit byte offset (maps below 2^28 points): the load takes the SGPR base + VGPR offset
    // form, one shift instead of a 64-bit address per point.
    int2 q = rows[0];  // unread when nothing is queued
    int j = 0, i = q.x, e = q.y & 0x7fffffff;
    bool inside = q.y < 0;
    // one point load in flight: trip t + 1's point is requested before trip t's is tested (the
    // last trip re-requests its own point, so no index runs past a row)
    auto ld = [&](int k) __attribute__((always_inline)) {
      return *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(m.pts) + (uint32_t)k * 16u);
    };
    float4 p = ld(total > 0 ? i : 0);
    for (int t = 0; t < total; ++t) {
      const bool in_cur = inside;
      const int cur = i;
      if (++i == e && t + 1 < total) {  // next queued row (every queued row is non-empty)
        q = rows[++j * kResThreads];
        i = q.x;
        e = q.y & 0x7fffffff;
        inside = q.y < 0;
      }
      const float4 pn = ld(t + 1 < total ? i : cur);
      float dist = 0.0f, diff;
      diff = qx - p.x; dist += diff * diff;  // flann::L2_Simple
      diff = qy - p.y; dist += diff * diff;
      diff = qz - p.z; dist += diff * diff;
      // the distance unconditionally, the box test only on rows that straddle the box: the
      // compiler otherwise sinks the distance under a branch on the test's result
      unsigned hi = (unsigned)__float_as_int(dist);
      if (!in_cur && crop_out(p, bx0, by0, bz0, bx1, by1, bz1)) hi = 0x7f800000u;
      FBR_KS(4, __int_as_float((int)hi) < knn_d(r.k[4]) ? 1 : 0);
      FBR_KS(10, __int_as_float((int)hi) <= fminf(bound, kBelowOne) ? 1 : 0);  // within the static cut
#ifdef FBR_KNN_STATS
      if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) {
        ks[7] += 1;  // one per wave iteration
        ks[11] += 1;
      }
#endif
      knn_insert<R>(r, ((unsigned long long)hi << 32) | (unsigned)__float_as_int(p.w));
      p = pn;
    }
  }
}

// Wide mode: the LPQ lanes of a query (consecutive lanes) exchange their lists in a butterfly and
// each keeps the 5 smallest keys of the union (the lanes scanned disjoint point sets, so keys are
// distinct and the result is the 5 nearest of the whole scanned set).
template <int LPQ>
__device__ __forceinline__ void knn5_merge(Knn5& r) {
#pragma unroll
  for (int off = 1; off < LPQ; off <<= 1) {
    unsigned long long o[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const unsigned lo = __shfl_xor((unsigned)r.k[t], off), hi = __shfl_xor((unsigned)(r.k[t] >> 32), off);
      o[t] = ((unsigned long long)hi << 32) | lo;
    }
#pragma unroll
    for (int t = 0; t < 5; ++t) knn_insert_f64(r, o[t]);
  }
}

// cornerOptimization body (:1016-1121): coefficient row for one corner query, false if rejected.
struct Nbr5 {
  float x[5], y[5], z[5];
};

// The part of a correspondence that depends only on its 5 map neighbours: the corner line (two
// points 0.1 along the principal axis through the mean, after the eigenvalue-ratio gate) or the
// plane (pa, pb, pc, pd after the 0.2 m check).  A query whose kNN returns the same 5 neighbours as
// in the previous Gauss-Newton iteration reuses it (bit-identical: same inputs, same operations);
// only the query-dependent residual below is recomputed.  f[0..5]; false = rejected.
__device__ bool corner_fit(const Nbr5& nn, float* f) {
  float cx = 0, cy = 0, cz = 0;
  for (int j = 0; j < 5; j++) { cx += nn.x[j]; cy += nn.y[j]; cz += nn.z[j]; }
  cx /= 5.0f; cy /= 5.0f; cz /= 5.0f;
  float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
  for (int j = 0; j < 5; j++) {
    const float ax = nn.x[j] - cx, ay = nn.y[j] - cy, az = nn.z[j] - cz;
    a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
    a22 += ay * ay; a23 += ay * az;
    a33 += az * az;
  }
  a11 /= 5.0f; a12 /= 5.0f; a13 /= 5.0f; a22 /= 5.0f; a23 /= 5.0f; a33 /= 5.0f;
  float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
  float D1[3], V1[9];
  jacobi_eigen<3>(A1, D1, V1);
  if (!(D1[0] > 3.0f * D1[1])) return false;
  f[0] = (float)((double)cx + 0.1 * (double)V1[0]);
  f[1] = (float)((double)cy + 0.1 * (double)V1[1]);
  f[2] = (float)((double)cz + 0.1 * (double)V1[2]);
  f[3] = (float)((double)cx - 0.1 * (double)V1[0]);
  f[4] = (float)((double)cy - 0.1 * (double)V1[1]);
  f[5] = (float)((double)cz - 0.1 * (double)V1[2]);
  return true;
}

// cornerOptimization's residual (:1083-1112) of query (x0, y0, z0) against the fitted line.
__device__ bool corner_apply(const float* f, float x0, float y0, float z0, float4& coeff) {
  const float x1 = f[0], y1 = f[1], z1 = f[2], x2 = f[3], y2 = f[4], z2 = f[5];
  const float a012 = sqrt_rn(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
  const float l12 = sqrt_rn((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
  const float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                    (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) / a012 / l12;
  const float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                     (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                     (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
  const float ld2 = a012 / l12;
  const float s = (float)(1.0 - 0.9 * (double)fabsf(ld2));
  coeff = make_float4(s * la, s * lb, s * lc, s * ld2);
  return (double)s > 0.1;
}

// surfOptimization's plane (:1145-1186): f[0..3] = (pa, pb, pc, pd); false when a neighbour is
// more than 0.2 from it.
__device__ bool surf_fit(const Nbr5& nn, float* f) {
  float A0[5][3], B0[5], X0[3];
  for (int j = 0; j < 5; j++) { A0[j][0] = nn.x[j]; A0[j][1] = nn.y[j]; A0[j][2] = nn.z[j]; B0[j] = -1.0f; }
  colpiv_solve53(A0, B0, X0);
  float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1.0f;
  const float ps = sqrt_rn(pa * pa + pb * pb + pc * pc);
  pa /= ps; pb /= ps; pc /= ps; pd /= ps;
  for (int j = 0; j < 5; j++)
    if ((double)fabsf(pa * nn.x[j] + pb * nn.y[j] + pc * nn.z[j] + pd) > 0.2) return false;
  f[0] = pa; f[1] = pb; f[2] = pc; f[3] = pd;
  return true;
}

// surfOptimization's residual (:1198-1211) of query (x0, y0, z0) against the plane.
__device__ bool surf_apply(const float* f, float x0, float y0, float z0, float4& coeff) {
  const float pa = f[0], pb = f[1], pc = f[2], pd = f[3];
  const float pd2 = pa * x0 + pb * y0 + pc * z0 + pd;
  const float s = (float)(1.0 - 0.9 * (double)fabsf(pd2) /
                                    (double)sqrt_rn(sqrt_rn(x0 * x0 + y0 * y0 + z0 * z0)));
  coeff = make_float4(s * pa, s * pb, s * pc, s * pd2);
  return (double)s > 0.1;
}

// Normal-equation product k of one row: 0-20 the upper AtA triangle, 21-26 AtB, 27 the count,
// 28-31 zero (compile-time k after unrolling).
__device__ __forceinline__ double res_product(int k, const float* row, float b, bool ok) {
  constexpr int kR[21] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 5};
  constexpr int kC[21] = {0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5, 2, 3, 4, 5, 3, 4, 5, 4, 5, 5};
  if (k < 21) return (double)row[kR[k]] * (double)row[kC[k]];
  if (k < 27) return (double)row[k - 21] * (double)b;
  if (k == 27) return ok ? 1.0 : 0.0;
  return 0.0;
}

// One transposed-butterfly step: H values per lane -> H/2 (the lower lane of each OFF pair keeps
// the first half, the upper lane the second).
template <int H, int OFF>
__device__ __forceinline__ void res_halve(double* v, int lane) {
  const bool up = (lane & OFF) != 0;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    const double lo = v[j], hi = v[j + H];
    v[j] = (up ? hi : lo) + __shfl_xor(up ? lo : hi, OFF);
  }
}

// The residual of query (x0, y0, z0) against its fitted line / plane (corner_apply / surf_apply)
// and its LMOptimization row (:1286-1332); false when the correspondence is rejected.
__device__ __forceinline__ bool res_apply_row(const GnState& g, bool corner, const float* fit, const float4& p, float x0,
                                              float y0, float z0, float* row, float& b) {
  float4 c;
  const bool ok = corner ? corner_apply(fit, x0, y0, z0, c) : surf_apply(fit, x0, y0, z0, c);
  if (ok) {
    // camera-frame swap
    const float srx = g.trig[0], crx = g.trig[1], sry = g.trig[2], cry = g.trig[3], srz = g.trig[4], crz = g.trig[5];
    const float pox = p.y, poy = p.z, poz = p.x;
    const float cox = c.y, coy = c.z, coz = c.x;
    const float arx = (crx * sry * srz * pox + crx * crz * sry * poy - srx * sry * poz) * cox +
                      (-srx * srz * pox - crz * srx * poy - crx * poz) * coy +
                      (crx * cry * srz * pox + crx * cry * crz * poy - cry * srx * poz) * coz;
    const float ary = ((cry * srx * srz - crz * sry) * pox + (sry * srz + cry * crz * srx) * poy + crx * cry * poz) * cox +
                      ((-cry * crz - srx * sry * srz) * pox + (cry * srz - crz * srx * sry) * poy - crx * sry * poz) * coz;
    const float arz = ((crz * srx * sry - cry * srz) * pox + (-cry * crz - srx * sry * srz) * poy) * cox +
                      (crx * crz * pox - crx * srz * poy) * coy +
                      ((sry * srz + cry * crz * srx) * pox + (crz * sry - cry * srx * srz) * poy) * coz;
    row[0] = arz; row[1] = arx; row[2] = ary; row[3] = coz; row[4] = cox; row[5] = coy;
    b = -c.w;
  }
  return ok;
}

// cornerOptimization / surfOptimization + the LMOptimization row (:1286-1332) of one query whose 5
// neighbours are the map points nb[0..4] (map indices); false when the correspondence is rejected.
// fc / fs: the query's fit cache (fit floats at stride kResThreads, state 0 none / 1 fitted /
// 2 rejected); same: the neighbours equal the previous iteration's, whose fit the cache holds.
__device__ __forceinline__ bool res_row(const GnState& g, const float4* by_id, const int32_t* nb, int stride,
                                        bool corner, const float4& p, float x0, float y0, float z0, float* row,
                                        float& b, float* fc, int8_t* fs, bool same) {
  float fit[6];
  bool fit_ok;
  const int8_t st = same ? *fs : (int8_t)0;
  if (st != 0) {
    fit_ok = st == 1;
    if (fit_ok) {
#pragma unroll
      for (int k = 0; k < 6; ++k) fit[k] = fc[k * kResThreads];
    }
  } else {
    Nbr5 nn;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float4 q = by_id[nb[k * stride]];
      nn.x[k] = q.x; nn.y[k] = q.y; nn.z[k] = q.z;
    }
    fit_ok = corner ? corner_fit(nn, fit) : surf_fit(nn, fit);
    *fs = fit_ok ? 1 : 2;
    if (fit_ok) {
#pragma unroll
      for (int k = 0; k < 6; ++k)
        if (corner || k < 4) fc[k * kResThreads] = fit[k];
    }
  }
  if (!fit_ok) return false;
  return res_apply_row(g, corner, fit, p, x0, y0, z0, row, b);
}

// The item's fp64 normal-equation partial (21 upper AtA entries, 6 AtB, count; 4 zero pads):
// every lane of the workgroup calls this with its row (zeros when it has none).  The wave sum is a
// transposed butterfly: at each halving step a lane keeps half of its values and trades the other
// half with its partner, so 32 values cost 32 shuffles instead of 6 per value.  Lane l (bit 0
// clear) ends with the wave sum of value ridx(l) (its bits 5..1 reversed); the 4 wave sums are
// added in LDS.  (A matrix-core form of this partial, v_mfma_f64_16x16x4 over the rows staged in
// LDS, bought 3 % of the kernel in round 4: the kernel is bound by its gathers and fits.)
__device__ __forceinline__ void res_reduce(double (*red)[28], int tid, const float* row, float b, bool ok,
                                           double* out) {
  const int lane = tid & 63, wave = tid >> 6;
  double v[16];
  const bool up5 = (lane & 32) != 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const double lo = res_product(j, row, b, ok), hi = res_product(j + 16, row, b, ok);
    v[j] = (up5 ? hi : lo) + __shfl_xor(up5 ? lo : hi, 32);
  }
  res_halve<8, 16>(v, lane);
  res_halve<4, 8>(v, lane);
  res_halve<2, 4>(v, lane);
  res_halve<1, 2>(v, lane);
  v[0] += __shfl_xor(v[0], 1);
  const int ridx = ((lane >> 5) & 1) * 16 + ((lane >> 4) & 1) * 8 + ((lane >> 3) & 1) * 4 + ((lane >> 2) & 1) * 2 +
                   ((lane >> 1) & 1);
  if (!(lane & 1) && ridx < 28) red[wave][ridx] = v[0];
  __syncthreads();
  if (tid < 28) {
    double s = 0.0;
    for (int w = 0; w < kResThreads / 64; ++w) s += red[w][tid];
    out[tid] = s;
  }
  __syncthreads();
}

// kNN pass: one lane per query, writes the 5 neighbour map indices (slot 0 = -1: no correspondence).
// R = grid cells per side covering radius 1 (both map grids share one cell size).  kFused: the
// same lane goes on to its residual row and the workgroup reduces the item's normal-equation
// partial (k_gn_residual's work, without re-reading the query and its neighbour indices).
// LPQ > 1 (wide mode, launches with few queries: single scans, tiny batches; neither fused nor
// flat): a workgroup covers 256 / LPQ queries of an item with LPQ lanes each, so a query's search
// chain is LPQ times shorter; lane `sub` == 0 of each query writes the results.
// One virtual workgroup v (item v / LPQ, query group v % LPQ) of the kNN pass (k_gn_knn's body).
template <int R, int RX, bool kFused, bool kFlat, bool kSparse, int LPQ>
__device__ __forceinline__ void gn_knn_block(const GnArgs& a, int v, int use_prev, double (*red)[28], int2* rows) {
  constexpr int QPB = kResThreads / LPQ;  // queries per workgroup
  const int sub = (int)threadIdx.x % LPQ;
  const int it = v / LPQ;
  const int tid = (v % LPQ) * QPB + (int)threadIdx.x / LPQ;  // query slot within the item
  const int4 item = a.items[it];
  const int job = item.x;
  const GnState& g = a.gn[job];
  if (!g.active) return;  // block-uniform
  float row[6] = {0, 0, 0, 0, 0, 0}, b = 0.0f;
  bool rok = false;
  if (tid < item.w) {
    const bool corner = item.y == 0;
    const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
    const float* T = g.T;
    // pointAssociateToMap (:397-403)
    const float x0 = T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3];
    const float y0 = T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7];
    const float z0 = T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11];
    const MapGrid& mg = corner ? a.mc : a.ms;
    int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
    float bound = __int_as_float(0x7f800000);
    int32_t oid[5] = {-1, -1, -1, -1, -1};
    const bool have_prev = use_prev && o[0] >= 0;
    if (have_prev) {  // warm start: the previous iteration's neighbours of this query
      float mx = 0.0f;
#pragma unroll
      for (int k = 0; k < 5; ++k) oid[k] = o[k * kResThreads];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float4 q = mg.by_id[oid[k]];
        float dist = 0.0f, diff;
        diff = x0 - q.x; dist += diff * diff;
        diff = y0 - q.y; dist += diff * diff;
        diff = z0 - q.z; dist += diff * diff;
        mx = fmaxf(mx, dist);
      }
      bound = mx;
    }
    Knn5 nn;
    unsigned ks[12] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    knn5_grid<R, RX, kFlat, kSparse, LPQ>(mg, x0, y0, z0, g.crop_min, g.crop_max, bound, nn, ks, rows, sub);
    if constexpr (LPQ > 1) knn5_merge<LPQ>(nn);
    const bool ok = nn.k[4] < kKnnEmpty;
    (void)ks;
    int32_t ids[5];
    bool same = have_prev && ok && a.fit_cache;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      ids[k] = knn_id(nn.k[k]);
      same = same && ids[k] == oid[k];
    }
    if (LPQ > 1) __builtin_amdgcn_wave_barrier();  // every lane of the query read o[] (warm start)
    if (sub == 0)
#pragma unroll
      for (int k = 0; k < 5; ++k) o[k * kResThreads] = ok ? ids[k] : -1;
    const int64_t q = (int64_t)it * kResThreads + tid;
    if (!kFused && sub == 0) a.nsame[q] = same ? 1 : 0;
#ifdef FBR_KNN_STATS
    ks[5] = ok;
    ks[6] = corner;
    ks[8] = have_prev;
    ks[9] = same;
    for (int k = 0; k < 10; ++k) atomicAdd(&a.knn_stats[k], (unsigned long long)ks[k]);
    if (kFlat && use_prev) {
      atomicAdd(&a.knn_stats[10], 1ull);
      atomicAdd(&a.knn_stats[11], (unsigned long long)ks[10]);
      atomicAdd(&a.knn_stats[12 + (ks[10] < 32 ? ks[10] : ks[10] < 64 ? 32 : 33)], 1ull);
      atomicAdd(&a.knn_stats[46], (unsigned long long)ks[3]);
      atomicAdd(&a.knn_stats[47], (unsigned long long)ks[11]);
    }
#endif
    if (kFused && ok)
      rok = res_row(g, mg.by_id, ids, 1, corner, p, x0, y0, z0, row, b, a.fitc + (int64_t)it * 6 * kResThreads + tid,
                    a.fits + q, same);
  }
  if (kFused) res_reduce(red, tid, row, b, rok, a.partial + (int64_t)it * kPartial);
}

// kLoop = false: virtual workgroup base + blockIdx.x only (one_item launches, k_gn_knn); true: a
// grid-stride loop from base (k_gn_loop_knn: single scans, wide mode, the items past a one-item grid).
template <int R, int RX, bool kFused, bool kFlat, bool kSparse, int LPQ, bool kLoop>
__device__ __forceinline__ void gn_knn_kernel(const GnArgs& a, int use_prev, int base) {
  static_assert(LPQ == 1 || (!kFused && !kFlat), "wide mode is the plain kNN pass");
  __shared__ double red[kFused ? kResThreads / 64 : 1][28];
  __shared__ int2 rows[kFlat ? (2 * R + 1) * (2 * R + 1) : 1][kResThreads];
  const int nitems = a.nitems[0];
  if constexpr (kLoop) {
    for (int v = base + blockIdx.x; v < nitems * LPQ; v += gridDim.x)
      gn_knn_block<R, RX, kFused, kFlat, kSparse, LPQ>(a, v, use_prev, red, &rows[0][threadIdx.x]);
  } else {
    const int v = base + (int)blockIdx.x;
    if (v < nitems * LPQ) gn_knn_block<R, RX, kFused, kFlat, kSparse, LPQ>(a, v, use_prev, red, &rows[0][threadIdx.x]);
  }
}
template <int R, int RX, bool kFused, bool kFlat, bool kSparse, int LPQ = 1>
__global__ void __launch_bounds__(kResThreads) k_gn_knn(GnArgs a, int use_prev, int base) {
  gn_knn_kernel<R, RX, kFused, kFlat, kSparse, LPQ, false>(a, use_prev, base);
}
template <int R, int RX, bool kFused, bool kFlat, bool kSparse, int LPQ = 1>
__global__ void __launch_bounds__(kResThreads) k_gn_loop_knn(GnArgs a, int use_prev, int base) {
  gn_knn_kernel<R, RX, kFused, kFlat, kSparse, LPQ, true>(a, use_prev, base);
}

// Items past a one-item launch's grid: a loop launch of at most GnArgs::rest_grid (default 2048)
// workgroups from `grid` (they return at once when the grid covered every item; while other
// streams' kernels hold the CUs, even returning workgroups wait for slots, so the host keeps the
// loop launch small when it sized the grid from a previous run's count).
constexpr int kRestGrid = 2048;
template <typename Kmain, typename Krest, typename... Args>
void launch_one_item(hipStream_t s, const GnArgs& a, int grid, int total, size_t lds, Kmain kmain, Krest krest,
                     Args... args) {
  if (a.one_item == 1 && grid < total) {
    if (a.one_part != 2) fbr_launch(kmain, dim3(grid), dim3(kResThreads), lds, s, args..., 0);
    if (a.one_part != 1)
      fbr_launch(krest, dim3(std::min(a.rest_grid > 0 ? a.rest_grid : kRestGrid, total - grid)), dim3(kResThreads), lds,
                 s, args..., grid);
  } else if (a.one_part != 2) {
    fbr_launch(a.one_item ? kmain : krest, dim3(grid), dim3(kResThreads), lds, s, args..., 0);
  }
}

// pcl::getTransformation (x,y,z,roll,pitch,yaw) in float with glibc's sinf / cosf
// (fbr_sincosf.h: the FMA variant restated bit for bit).
__device__ void pose_to_T(const float* tr, float* T, float* trig) {
  const float roll = tr[0], pitch = tr[1], yaw = tr[2];
  const float A = gl_cosf(yaw), B = gl_sinf(yaw), C = gl_cosf(pitch), D = gl_sinf(pitch), E = gl_cosf(roll),
              F = gl_sinf(roll);
  const float DE = D * E, DF = D * F;
  T[0] = A * C; T[1] = A * DF - B * E; T[2] = B * F + A * DE; T[3] = tr[3];
  T[4] = B * C; T[5] = A * E + B * DF; T[6] = B * DE - A * F; T[7] = tr[4];
  T[8] = -D;    T[9] = C * F;          T[10] = C * E;         T[11] = tr[5];
  // LMOptimization (:1259-1264): srx, crx (pitch), sry, cry (yaw), srz, crz (roll)
  trig[0] = D; trig[1] = C; trig[2] = B; trig[3] = A; trig[4] = F; trig[5] = E;
}

// The residual rows of work item `it` and its normal-equation partial (k_gn_residual's body).
// (Round 6 measured packing an item's refits into the first waves -- list them in LDS, fit, barrier,
// apply: -15 % VALU instructions per dispatch but +6 % duration alone, the two extra barriers
// exposing the gathers' latency; profiles/r06b_residual_refit_compaction_ab.txt.)
__device__ __forceinline__ void gn_residual_item(const GnArgs& a, int it, double (*red)[28]) {
  const int tid = threadIdx.x;
  const int4 item = a.items[it];
  const int job = item.x;
  const GnState& g = a.gn[job];
  if (!g.active) return;  // block-uniform
  float row[6] = {0, 0, 0, 0, 0, 0}, b = 0.0f;
  bool ok = false;
  const int32_t* nb = a.nbr + (int64_t)it * 5 * kResThreads + tid;
  if (tid < item.w && nb[0] >= 0) {
    const bool corner = item.y == 0;
    const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
    const float* T = g.T;
    const float x0 = T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3];
    const float y0 = T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7];
    const float z0 = T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11];
    const int64_t q = (int64_t)it * kResThreads + tid;
    ok = res_row(g, corner ? a.mc.by_id : a.ms.by_id, nb, kResThreads, corner, p, x0, y0, z0, row, b,
                 a.fitc + (int64_t)it * 6 * kResThreads + tid, a.fits + q, a.nsame[q] != 0);
  }
  res_reduce(red, tid, row, b, ok, a.partial + (int64_t)it * kPartial);
}

// The normal equations of one job in float, as LMOptimization forms them (matAtA / matAtB).
__device__ __forceinline__ void gn_normal_eq(const double* acc, float* AtA, float* X) {
  int q = 0;
  for (int r = 0; r < 6; ++r)
    for (int c = r; c < 6; ++c) {
      AtA[r * 6 + c] = (float)acc[q];
      AtA[c * 6 + r] = (float)acc[q];
      ++q;
    }
  for (int r = 0; r < 6; ++r) X[r] = (float)acc[21 + r];
}

// Iteration-0 degeneracy projection (:1280-1305): 6x6 Jacobi, eigenvalues < 100 zero rows of V2,
// matP = V^-1 * V2 by LU.  It depends only on AtA, so the second wave of k_gn_solve computes it
// (the Jacobi rotations spread over its lanes, jacobi_eigen_wave) while the first solves
// AtA X = AtB.  All 64 lanes of the wave call it; matP / degenerate are written by lane 0.  A
// matrix whose eigenvalues are certified above 100 (eig_above_certified: an LDL^T test with a
// 1e-3 ||A|| margin, the common case) skips the Jacobi and the LU: degenerate = 0, and matP is
// then never read (gn_solve_job applies it only when degenerate).
struct EigenLds {
  float A[36], V[36], W[6];
  int R[6], C[6];
};
__device__ void gn_degeneracy(const double* acc, EigenLds& e, float* matP, int* degenerate) {
  const int lane = threadIdx.x & 63;
  if (lane < 36) {
    const int r = lane / 6, c = lane % 6, lo = r < c ? r : c, hi = r < c ? c : r;
    e.A[lane] = (float)acc[lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];  // upper-triangle order
  }
  wave_lds_sync();
  if (eig_above_certified<6>(e.A, 100.0f)) {  // every eigenvalue >= 100: not degenerate, matP unused
    if (lane == 0) *degenerate = 0;
    return;
  }
  jacobi_eigen_wave<6>(e.A, e.W, e.V, e.R, e.C);
  if (lane != 0) return;
  float E[6], V[36], V2[36], Vi[36];
  for (int k = 0; k < 6; ++k) E[k] = e.W[k];
  for (int k = 0; k < 36; ++k) V[k] = e.V[k];
  for (int k = 0; k < 36; ++k) V2[k] = V[k];
  int deg = 0;
  for (int i = 5; i >= 0; i--) {
    if (E[i] < 100.0f) {
      for (int j = 0; j < 6; j++) V2[i * 6 + j] = 0.0f;
      deg = 1;
    } else {
      break;
    }
  }
  *degenerate = deg;
  if (!lu_inv6(V, Vi))
    for (int k = 0; k < 36; ++k) Vi[k] = 0.0f;
  float P[36];
  for (int k = 0; k < 36; ++k) P[k] = 0.0f;
  gemm_f32_acc64<6, 6, 6>(Vi, V2, P);
  for (int k = 0; k < 36; ++k) matP[k] = P[k];
}

// matAtA X = matAtB by OpenCV's float Householder QR (:1276); X = 0 if singular.
__device__ void gn_qr_step(const double* acc, float* X) {
  float AtA[36];
  gn_normal_eq(acc, AtA, X);
  if (!qr_solve6(AtA, X))
    for (int k = 0; k < 6; ++k) X[k] = 0.0f;
}

// One job's LMOptimization step on one lane (acc = the job's summed normal-equation products,
// X = gn_qr_step's solution, matP0 / deg0 = gn_degeneracy's result at iteration 0).
__device__ void gn_solve_job(const GnArgs& a, int job, const double* acc, float* X, const float* matP0, int deg0) {
  GnState& g = a.gn[job];
  const int iterCount = g.iter;
  g.iter = iterCount + 1;
  const int sel = (int)acc[27];
  g.n_sel = sel;
  if (a.trace) {
    // filled below after the update; pre-fill with the current pose for the early-return case
    for (int k = 0; k < 6; ++k) a.trace[((int64_t)job * a.max_iter + iterCount) * 6 + k] = g.pose[k];
  }
  if (sel < 50) {  // :1268 return false
    if (g.iter >= a.max_iter) g.active = 0;
    return;
  }
  // the local cv::Mat matP (:1278) is zero after iteration 0
  if (iterCount == 0) g.degenerate = deg0;
  if (g.degenerate) {
    float X2[6];
    for (int k = 0; k < 6; ++k) X2[k] = X[k];
    if (iterCount == 0) {
      float P[36];
      for (int k = 0; k < 36; ++k) P[k] = matP0[k];
      gemm_f32_acc64<6, 6, 1>(P, X2, X);
    } else {
      float P[36];
      for (int k = 0; k < 36; ++k) P[k] = 0.0f;
      gemm_f32_acc64<6, 6, 1>(P, X2, X);
    }
  }
  for (int k = 0; k < 6; ++k) g.pose[k] += X[k];
  if (a.trace)
    for (int k = 0; k < 6; ++k) a.trace[((int64_t)job * a.max_iter + iterCount) * 6 + k] = g.pose[k];
  const double r0 = (double)(X[0] * 57.29578f), r1 = (double)(X[1] * 57.29578f), r2 = (double)(X[2] * 57.29578f);
  const float deltaR = (float)sqrt(r0 * r0 + r1 * r1 + r2 * r2);
  const double t0 = (double)(X[3] * 100.0f), t1 = (double)(X[4] * 100.0f), t2 = (double)(X[5] * 100.0f);
  const float deltaT = (float)sqrt(t0 * t0 + t1 * t1 + t2 * t2);
  if ((double)deltaR < 0.05 && (double)deltaT < 0.05) {
    g.converged = 1;
    g.active = 0;
  } else if (g.iter >= a.max_iter) {
    g.active = 0;
  }
  pose_to_T(g.pose, g.T, g.trig);
}

// One job's LMOptimization step by the first two waves of a workgroup (k_gn_solve's body; extra
// waves only pass the barriers).
struct SolveLds {
  double acc[28];
  float matP0[36];
  int deg0;
  EigenLds eig;
};
__device__ __forceinline__ void gn_solve_block(const GnArgs& a, int job, SolveLds& s) {
  const int tid = threadIdx.x;
  GnState& g = a.gn[job];
  if (!g.active) return;  // block-uniform
  const int iter0 = g.iter == 0;  // read before lane 0 updates it (ordered by the barriers)
  if (tid < 28) {
    double sum = 0.0;
    const int i0 = a.item_range[2 * job], i1 = a.item_range[2 * job + 1];
#pragma unroll 8
    for (int it = i0; it < i1; ++it) sum += a.partial[(int64_t)it * kPartial + tid];
    s.acc[tid] = sum;
  }
  __syncthreads();
  float X[6];
  const bool solve = (int)s.acc[27] >= 50;
  if (tid >= 64 && tid < 128 && iter0 && solve) gn_degeneracy(s.acc, s.eig, s.matP0, &s.deg0);
  if (tid == 0 && solve) gn_qr_step(s.acc, X);
  __syncthreads();
  if (tid == 0) gn_solve_job(a, job, s.acc, X, s.matP0, s.deg0);
  __syncthreads();
}

// Host launchers of the kNN pass.  launch_gn_knn_r<R, F> is instantiated in k_knn_*.hip.
template <int R, bool F, bool L, bool S, int LPQ = 1>
void launch_gn_knn_rls(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  const float invx = a.mc.g.inv_x;  // == a.ms.g.inv_x
  grid *= LPQ;
  const int total = a.max_items * LPQ;
  // one-item launches at one lane per query (wide mode loops)
  constexpr bool kOne = LPQ == 1;
  auto go = [&](auto rx) {
    constexpr int RX = decltype(rx)::value;
    if constexpr (kOne)
      launch_one_item(s, a, grid, total, 0, k_gn_knn<R, RX, F, L, S, LPQ>, k_gn_loop_knn<R, RX, F, L, S, LPQ>, a,
                      use_prev);
    else if (a.one_part != 2)
      fbr_launch((k_gn_loop_knn<R, RX, F, L, S, LPQ>), dim3(grid), dim3(kResThreads), 0, s, a, use_prev, 0);
  };
  if (invx > 4.0f) go(std::integral_constant<int, 8>{});       // 0.125 m
  else if (invx > 2.0f) go(std::integral_constant<int, 4>{});  // 0.25 m
  else if (invx > 1.0f) go(std::integral_constant<int, 2>{});  // 0.5 m
  else go(std::integral_constant<int, 1>{});                  // >= 1 m
}
// Dense or hashed-chunk map grids (one flag for both maps: fbr_set_map builds them alike).
template <int R, bool F, bool L, int LPQ = 1>
void launch_gn_knn_rl(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  if (a.mc.g.sparse || a.ms.g.sparse) launch_gn_knn_rls<R, F, L, true, LPQ>(s, a, grid, use_prev);
  else launch_gn_knn_rls<R, F, L, false, LPQ>(s, a, grid, use_prev);
}

// Lanes per query of the plain kNN pass (FBR_KNN_LPQ = 1 or 8; default 8 for sub-batches of at
// most 2 jobs, where one lane per query leaves the chip idle and the launch is one query's chain).
inline int knn_lpq(int jobs) {
  static const int forced = [] {
    const char* e = std::getenv("FBR_KNN_LPQ");
    return e ? (std::atoi(e) >= 8 ? 8 : 1) : 0;
  }();
  if (forced) return forced;
  return jobs <= 2 ? 8 : 1;
}

// Flat row queue (FBR_KNN_FLAT=0 disables): from iteration 1 on (warm-start bound), 1 m y/z cells
// (9 rows: the queue is 18 KB of LDS per workgroup), not in the fused tail launch.
inline bool knn_flat() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_KNN_FLAT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

template <int R, bool F>
void launch_gn_knn_r(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  if constexpr (!F) {
    if (knn_lpq(a.B) == 8) return launch_gn_knn_rl<R, F, false, 8>(s, a, grid, use_prev);
  }
  // flat queue for the 1 m cells from iteration 1 (round 4 measured it slower in iteration 0, with
  // no warm-start bound, and for the 0.5 m cells, whose 25-row queue costs occupancy)
  if constexpr (R == 1 && !F) {
    if (use_prev && knn_flat()) return launch_gn_knn_rl<R, F, true>(s, a, grid, use_prev);
  }
  launch_gn_knn_rl<R, F, false>(s, a, grid, use_prev);
}

}  // namespace fbr
