// k_register.hip — A10-A18: scan2MapOptimization on the device.
//
// Reference: /root/reference/src/mapOptmization.h
//   registration()            :263-343  crop box (:284-304), pose <-> transformTobeMapped (:309,:326)
//   cornerOptimization()      :1002-1124 point-to-line residual, kNN-5, 3x3 cv::eigen
//   surfOptimization()        :1126-1215 point-to-plane residual, kNN-5, 5x3 colPivHouseholderQr
//   combineOptimizationCoeffs :1218-1243 corner rows (index order) then surf rows
//   LMOptimization()          :1246-1401 camera-frame Jacobian rows, AtA/AtB, QR solve,
//                                        iteration-0 degeneracy (eigen < 100), update, 0.05/0.05 stop
//   scan2MapOptimization()    :1403-1442 feature gate, <= 30 iterations
//   transformUpdate()         :1444-1489 IMU roll/pitch slerp when a deskew table says
//                                        imuAvailable (fbr_set_deskew), tolerance clamps
//
// Design (MI355X-first, results identical to the reference's KD-tree path):
//   * The reference rebuilds two FLANN KD-trees on the cropped local map every scan.  Here the
//     global map is bucketed ONCE into a dense grid with power-of-two cells (exact integer cell
//     coordinates); the per-scan CropBox becomes a per-candidate box test.  Because a
//     correspondence is kept only if the 5th neighbour has d2 < 1.0 (:1027, :1154), keeping the 5
//     smallest (d2, index) with d2 < 1.0 among the cells within radius 1 selects exactly the same
//     neighbours as exact kNN-5 on the cropped cloud.  Cells are pruned with a float lower bound
//     that provably never exceeds a member point's computed distance (see axis_lb).
//   * k_gn_knn: one lane per query (corner and surf queries of every active job of the batch are
//     packed into 256-query work items; the mapping-DS clouds are in Morton order, so a wave's
//     queries are spatially compact); writes the 5 neighbours' map indices per query.
//   * k_gn_residual: gathers the 5 neighbours, residual and Jacobian row in float with the
//     reference's operation order; the 21+6 normal-equation products are reduced in fp64
//     (OpenCV's CV_32F gemm accumulates in double) by a transposed wave butterfly into one
//     partial per item.  (k_gn_knn<.., true> does both in one launch: the GN tail mode.)
//   * k_gn_solve: one lane per job sums its items in order (corner items, then surf items: the
//     combineOptimizationCoeffs row order), rounds AtA/AtB to float and runs the reference's float
//     QR solve / Jacobi / LU; the Gauss-Newton state never leaves the device.
// Roofline: HBM/L2 gather-bound.  Algorithmic bytes per query per iteration: 16 (query) +
// 5 x 16 (neighbours) = 96 B.
#include <cstdlib>

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

// Branch-free sorted insertion: the "less than slot t" flags are monotone over t, so every slot
// takes its own key, its left neighbour's, or the new one (5 compares + 20 selects, no SALU mask
// arithmetic and no serial compare-swap chain).
__device__ __forceinline__ void knn_insert(Knn5& r, unsigned long long x) {
  bool lt[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) lt[t] = x < r.k[t];
#pragma unroll
  for (int t = 4; t > 0; --t) r.k[t] = lt[t - 1] ? r.k[t - 1] : (lt[t] ? x : r.k[t]);  // lt[t-1] implies lt[t]
  r.k[0] = lt[0] ? x : r.k[0];
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
// warm-started queries, queries whose neighbours equal the previous iteration's]
__device__ unsigned long long fbr_knn_stats[10];
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
// LDS map tile (k_gn_knn_tile): the points of the cells [X0, X0 + NX1 - 1] of the rows
// (Y0.., Z0..) copied to LDS in map order, and per row the LDS offsets of those cells' starts.
struct TileView {
  const float4* pts;  // LDS points
  const int* cs;      // [row][NX1] LDS offset of cell X0 + j (j = NX1 - 1: the row end)
  int X0, Y0, Z0, NX1, NY;
};

// kTile: the search reads the cells' point ranges and points from the workgroup's LDS tile (`tv`)
// instead of the map grid in HBM; same rows, same ranges, same points in the same order.
template <int R, int RX, bool kFlat = false, bool kSparse = false, int LPQ = 1, bool kTile = false>
__device__ void knn5_grid(const MapGrid& m, float qx, float qy, float qz, const float* bmin, const float* bmax,
                          float bound, Knn5& r, unsigned* ks, int2* rows = nullptr, int sub = 0,
                          const TileView* tv = nullptr) {
  static_assert(!kTile || (!kFlat && !kSparse && LPQ == 1), "tile mode: dense grid, per-row loop");
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
    oyk[k] = rank_offset(k, sgy);
    ozk[k] = rank_offset(k, sgz);
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
      if constexpr (kTile) {
        const int* cs = tv->cs + ((z - tv->Z0) * tv->NY + (y - tv->Y0)) * tv->NX1 - tv->X0;
        b = cs[x0];
        e = cs[x1 + 1];
      } else if (!row_range<kSparse>(m, y, z, x0, x1, b, e)) {
        continue;
      }
      FBR_KS(2, 1);
      FBR_KS(3, e - b);
      // the whole row inside the crop box (pcl::CropBox, inclusive) -> no per-point test
      const float ylo = (fy + (float)oyk[ky]) * c, zlo = (fz + (float)ozk[kz]) * c;
      const bool inside = xin & (ylo >= by0) & (ylo + c <= by1) & (zlo >= bz0) & (zlo + c <= bz1);
      if constexpr (kFlat) {
        if (e > b) rows[nrow++ * kResThreads] = make_int2(b, inside ? (int)((unsigned)e | 0x80000000u) : e);
        continue;
      }
      for (int i = LPQ == 1 ? b : b + ((sub - b) & (LPQ - 1)); i < e; i += LPQ) {
        const float4 p = kTile ? tv->pts[i] : m.pts[i];
        // pcl::CropBox (inclusive) as one mask: a point outside gets d2 = +inf (never inserted)
        bool out = false;  // rows inside the box skip the test
        if (!inside) out = (p.x < bx0) | (p.y < by0) | (p.z < bz0) | (p.x > bx1) | (p.y > by1) | (p.z > bz1);
        float dist = 0.0f, diff;
        diff = qx - p.x; dist += diff * diff;                            // flann::L2_Simple
        diff = qy - p.y; dist += diff * diff;
        diff = qz - p.z; dist += diff * diff;
        const unsigned hi = out ? 0x7f800000u : (unsigned)__float_as_int(dist);
        FBR_KS(4, __int_as_float((int)hi) < knn_d(r.k[4]) ? 1 : 0);
#ifdef FBR_KNN_STATS
        if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) ks[7] += 1;  // one per wave iteration
#endif
        knn_insert(r, ((unsigned long long)hi << 32) | (unsigned)__float_as_int(p.w));
      }
    }
  }
  if constexpr (kFlat) {
    int j = 0, i = 0, e = 0;
    bool inside = true;
    while (true) {
      if (i >= e) {  // next queued row (every queued row is non-empty)
        if (j >= nrow) break;
        const int2 q = rows[j++ * kResThreads];
        i = q.x;
        e = q.y & 0x7fffffff;
        inside = q.y < 0;
      }
      const float4 p = m.pts[i++];
      bool out = false;
      if (!inside) out = (p.x < bx0) | (p.y < by0) | (p.z < bz0) | (p.x > bx1) | (p.y > by1) | (p.z > bz1);
      float dist = 0.0f, diff;
      diff = qx - p.x; dist += diff * diff;  // flann::L2_Simple
      diff = qy - p.y; dist += diff * diff;
      diff = qz - p.z; dist += diff * diff;
      const unsigned hi = out ? 0x7f800000u : (unsigned)__float_as_int(dist);
      FBR_KS(4, __int_as_float((int)hi) < knn_d(r.k[4]) ? 1 : 0);
#ifdef FBR_KNN_STATS
      if (__lane_id() == __ffsll((long long)__ballot(1)) - 1) ks[7] += 1;  // one per wave iteration
#endif
      knn_insert(r, ((unsigned long long)hi << 32) | (unsigned)__float_as_int(p.w));
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
    for (int t = 0; t < 5; ++t) knn_insert(r, o[t]);
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

__global__ void k_gn_init(GnArgs a) {
  __shared__ int32_t scan[1024];
  const int tid = threadIdx.x;
  int base = 0;
  for (int j0 = 0; j0 < a.B; j0 += 1024) {
    const int job = j0 + tid;
    int nc_items = 0, ns_items = 0;
    if (job < a.B) {
      GnState& g = a.gn[job];
      for (int k = 0; k < 6; ++k) g.pose[k] = a.guess[job * 6 + k];
      pose_to_T(g.pose, g.T, g.trig);
      for (int k = 0; k < 3; ++k) {  // edge = size + origin (float), :289-292
        g.crop_min[k] = a.nocrop ? -FLT_MAX : -a.crop_half[k] + g.pose[3 + k];  // keyframe map: no CropBox
        g.crop_max[k] = a.nocrop ? FLT_MAX : a.crop_half[k] + g.pose[3 + k];
      }
      for (int k = 0; k < 36; ++k) g.matP[k] = 0.0f;
      const int nc = a.ncds[job], ns = a.nsds[job];
      g.iter = 0; g.converged = 0; g.n_sel = 0;
      // isDegenerate is a class member: an iteration-0 early return (< 50 rows) keeps the previous
      // scan's value (single-scan paths carry it; independent batch jobs start from false)
      g.degenerate = a.deg_carry ? 1 : 0;
      if (nc > a.edge_min && ns > a.surf_min) {
        g.status = FBR_REG_OK;
        g.active = 1;
        nc_items = (nc + kResThreads - 1) / kResThreads;
        ns_items = (ns + kResThreads - 1) / kResThreads;
      } else {
        g.status = FBR_REG_NOT_ENOUGH_FEATURES;
        g.active = 0;
      }
    }
    scan[tid] = nc_items + ns_items;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int v = tid >= off ? scan[tid - off] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    const int incl = scan[tid];
    const int excl = base + incl - (nc_items + ns_items);
    if (job < a.B) {
      a.item_range[2 * job] = excl;
      a.item_range[2 * job + 1] = excl + nc_items + ns_items;
      const int nc = a.ncds[job], ns = a.nsds[job];
      int it = excl;
      for (int t = 0; t < nc_items; ++t, ++it)
        if (it < a.max_items) a.items[it] = make_int4(job, 0, t * kResThreads, min(kResThreads, nc - t * kResThreads));
      for (int t = 0; t < ns_items; ++t, ++it)
        if (it < a.max_items) a.items[it] = make_int4(job, 1, t * kResThreads, min(kResThreads, ns - t * kResThreads));
    }
    base += scan[1023];
    __syncthreads();
  }
  if (tid == 0) a.nitems[0] = min(base, a.max_items);
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

// The item's fp64 normal-equation partial (21 upper AtA entries, 6 AtB, count; 4 zero pads):
// every lane of the workgroup calls this with its row (zeros when it has none).  The wave sum is a
// transposed butterfly: at each halving step a lane keeps half of its values and trades the other
// half with its partner, so 32 values cost 32 shuffles instead of 6 per value.  Lane l (bit 0
// clear) ends with the wave sum of value res_index(l); the 4 wave sums are added in LDS.
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

__global__ void __launch_bounds__(kResThreads)
k_gn_residual(GnArgs a) {
  __shared__ double red[kResThreads / 64][28];
  const int tid = threadIdx.x;
  const int nitems = a.nitems[0];
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int4 item = a.items[it];
    const int job = item.x;
    const GnState& g = a.gn[job];
    if (!g.active) continue;  // block-uniform
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
}

// kNN pass: one lane per query, writes the 5 neighbour map indices (slot 0 = -1: no correspondence).
// R = grid cells per side covering radius 1 (both map grids share one cell size).  kFused: the
// same lane goes on to its residual row and the workgroup reduces the item's normal-equation
// partial (k_gn_residual's work, without re-reading the query and its neighbour indices).
// LPQ > 1 (wide mode, launches with few queries: single scans, tiny batches; neither fused nor
// flat): a workgroup covers 256 / LPQ queries of an item with LPQ lanes each, so a query's search
// chain is LPQ times shorter; lane `sub` == 0 of each query writes the results.
template <int R, int RX, bool kFused, bool kFlat, bool kSparse, int LPQ = 1>
__global__ void __launch_bounds__(kResThreads)
k_gn_knn(GnArgs a, int use_prev) {
  static_assert(LPQ == 1 || (!kFused && !kFlat), "wide mode is the plain kNN pass");
  __shared__ double red[kFused ? kResThreads / 64 : 1][28];
  __shared__ int2 rows[kFlat ? (2 * R + 1) * (2 * R + 1) : 1][kResThreads];
  constexpr int QPB = kResThreads / LPQ;  // queries per workgroup
  const int sub = (int)threadIdx.x % LPQ;
  const int nitems = a.nitems[0];
  for (int v = blockIdx.x; v < nitems * LPQ; v += gridDim.x) {
    const int it = v / LPQ;
    const int tid = (v % LPQ) * QPB + (int)threadIdx.x / LPQ;  // query slot within the item
    const int4 item = a.items[it];
    const int job = item.x;
    const GnState& g = a.gn[job];
    if (!g.active) continue;  // block-uniform
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
      unsigned ks[10] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      knn5_grid<R, RX, kFlat, kSparse, LPQ>(mg, x0, y0, z0, g.crop_min, g.crop_max, bound, nn, ks,
                                            &rows[0][threadIdx.x], sub);
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
      for (int k = 0; k < 10; ++k) atomicAdd(&fbr_knn_stats[k], (unsigned long long)ks[k]);
#endif
      if (kFused && ok)
        rok = res_row(g, mg.by_id, ids, 1, corner, p, x0, y0, z0, row, b, a.fitc + (int64_t)it * 6 * kResThreads + tid,
                      a.fits + q, same);
    }
    if (kFused) res_reduce(red, tid, row, b, rok, a.partial + (int64_t)it * kPartial);
  }
}

// LDS-staged map tiles (dense maps: C3 / C5 mapping leaves).  The work item's 256
// Morton-ordered queries are spatially compact, so their candidate cells overlap: the workgroup
// takes the union box of the cells each query may visit (per axis, the cells whose lower-bound
// distance is within min(warm-start bound, 1), the same float bounds the search prunes with),
// copies those cells' points into LDS once with coalesced loads, and every lane then runs the
// unchanged search over the LDS copy (same rows, same ranges, same points in the same order, so
// the same neighbours).  Items whose box exceeds the tile capacity (iteration 0 has no warm-start
// bound) search HBM as k_gn_knn does.  On dense maps the per-query point loads of the HBM search
// miss L2 and wait on memory; from LDS they do not.
constexpr int kTilePts = 2048;  // float4 points per tile (32 KB of dynamic LDS)
constexpr int kTileCs = 2048;   // row cell offsets per tile
constexpr int kTileRows = 256;  // (y, z) rows per tile

template <int R, int RX>
__global__ void __launch_bounds__(kResThreads)
k_gn_knn_tile(GnArgs a, int use_prev) {
  extern __shared__ float4 tpts[];        // [kTilePts]
  __shared__ int tcs[kTileCs];
  __shared__ int rowoff[kTileRows + 1];   // per tile row: LDS offset of its points
  __shared__ int rowgb[kTileRows];        // per tile row: map index of its first point
  __shared__ int box[6];                  // X0, Y0, Z0, X1, Y1, Z1 (cells)
  const int tid = threadIdx.x;
  const int nitems = a.nitems[0];
  for (int it = blockIdx.x; it < nitems; it += gridDim.x) {
    const int4 item = a.items[it];
    const int job = item.x;
    const GnState& g = a.gn[job];
    if (!g.active) continue;  // block-uniform
    const bool corner = item.y == 0;
    const MapGrid& mg = corner ? a.mc : a.ms;
    const bool valid = tid < item.w;
    float x0 = 0.0f, y0 = 0.0f, z0 = 0.0f, bound = __int_as_float(0x7f800000);
    int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
    int32_t oid[5] = {-1, -1, -1, -1, -1};
    bool have_prev = false;
    if (tid < 6) box[tid] = tid < 3 ? INT_MAX : INT_MIN;
    __syncthreads();
    if (valid) {
      const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
      const float* T = g.T;
      x0 = T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3];  // pointAssociateToMap (:397-403)
      y0 = T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7];
      z0 = T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11];
      have_prev = use_prev && o[0] >= 0;
      if (have_prev) {
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
      // the cells this query may visit (knn5_grid's cell arithmetic and lower bounds)
      const float inv = mg.g.inv_cell, c = 1.0f / inv, invx = mg.g.inv_x, cxs = 1.0f / invx;
      const float sx = x0 * invx, sy = y0 * inv, sz = z0 * inv;
      const float fx = floorf(sx), fy = floorf(sy), fz = floorf(sz);
      if (fabsf(fx) < 1e7f && fabsf(fy) < 1e7f && fabsf(fz) < 1e7f) {
        const int cx = (int)fx - (int)mg.g.origin[0], cy = (int)fy - (int)mg.g.origin[1], cz = (int)fz - (int)mg.g.origin[2];
        if (!(cx < -RX || cy < -R || cz < -R || cx >= mg.g.dims[0] + RX || cy >= mg.g.dims[1] + R ||
              cz >= mg.g.dims[2] + R)) {
          const float Bp = fminf(bound, kBelowOne);
          int ylo = 0, yhi = 0, zlo = 0, zhi = 0, xlo = 0, xhi = 0;
#pragma unroll
          for (int oo = 1; oo <= R; ++oo) {
            float l;
            l = axis_lb(y0, fy, -oo, c); if (l * l <= Bp) ylo = -oo;
            l = axis_lb(y0, fy, oo, c); if (l * l <= Bp) yhi = oo;
            l = axis_lb(z0, fz, -oo, c); if (l * l <= Bp) zlo = -oo;
            l = axis_lb(z0, fz, oo, c); if (l * l <= Bp) zhi = oo;
          }
#pragma unroll
          for (int oo = 1; oo <= RX; ++oo) {
            float l;
            l = axis_lb(x0, fx, -oo, cxs); if (l * l <= Bp) xlo = -oo;
            l = axis_lb(x0, fx, oo, cxs); if (l * l <= Bp) xhi = oo;
          }
          atomicMin(&box[0], cx + xlo);
          atomicMin(&box[1], cy + ylo);
          atomicMin(&box[2], cz + zlo);
          atomicMax(&box[3], cx + xhi);
          atomicMax(&box[4], cy + yhi);
          atomicMax(&box[5], cz + zhi);
        }
      }
    }
    __syncthreads();
    // clamp to the grid (the search skips cells outside it) and size the tile
    const int X0 = max(box[0], 0), Y0 = max(box[1], 0), Z0 = max(box[2], 0);
    const int X1 = min(box[3], mg.g.dims[0] - 1), Y1 = min(box[4], mg.g.dims[1] - 1), Z1 = min(box[5], mg.g.dims[2] - 1);
    const int NX1 = X1 - X0 + 2, NY = Y1 - Y0 + 1, NZ = Z1 - Z0 + 1;
    bool tile = X1 >= X0 && Y1 >= Y0 && Z1 >= Z0 && NY * NZ <= kTileRows && NY * NZ * NX1 <= kTileCs;
    if (tile) {
      const int rows = NY * NZ;
      for (int e = tid; e < rows * NX1; e += kResThreads) {  // global cell starts of the tile rows
        const int t = e / NX1, j = e - t * NX1;
        const int y = Y0 + t % NY, z = Z0 + t / NY;
        tcs[e] = mg.cell_start[(z * mg.g.dims[1] + y) * mg.g.dims[0] + X0 + j];
      }
      __syncthreads();
      if (tid < 64) {  // exclusive prefix of the row point counts (one wave)
        int carry = 0;
        for (int t0 = 0; t0 < rows; t0 += 64) {
          const int t = t0 + tid;
          const int cnt = t < rows ? tcs[t * NX1 + NX1 - 1] - tcs[t * NX1] : 0;
          int inc = cnt;
          for (int d = 1; d < 64; d <<= 1) {
            const int v = __shfl_up(inc, d);
            if (tid >= d) inc += v;
          }
          if (t < rows) rowoff[t] = carry + inc - cnt;
          carry += __shfl(inc, 63);
        }
        if (tid == 0) rowoff[rows] = carry;
      }
      __syncthreads();
      tile = rowoff[rows] <= kTilePts;
      if (tile) {
        // copy the rows' points (coalesced), then turn the cell starts into LDS offsets
        for (int t = 0; t < rows; ++t) {
          const int gb = tcs[t * NX1], n = tcs[t * NX1 + NX1 - 1] - gb, lo = rowoff[t];
          for (int i = tid; i < n; i += kResThreads) tpts[lo + i] = mg.pts[gb + i];
          if (tid == 0) rowgb[t] = gb;
        }
        __syncthreads();
        for (int e = tid; e < rows * NX1; e += kResThreads) {
          const int t = e / NX1;
          tcs[e] = rowoff[t] + (tcs[e] - rowgb[t]);
        }
      }
    }
    __syncthreads();
    if (valid) {
      Knn5 nn;
      unsigned ks[10] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      if (tile) {
        const TileView tv{tpts, tcs, X0, Y0, Z0, NX1, NY};
        knn5_grid<R, RX, false, false, 1, true>(mg, x0, y0, z0, g.crop_min, g.crop_max, bound, nn, ks, nullptr, 0, &tv);
      } else {
        knn5_grid<R, RX, false, false>(mg, x0, y0, z0, g.crop_min, g.crop_max, bound, nn, ks);
      }
      (void)ks;
      const bool ok = nn.k[4] < kKnnEmpty;
      bool same = have_prev && ok && a.fit_cache;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int id = knn_id(nn.k[k]);
        same = same && id == oid[k];
        o[k * kResThreads] = ok ? id : -1;
      }
      a.nsame[(int64_t)it * kResThreads + tid] = same ? 1 : 0;
    }
    __syncthreads();  // the next item reuses the tile
  }
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
// AtA X = AtB.  All 64 lanes of the wave call it; matP / degenerate are written by lane 0.
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

// Two waves per job: wave 0's lanes 0..27 sum the job's item partials (each entry in item order,
// as before); then wave 0's lane 0 solves the normal equations while, at iteration 0, wave 1's
// lane 0 computes the degeneracy projection (the two are independent; on one wave they would run
// back to back); lane 0 then runs the rest of the LMOptimization step.  The number of jobs still
// iterating is accumulated with agent-scope atomics; the last workgroup to finish publishes it to
// host-mapped memory as (generation << 32 | count) so the host stops enqueueing iterations once
// the batch converged.
__global__ void __launch_bounds__(kSolveThreads) k_gn_solve(GnArgs a, int iter_idx, unsigned long long gen) {
  __shared__ double acc[28];
  __shared__ float matP0[36];
  __shared__ int deg0;
  __shared__ EigenLds eig;
  const int job = blockIdx.x, tid = threadIdx.x;
  GnState& g = a.gn[job];
  if (g.active) {  // block-uniform
    const int iter0 = g.iter == 0;  // read before lane 0 updates it (ordered by the barriers)
    if (tid < 28) {
      double sum = 0.0;
      const int i0 = a.item_range[2 * job], i1 = a.item_range[2 * job + 1];
#pragma unroll 8
      for (int it = i0; it < i1; ++it) sum += a.partial[(int64_t)it * kPartial + tid];
      acc[tid] = sum;
    }
    __syncthreads();
    float X[6];
    const bool solve = (int)acc[27] >= 50;
    if (tid >= 64 && iter0 && solve) gn_degeneracy(acc, eig, matP0, &deg0);
    if (tid == 0 && solve) gn_qr_step(acc, X);
    __syncthreads();
    if (tid == 0) gn_solve_job(a, job, acc, X, matP0, deg0);
  }
  if (tid == 0) {
    atomicAdd(&a.iter_cnt[2 * iter_idx], g.active);
    __threadfence();
    const int done = atomicAdd(&a.iter_cnt[2 * iter_idx + 1], 1);
    if (done == a.B - 1) {
      __threadfence();
      const int cnt = atomicAdd(&a.iter_cnt[2 * iter_idx], 0);
      if (a.iter_flags)
        __hip_atomic_store(&a.iter_flags[iter_idx], (gen << 32) | (unsigned long long)cnt, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void k_gn_finalize(GnArgs a) {
  const int job = blockIdx.x * blockDim.x + threadIdx.x;
  if (job >= a.B) return;
  GnState& g = a.gn[job];
  float p[6];
  for (int k = 0; k < 6; ++k) p[k] = g.pose[k];
  if (g.status == FBR_REG_OK) {  // transformUpdate (:1444-1479)
    if (a.desk_mode && (a.desk_mode[job] & kDeskImu))  // cloudInfo.imuAvailable: IMU slerp (:1447-1474)
      imu_slerp_update(p, a.desk[job].imu_roll_init, a.desk[job].imu_pitch_init);
    auto clampf = [](float v, float lim) {
      if (v < -lim) v = -lim;
      if (v > lim) v = lim;
      return v;
    };
    p[0] = clampf(p[0], a.rot_tol);
    p[1] = clampf(p[1], a.rot_tol);
    p[5] = clampf(p[5], a.z_tol);
  }
  for (int k = 0; k < 6; ++k) a.pose_out[job * 6 + k] = p[k];
  fbr_reg_stats& s = a.stats[job];
  s.status = g.status;
  s.iterations = g.iter;
  s.converged = g.converged;
  s.degenerate = g.degenerate;
  s.n_sel = g.n_sel;
  s.n_corner_ds = a.ncds[job];
  s.n_surf_ds = a.nsds[job];
}

// CropBox counts of the global map for every job's box (laserCloud{Corner,Surf}FromMapDSNum,
// statistics only: the registration applies the box per kNN candidate).  The box is the guess's
// translation +- crop_half (registration :289-304), identical to the one k_gn_init stores.
__global__ void k_crop_count(GnArgs a, const float4* pts, int64_t n, int which, int32_t* counts) {
  extern __shared__ int32_t c[];
  for (int j = threadIdx.x; j < a.B; j += blockDim.x) c[j] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = pts[i];
    for (int j = 0; j < a.B; ++j) {
      const float* gp = a.guess + 6 * j;
      const float mn0 = -a.crop_half[0] + gp[3], mn1 = -a.crop_half[1] + gp[4], mn2 = -a.crop_half[2] + gp[5];
      const float mx0 = a.crop_half[0] + gp[3], mx1 = a.crop_half[1] + gp[4], mx2 = a.crop_half[2] + gp[5];
      if (p.x < mn0 || p.y < mn1 || p.z < mn2) continue;
      if (p.x > mx0 || p.y > mx1 || p.z > mx2) continue;
      atomicAdd(&c[j], 1);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.B; j += blockDim.x)
    if (c[j]) atomicAdd(&counts[2 * j + which], c[j]);
}

// 32-byte pose record per job {pose[6], iterations, status} for the cross-GPU gather.
__global__ void k_export_records(int B, const float* pose_out, const fbr_reg_stats* stats, float* dst) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  for (int k = 0; k < 6; ++k) dst[8 * j + k] = pose_out[6 * j + k];
  dst[8 * j + 6] = __int_as_float(stats[j].iterations);
  dst[8 * j + 7] = __int_as_float(stats[j].status);
}

__global__ void k_pack_results(int B, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                               const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf,
                               const int32_t* cropcnt, const int32_t* err, JobResult* out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  JobResult r;
  if (with_reg) {
    for (int k = 0; k < 6; ++k) r.pose[k] = pose_out[6 * j + k];
    r.st = stats[j];
    r.st.n_corner_map = cropcnt[2 * j];
    r.st.n_surf_map = cropcnt[2 * j + 1];
  } else {
    for (int k = 0; k < 6; ++k) r.pose[k] = 0.0f;
    r.st = fbr_reg_stats{};
    r.st.status = FBR_REG_SKIPPED_INTERVAL;
  }
  r.st.n_points = nvalid[j];
  r.st.n_corner = ncorner[j];
  r.st.n_surf = nsurf[j];
  r.err = err[j];
  r.pad = 0;
  out[j] = r;
}

void launch_pack_results(hipStream_t s, int B, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                         const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf, const int32_t* cropcnt,
                         const int32_t* err, JobResult* out) {
  fbr_launch(k_pack_results, dim3((B + 63) / 64), dim3(64), 0, s, B, with_reg, pose_out, stats, nvalid, ncorner, nsurf,
             cropcnt, err, out);
}

void launch_export_records(hipStream_t s, int B, const float* pose_out, const fbr_reg_stats* stats, float* dst) {
  fbr_launch(k_export_records, dim3((B + 63) / 64), dim3(64), 0, s, B, pose_out, stats, dst);
}

void launch_gn_init(hipStream_t s, const GnArgs& a) { fbr_launch(k_gn_init, dim3(1), dim3(1024), 0, s, a); }
template <int R, bool F, bool L, bool S, int LPQ = 1>
void launch_gn_knn_rls(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  const float invx = a.mc.g.inv_x;  // == a.ms.g.inv_x
  grid *= LPQ;
  if (invx > 4.0f) fbr_launch((k_gn_knn<R, 8, F, L, S, LPQ>), dim3(grid), dim3(kResThreads), 0, s, a, use_prev);       // 0.125 m
  else if (invx > 2.0f) fbr_launch((k_gn_knn<R, 4, F, L, S, LPQ>), dim3(grid), dim3(kResThreads), 0, s, a, use_prev);  // 0.25 m
  else if (invx > 1.0f) fbr_launch((k_gn_knn<R, 2, F, L, S, LPQ>), dim3(grid), dim3(kResThreads), 0, s, a, use_prev);  // 0.5 m
  else fbr_launch((k_gn_knn<R, 1, F, L, S, LPQ>), dim3(grid), dim3(kResThreads), 0, s, a, use_prev);                  // >= 1 m
}
// Dense or hashed-chunk map grids (one flag for both maps: fbr_set_map builds them alike).
template <int R, bool F, bool L, int LPQ = 1>
void launch_gn_knn_rl(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  if (a.mc.g.sparse || a.ms.g.sparse) launch_gn_knn_rls<R, F, L, true, LPQ>(s, a, grid, use_prev);
  else launch_gn_knn_rls<R, F, L, false, LPQ>(s, a, grid, use_prev);
}

// Lanes per query of the plain kNN pass (FBR_KNN_LPQ = 1 or 8; default 8 for sub-batches of at
// most 2 jobs, where one lane per query leaves the chip idle and the launch is one query's chain).
int knn_lpq(int jobs) {
  static const int forced = [] {
    const char* e = std::getenv("FBR_KNN_LPQ");
    return e ? (std::atoi(e) >= 8 ? 8 : 1) : 0;
  }();
  if (forced) return forced;
  return jobs <= 2 ? 8 : 1;
}

// Flat row queue (FBR_KNN_FLAT=0 disables): from iteration 1 on (warm-start bound), 1 m y/z cells
// (9 rows: the queue is 18 KB of LDS per workgroup), not in the fused tail launch.
bool knn_flat() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_KNN_FLAT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// LDS map tiles (FBR_KNN_TILE = 0 / 1; default on for dense maps, y/z cells below 1 m, i.e. the
// C3 / C5 mapping leaves): the plain kNN pass on dense grids.
bool knn_tile(const GnArgs& a) {
  static const int forced = [] {
    const char* e = std::getenv("FBR_KNN_TILE");
    return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }();
  if (a.mc.g.sparse || a.ms.g.sparse) return false;
  return forced >= 0 ? forced == 1 : a.mc.g.inv_cell > 1.0f;
}

template <int R, int RX>
void launch_gn_knn_tile(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  fbr_launch((k_gn_knn_tile<R, RX>), dim3(grid), dim3(kResThreads), (uint32_t)(sizeof(float4) * kTilePts), s, a, use_prev);
}

template <int R, bool F>
void launch_gn_knn_r(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  if constexpr (!F) {
    if (knn_lpq(a.B) == 8) return launch_gn_knn_rl<R, F, false, 8>(s, a, grid, use_prev);
    if (knn_tile(a)) {
      const float invx = a.mc.g.inv_x;
      if (invx > 4.0f) return launch_gn_knn_tile<R, 8>(s, a, grid, use_prev);
      if (invx > 2.0f) return launch_gn_knn_tile<R, 4>(s, a, grid, use_prev);
      if (invx > 1.0f) return launch_gn_knn_tile<R, 2>(s, a, grid, use_prev);
      return launch_gn_knn_tile<R, 1>(s, a, grid, use_prev);
    }
  }
  if constexpr (R == 1 && !F) {
    if (use_prev && knn_flat()) return launch_gn_knn_rl<R, F, true>(s, a, grid, use_prev);
  }
  launch_gn_knn_rl<R, F, false>(s, a, grid, use_prev);
}

template <bool F>
void launch_gn_knn_f(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  const float inv = a.mc.g.inv_cell;  // == a.ms.g.inv_cell (fbr_set_map): y / z cells
  if (inv > 2.0f) launch_gn_knn_r<4, F>(s, a, grid, use_prev);       // 0.25 m
  else if (inv > 1.0f) launch_gn_knn_r<2, F>(s, a, grid, use_prev);  // 0.5 m
  else launch_gn_knn_r<1, F>(s, a, grid, use_prev);                  // >= 1 m
}

void launch_gn_knn(hipStream_t s, const GnArgs& a, int grid, int iter, bool fused) {
  const int use_prev = iter > 0;  // nbr holds this launch's previous iteration
  if (fused) launch_gn_knn_f<true>(s, a, grid, use_prev);
  else launch_gn_knn_f<false>(s, a, grid, use_prev);
}
void launch_gn_residual(hipStream_t s, const GnArgs& a, int grid) {
  fbr_launch(k_gn_residual, dim3(grid), dim3(kResThreads), 0, s, a);
}
void launch_gn_solve(hipStream_t s, const GnArgs& a, int iter_idx, unsigned long long gen) {
  fbr_launch(k_gn_solve, dim3(a.B), dim3(kSolveThreads), 0, s, a, iter_idx, gen);
}
void launch_gn_finalize(hipStream_t s, const GnArgs& a) {
  fbr_launch(k_gn_finalize, dim3((a.B + 63) / 64), dim3(64), 0, s, a);
}
void launch_crop_count(hipStream_t s, const GnArgs& a, const float4* pts, int64_t n, int which, int32_t* counts) {
  if (n <= 0) return;
  int grid = (int)std::min<int64_t>((n + 255) / 256, 1024);
  fbr_launch(k_crop_count, dim3(grid), dim3(256), sizeof(int32_t) * a.B, s, a, pts, n, which, counts);
}

}  // namespace fbr

#ifdef FBR_KNN_STATS
// Diagnostic builds only: read (and optionally reset) the kNN counters of k_gn_knn.
extern "C" int fbr_diag_knn_stats(unsigned long long* out, int reset) {
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(fbr::fbr_knn_stats), sizeof(unsigned long long) * 10) != hipSuccess)
    return FBR_ERR_HIP;
  if (reset) {
    unsigned long long z[10] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(fbr::fbr_knn_stats), z, sizeof(z)) != hipSuccess) return FBR_ERR_HIP;
  }
  return FBR_OK;
}
#endif
