// k_knn_tile.hip — LDS-staged map tiles for the neighbour search on dense maps (north_star: "LDS-
// staged map tiles for the neighbour search"; BASELINE configs[2] / configs[4]).
//
// Reference: /root/reference/src/mapOptmization.h:1143 (surf kdtree->nearestKSearch(pointSel, 5)),
// :1022 (corner), :1413-1414 (the per-scan KD-tree builds on the cropped local maps).
//
// The global grid (k_grid.hip) has 0.5 m y/z x 0.125 m x cells on dense maps.  At C5's density
// (mapping leaves 0.05 m: ~400 map points per m^2 of surface) a query's pruned search still walks
// ~140 points, because a grid row is 0.5 m x 0.5 m in cross-section; finer global cells need
// 4x-16x more rows per query and measured 2-6x slower.  From the second
// Gauss-Newton iteration on, every query knows an upper bound of its 5th-neighbour distance (its
// previous neighbours, `bound` in knn5_grid), typically ~0.05 m on these maps.  So:
//   * one 64-lane workgroup serves 64 consecutive queries of a work item (Morton order: a compact
//     patch of the scan);
//   * the wave's tile box is the union of its queries' bound boxes in FINE cells (0.125 m cubes);
//   * the tile is loaded once from the global grid rows that overlap the box (coalesced), keeping
//     only the points inside the box and inside the job's CropBox, and counting-sorted into the fine
//     cells in LDS (<= 512 points, <= 512 cells: 10 KB);
//   * each query then walks only the fine cells of its own bound box, out of LDS, with no CropBox
//     test per point (the tile holds in-box points only): ~6-25 points instead of ~140.
// Lanes whose bound is missing (no previous neighbours), too large (> `reach` fine cells), or whose
// tile does not fit, are queued (fb_list) and a second launch runs the global search (knn5_grid)
// on the queue, so they do not hold up the waves the tiles serve.
//
// Exactness.  The scanned set of every query still contains every crop-box point whose computed d2
// is <= bound: a point with fl(q - p)^2 summed <= bound has |q_x - p_x| <= sqrt(bound) (1 + 2^-22)
// per axis, and the box edge fl(q_x - r_up) with r_up = sqrtf(bound) * (1 + 2^-7) + 1e-6 (1 + |q|)
// stays below p_x (the margins exceed every rounding involved), so floor(p_x * inv_f), an exact
// power-of-two scaling, lies in the query's cell range.  The 5-NN list (5 smallest (d2, index)
// keys with d2 < 1.0) is a function of the scanned set once that set holds the true 5 nearest, so
// the neighbours are bit-identical to the global search's (`test_knn_tile_is_bit_identical`).
#include "fbr_gn.h"

namespace fbr {

namespace {
constexpr int kTileLoadRows = 16;  // global grid rows a tile may be loaded from
constexpr int kTileLoadMax = 8192; // points a tile load may scan
}  // namespace

// PTS map points, CELLS fine cells per wave tile
template <int PTS, int CELLS>
struct TileLds {
  float4 pts[PTS];                // the tile's points, by fine cell (w = map index bits)
  uint32_t cs[CELLS];             // per-cell counts -> starts -> ends (cs[c] = end of cell c)
  int2 rows[kTileLoadRows];       // global point ranges of the tile load
  int rpre[kTileLoadRows + 1];    // their running lengths
};

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Fine-cell coordinate of a metric coordinate (inv_f a power of two: the product is exact).
__device__ __forceinline__ int fine(float x, float inv_f) { return (int)floorf(x * inv_f); }

// Global cells [g0, g1] covering fine cells [f0, f1] (s = log2(global cell / fine cell): 2^s fine
// cells nest in a global cell when s >= 0, a fine cell spans 2^-s global cells when s < 0).
__device__ __forceinline__ void fine_to_global(int f0, int f1, int s, int& g0, int& g1) {
  if (s >= 0) {
    g0 = f0 >> s;  // arithmetic shift: floor
    g1 = f1 >> s;
  } else {
    g0 = f0 * (1 << -s);
    g1 = (f1 + 1) * (1 << -s) - 1;
  }
}

// Load the map points of fine-cell box [X0, X0 + Dx) x [Y0, Y0 + Dy) x [Z0, Z0 + Dz) that lie
// inside the CropBox into T, counting-sorted by fine cell (T.cs[c] = end of cell c).  Wave-uniform
// result: false when the box, its global rows or its points exceed the tile.
template <int PTS, int CELLS>
__device__ bool tile_build(TileLds<PTS, CELLS>& T, const MapGrid& mg, int X0, int Y0, int Z0, int Dx, int Dy, int Dz,
                           float inv_f, int sx, int sy, const float* bmin, const float* bmax,
                           unsigned long long* tile_stats) {
  const int lane = threadIdx.x;
  const bool small = Dx <= CELLS && Dy <= CELLS && Dz <= CELLS && (int64_t)Dx * Dy * Dz <= CELLS;
  const int ncell = small ? Dx * Dy * Dz : CELLS + 1;
  // global cells holding the box (fine_to_global: x by sx, y and z by sy)
  int ax, bx, ay, by, az, bz;
  fine_to_global(X0, X0 + Dx - 1, sx, ax, bx);
  fine_to_global(Y0, Y0 + Dy - 1, sy, ay, by);
  fine_to_global(Z0, Z0 + Dz - 1, sy, az, bz);
  const int gx0 = max(ax - (int)mg.g.origin[0], 0), gx1 = min(bx - (int)mg.g.origin[0], mg.g.dims[0] - 1);
  const int gy0 = max(ay - (int)mg.g.origin[1], 0), gy1 = min(by - (int)mg.g.origin[1], mg.g.dims[1] - 1);
  const int gz0 = max(az - (int)mg.g.origin[2], 0), gz1 = min(bz - (int)mg.g.origin[2], mg.g.dims[2] - 1);
  const int ny = gy1 - gy0 + 1, nz = gz1 - gz0 + 1;
  const int nrows = (gx0 <= gx1 && ny > 0 && nz > 0) ? ny * nz : 0;
  if (!(ncell <= CELLS && nrows <= kTileLoadRows)) {
    if (tile_stats && lane == 0) atomicAdd(&tile_stats[5], 1ull);
    return false;
  }
  int len = 0;
  if (lane < nrows) {
    const int y = gy0 + lane % ny, z = gz0 + lane / ny;
    const int rowbase = (z * mg.g.dims[1] + y) * mg.g.dims[0];
    const int b = mg.cell_start[rowbase + gx0], e = mg.cell_start[rowbase + gx1 + 1];
    T.rows[lane] = make_int2(b, e);
    len = e - b;
  }
  int inc = len;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(inc, off);
    if (lane >= off) inc += y;
  }
  if (lane < nrows) T.rpre[lane + 1] = inc;
  if (lane == 0) T.rpre[0] = 0;
  const int L = __shfl(inc, 63);
  if (L > kTileLoadMax) {
    if (tile_stats && lane == 0) atomicAdd(&tile_stats[6], 1ull);
    return false;
  }
  for (int c = lane; c < ncell; c += 64) T.cs[c] = 0u;
  __syncthreads();
  const float bx0 = bmin[0], by0 = bmin[1], bz0 = bmin[2], bx1 = bmax[0], by1 = bmax[1], bz1 = bmax[2];
  // pass 1: per-cell counts of the points inside the box and the CropBox
  int j = 0;
  for (int t = lane; t < L; t += 64) {
    while (T.rpre[j + 1] <= t) ++j;
    const float4 q = mg.pts[T.rows[j].x + (t - T.rpre[j])];
    const int cx = fine(q.x, inv_f) - X0, cy = fine(q.y, inv_f) - Y0, cz = fine(q.z, inv_f) - Z0;
    const bool in = (unsigned)cx < (unsigned)Dx && (unsigned)cy < (unsigned)Dy && (unsigned)cz < (unsigned)Dz &&
                    !((q.x < bx0) | (q.y < by0) | (q.z < bz0) | (q.x > bx1) | (q.y > by1) | (q.z > bz1));
    if (in) atomicAdd(&T.cs[cx + Dx * (cy + Dy * cz)], 1u);
  }
  __syncthreads();
  // exclusive starts, 64 cells per step (a wave scan plus the running carry)
  uint32_t carry = 0;
  for (int c0 = 0; c0 < ncell; c0 += 64) {
    const int c = c0 + lane;
    const uint32_t n = c < ncell ? T.cs[c] : 0u;
    uint32_t incs = n;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incs, off);
      if (lane >= off) incs += y;
    }
    if (c < ncell) T.cs[c] = carry + incs - n;
    carry += __shfl(incs, 63);
  }
  if (carry > (uint32_t)PTS) {
    if (tile_stats && lane == 0) atomicAdd(&tile_stats[7], 1ull);
    __syncthreads();
    return false;
  }
  const uint32_t total = carry;
  __syncthreads();
  // pass 2: scatter (cs[c] ends as the end of cell c)
  j = 0;
  for (int t = lane; t < L; t += 64) {
    while (T.rpre[j + 1] <= t) ++j;
    const float4 q = mg.pts[T.rows[j].x + (t - T.rpre[j])];
    const int cx = fine(q.x, inv_f) - X0, cy = fine(q.y, inv_f) - Y0, cz = fine(q.z, inv_f) - Z0;
    const bool in = (unsigned)cx < (unsigned)Dx && (unsigned)cy < (unsigned)Dy && (unsigned)cz < (unsigned)Dz &&
                    !((q.x < bx0) | (q.y < by0) | (q.z < bz0) | (q.x > bx1) | (q.y > by1) | (q.z > bz1));
    if (in) T.pts[atomicAdd(&T.cs[cx + Dx * (cy + Dy * cz)], 1u)] = q;
  }
  __syncthreads();
  if (tile_stats && lane == 0) {
    atomicAdd(&tile_stats[2], 1ull);
    atomicAdd(&tile_stats[3], (unsigned long long)total);
  }
  return true;
}

// sx / sy: log2(inv_f / inv_x), log2(inv_f / inv_cell) (fine_to_global).  Clusters: the eligible
// lanes are served in up to kRounds tiles, each around the lowest still-pending lane (the anchor):
// lanes whose bound box lies within `span` fine cells of the anchor's join its tile, so one far
// query (Morton order jumps between octree blocks) does not blow up the box of the others.
// tile_stats (diagnostic, may be null): [queries, tile-served, tile loads, points loaded, tile
// fails, of which: box over CELLS cells or kTileLoadRows rows, load over kTileLoadMax, over PTS].
template <int R, int RX, int PTS, int CELLS>
__global__ void __launch_bounds__(64) k_gn_knn_tile(GnArgs a, int iter, float inv_f, int sx, int sy, float rmax2,
                                                   int span, int rounds, unsigned long long* tile_stats) {
  static_assert(CELLS % 64 == 0 && CELLS <= 4096, "cell starts: CELLS / 64 per lane");
  __shared__ TileLds<PTS, CELLS> T;
  const int lane = threadIdx.x;
  const int nitems = a.nitems[0];
  for (int v = blockIdx.x; v < nitems * 4; v += gridDim.x) {
    const int it = v >> 2, tid = (v & 3) * 64 + lane;
    const int4 item = a.items[it];
    const int job = item.x;
    const GnState& g = a.gn[job];
    if (!g.active) continue;  // block-uniform
    const bool corner = item.y == 0;
    const MapGrid& mg = corner ? a.mc : a.ms;
    const bool has_q = tid < item.w;
    // ---- the query, its previous neighbours and bound (gn_knn_block's arithmetic) ----
    float x0 = 0.0f, y0 = 0.0f, z0 = 0.0f, bound = __int_as_float(0x7f800000);
    int32_t oid[5] = {-1, -1, -1, -1, -1};
    int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
    bool have_prev = false;
    if (has_q) {
      const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
      const float* Tm = g.T;
      x0 = Tm[0] * p.x + Tm[1] * p.y + Tm[2] * p.z + Tm[3];
      y0 = Tm[4] * p.x + Tm[5] * p.y + Tm[6] * p.z + Tm[7];
      z0 = Tm[8] * p.x + Tm[9] * p.y + Tm[10] * p.z + Tm[11];
      have_prev = o[0] >= 0;
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
    }
    const bool el = has_q && have_prev && bound <= rmax2;
    int lx0 = 0, lx1 = -1, ly0 = 0, ly1 = -1, lz0 = 0, lz1 = -1;
    if (el) {
      const float r_up = sqrtf(bound) * 1.0078125f + 1e-6f * (1.0f + fabsf(x0) + fabsf(y0) + fabsf(z0));
      lx0 = fine(x0 - r_up, inv_f); lx1 = fine(x0 + r_up, inv_f);
      ly0 = fine(y0 - r_up, inv_f); ly1 = fine(y0 + r_up, inv_f);
      lz0 = fine(z0 - r_up, inv_f); lz1 = fine(z0 + r_up, inv_f);
    }
    Knn5 nn;
#pragma unroll
    for (int t = 0; t < 5; ++t) nn.k[t] = kKnnEmpty;
    bool served = false;
    uint64_t pending = __ballot(el);
    for (int rd = 0; rd < rounds && pending; ++rd) {
      // ---- this round's cluster and its tile box (fine cells) ----
      const int an = __ffsll((unsigned long long)pending) - 1;
      const int ax0 = __shfl(lx0, an), ax1 = __shfl(lx1, an), ay0 = __shfl(ly0, an), ay1 = __shfl(ly1, an);
      const int az0 = __shfl(lz0, an), az1 = __shfl(lz1, an);
      const bool mine = ((pending >> lane) & 1ull) && lx0 >= ax0 - span && lx1 <= ax1 + span && ly0 >= ay0 - span &&
                        ly1 <= ay1 + span && lz0 >= az0 - span && lz1 <= az1 + span;
      const uint64_t cl = __ballot(mine);  // holds the anchor
      pending &= ~cl;
      const int big = 0x3fffffff;
      const int X0 = wave_min_i(mine ? lx0 : big), Y0 = wave_min_i(mine ? ly0 : big), Z0 = wave_min_i(mine ? lz0 : big);
      const int Dx = wave_max_i(mine ? lx1 : -big) - X0 + 1, Dy = wave_max_i(mine ? ly1 : -big) - Y0 + 1;
      const int Dz = wave_max_i(mine ? lz1 : -big) - Z0 + 1;
      if (!tile_build(T, mg, X0, Y0, Z0, Dx, Dy, Dz, inv_f, sx, sy, g.crop_min, g.crop_max, tile_stats)) {
        if (tile_stats && lane == 0) atomicAdd(&tile_stats[4], 1ull);
        continue;  // the cluster's lanes take the global search
      }
      // ---- the tile search: the lane's fine rows (y, z), each one contiguous x-cell range ----
      if (mine) {
        served = true;
        const int nyr = ly1 - ly0 + 1, nr = nyr * (lz1 - lz0 + 1);
        int r = 0, i = 0, e = 0;
        while (true) {
          if (i >= e) {
            if (r >= nr) break;
            const int y = ly0 + r % nyr - Y0, z = lz0 + r / nyr - Z0;
            const int base = Dx * (y + Dy * z);
            const int ca = base + (lx0 - X0), cb = base + (lx1 - X0);
            i = ca ? (int)T.cs[ca - 1] : 0;
            e = (int)T.cs[cb];
            ++r;
            continue;
          }
          const float4 q = T.pts[i++];
          float dist = 0.0f, diff;
          diff = x0 - q.x; dist += diff * diff;  // flann::L2_Simple
          diff = y0 - q.y; dist += diff * diff;
          diff = z0 - q.z; dist += diff * diff;
          knn_insert(nn, ((unsigned long long)(unsigned)__float_as_int(dist) << 32) | (unsigned)__float_as_int(q.w));
        }
      }
      __syncthreads();  // the next round rebuilds the tile
    }
    // queries not served here are queued for the grid search (k_gn_knn_list), one atomic per wave
    const bool fb = has_q && !served;
    const uint64_t fbm = __ballot(fb);
    if (fbm) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&a.iter_cnt[2 * max(1, a.max_iter) + iter], __popcll(fbm));
      base = __shfl(base, 0);
      if (fb) a.fb_list[base + __popcll(fbm & ((1ull << lane) - 1ull))] = it * kResThreads + tid;
    }
    if (tile_stats) {
      const uint64_t hq = __ballot(has_q), sv = __ballot(served);
      if (lane == 0) {
        atomicAdd(&tile_stats[0], (unsigned long long)__popcll(hq));
        atomicAdd(&tile_stats[1], (unsigned long long)__popcll(sv));
      }
    }
    if (served) {
      const bool ok = nn.k[4] < kKnnEmpty;
      int32_t ids[5];
      bool same = ok && a.fit_cache;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        ids[k] = knn_id(nn.k[k]);
        same = same && ids[k] == oid[k];
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) o[k * kResThreads] = ok ? ids[k] : -1;
      a.nsame[(int64_t)it * kResThreads + tid] = same ? 1 : 0;
    }
    __syncthreads();  // the next virtual block reuses the tile
  }
}

// The grid search (knn5_grid, gn_knn_block's per-query body) for the query slots the tile kernel
// queued (fb_list[0, count), it * 256 + slot, in arrival order: each query's result depends on the
// query only).  Lanes take consecutive list entries.
template <int R, int RX>
__global__ void __launch_bounds__(256) k_gn_knn_list(GnArgs a, int iter) {
  const int n = a.iter_cnt[2 * max(1, a.max_iter) + iter];
  for (int q = blockIdx.x * 256 + threadIdx.x; q < n; q += gridDim.x * 256) {
    const int id = a.fb_list[q];
    const int it = id / kResThreads, tid = id % kResThreads;
    const int4 item = a.items[it];
    const int job = item.x;
    const GnState& g = a.gn[job];
    const bool corner = item.y == 0;
    const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
    const float* T = g.T;
    const float x0 = T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3];
    const float y0 = T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7];
    const float z0 = T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11];
    const MapGrid& mg = corner ? a.mc : a.ms;
    int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
    float bound = __int_as_float(0x7f800000);
    int32_t oid[5] = {-1, -1, -1, -1, -1};
    const bool have_prev = o[0] >= 0;
    if (have_prev) {
      float mx = 0.0f;
#pragma unroll
      for (int k = 0; k < 5; ++k) oid[k] = o[k * kResThreads];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float4 m = mg.by_id[oid[k]];
        float dist = 0.0f, diff;
        diff = x0 - m.x; dist += diff * diff;
        diff = y0 - m.y; dist += diff * diff;
        diff = z0 - m.z; dist += diff * diff;
        mx = fmaxf(mx, dist);
      }
      bound = mx;
    }
    Knn5 nn;
    unsigned ks[10] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    knn5_grid<R, RX, false, false, 1>(mg, x0, y0, z0, g.crop_min, g.crop_max, bound, nn, ks);
    (void)ks;
    const bool ok = nn.k[4] < kKnnEmpty;
    int32_t ids[5];
    bool same = have_prev && ok && a.fit_cache;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      ids[k] = knn_id(nn.k[k]);
      same = same && ids[k] == oid[k];
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k * kResThreads] = ok ? ids[k] : -1;
    a.nsame[(int64_t)it * kResThreads + tid] = same ? 1 : 0;
  }
}

// FBR_KNN_TILE: 1 serves iterations >= 1 on dense 0.5 m x 0.125 m grids from wave tiles; 0 (the
// default until the tiles measure faster) keeps the global search.  FBR_KNN_TILE_CELL: the fine cell (m, power of two, default 0.125);
// FBR_KNN_TILE_REACH: the largest bound served, in fine cells (default 1).
static bool knn_tile_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_KNN_TILE");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}
static float knn_tile_inv() {
  static const float v = [] {
    const char* e = std::getenv("FBR_KNN_TILE_CELL");
    const float c = e ? std::strtof(e, nullptr) : 0.125f;
    return c > 0.0f ? std::exp2(-std::round(std::log2(c))) : 8.0f;
  }();
  return v;
}

unsigned long long* knn_tile_stats_buffer();

bool launch_gn_knn_tile(hipStream_t s, const GnArgs& a, int grid, int iter) {
  if (iter <= 0 || !knn_tile_enabled() || a.mc.g.sparse || a.ms.g.sparse) return false;
  const float inv_x = a.mc.g.inv_x, inv = a.mc.g.inv_cell;
  if (inv_x != 8.0f || inv != 2.0f) return false;  // instantiated for the dense-map cells (R = 2, RX = 8)
  const float inv_f = knn_tile_inv();
  if (inv_f < 0.5f || inv_f > 64.0f) return false;
  const int sx = (int)std::lround(std::log2(inv_f / inv_x)), sy = (int)std::lround(std::log2(inv_f / inv));
  static const float reach = [] {
    const char* e = std::getenv("FBR_KNN_TILE_REACH");
    const float r = e ? std::strtof(e, nullptr) : 1.0f;
    return r > 0.0f ? std::min(r, 4.0f) : 1.0f;
  }();
  const float rmax2 = reach * reach / (inv_f * inv_f);  // bound boxes up to `reach` fine cells
  const int g4 = (int)std::min<int64_t>((int64_t)grid * 4, 1 << 20);
  static const int cap = [] {  // tile capacity (FBR_KNN_TILE_CAP): 0 512 points / 512 cells, 1 1024 / 1024, 2 2048 / 2048
    const char* e = std::getenv("FBR_KNN_TILE_CAP");
    return e ? std::max(0, std::min(2, std::atoi(e))) : 1;
  }();
  static const int span = [] {  // cluster reach around the anchor's box, fine cells (FBR_KNN_TILE_SPAN)
    const char* e = std::getenv("FBR_KNN_TILE_SPAN");
    return e ? std::max(0, std::atoi(e)) : 3;
  }();
  static const int rounds = [] {  // tiles per wave (FBR_KNN_TILE_ROUNDS)
    const char* e = std::getenv("FBR_KNN_TILE_ROUNDS");
    return e ? std::max(1, std::min(64, std::atoi(e))) : 4;
  }();
  unsigned long long* st = knn_tile_stats_buffer();
  if (cap == 0)
    fbr_launch((k_gn_knn_tile<2, 8, 512, 512>), dim3(g4), dim3(64), 0, s, a, iter, inv_f, sx, sy, rmax2, span, rounds, st);
  else if (cap == 1)
    fbr_launch((k_gn_knn_tile<2, 8, 1024, 1024>), dim3(g4), dim3(64), 0, s, a, iter, inv_f, sx, sy, rmax2, span, rounds, st);
  else
    fbr_launch((k_gn_knn_tile<2, 8, 2048, 2048>), dim3(g4), dim3(64), 0, s, a, iter, inv_f, sx, sy, rmax2, span, rounds, st);
  fbr_launch((k_gn_knn_list<2, 8>), dim3(std::max(1, grid)), dim3(256), 0, s, a, iter);
  return true;
}

// Diagnostic counters (FBR_KNN_TILE_STATS=1): allocated once, null otherwise.
unsigned long long* knn_tile_stats_buffer() {
  static unsigned long long* p = [] {
    const char* e = std::getenv("FBR_KNN_TILE_STATS");
    if (!e || std::atoi(e) == 0) return (unsigned long long*)nullptr;
    unsigned long long* q = nullptr;
    if (hipMalloc(&q, sizeof(unsigned long long) * 8) != hipSuccess) return (unsigned long long*)nullptr;
    if (hipMemset(q, 0, sizeof(unsigned long long) * 8) != hipSuccess) return (unsigned long long*)nullptr;
    return q;
  }();
  return p;
}

}  // namespace fbr

// [queries, tile-served queries, tile loads, points loaded into tiles, tile failures, of which box
// too large / load too long / too many points] since the last reset; -1 when the counters are off
// (FBR_KNN_TILE_STATS unset).
extern "C" int fbr_diag_knn_tile_stats(unsigned long long* out, int reset) {
  unsigned long long* p = fbr::knn_tile_stats_buffer();
  if (!p) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out, p, sizeof(unsigned long long) * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (reset && hipMemset(p, 0, sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  return 0;
}
