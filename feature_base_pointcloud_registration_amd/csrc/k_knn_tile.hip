// k_knn_tile.hip — query-binned LDS map tiles for the neighbour search on dense maps (north_star:
// "LDS-staged map tiles for the neighbour search"; BASELINE configs[2] / configs[4]).
//
// Reference: /root/reference/src/mapOptmization.h:1143 (surf kdtree->nearestKSearch(pointSel, 5)),
// :1022 (corner), :1413-1414 (the per-scan KD-tree builds on the cropped local maps).
//
// The global grid (k_grid.hip) has 0.5 m y/z x 0.125 m x cells on dense maps.  At C5's density
// (mapping leaves 0.05 m, ~400 map points per m^2 of surface) a query's pruned search still walks
// ~140 points, because a grid row is 0.5 m x 0.5 m in cross-section; finer global cells need
// 4-16x more unrolled rows per query and measured 2-6x slower.  From the second
// Gauss-Newton iteration on, every query knows an upper bound of its 5th-neighbour distance (the
// distance to its previous neighbours, `bound` in knn5_grid), mostly below 0.125 m on these maps.
// The jobs of a batch share the map, so the queries of all jobs are binned by map block:
//   k_bin_count    one lane per query: bound, block (0.5 m cube = 4 x 4 x 4 fine 0.125 m cells of
//                  the grid) when the query's bound box stays within its block +- one fine cell,
//                  else the query is queued for the grid search (fb_list); per-block counts and the
//                  list of non-empty blocks;
//   k_bin_scan     one workgroup: exclusive scan of the non-empty blocks' counts -> cursors;
//   k_bin_scatter  one lane per binned query: its slot in its block's run of the query list;
//   k_bin_tile     one workgroup per non-empty block: the map points of the block +- one fine cell
//                  (6^3 fine cells, from 9 global rows) are loaded once into LDS, counting-sorted by
//                  fine cell, and every query of the block (all jobs) walks only the fine cells of
//                  its own bound box: ~10-30 points instead of ~140, each an LDS read;
//   k_gn_knn_list  the grid search for the queued queries.
// Queries of different jobs share a tile, so a job's CropBox is tested per point unless the tile
// lies inside it (then never).
//
// Exactness.  The scanned set of every query still contains every crop-box point whose computed d2
// is <= bound: a point with fl(q - p)^2 summed <= bound has |q_x - p_x| <= sqrt(bound) (1 + 2^-22)
// per axis, and the box edge fl(q_x - r_up) with r_up = sqrtf(bound) * (1 + 2^-7) + 1e-6 (1 + |q|)
// stays below p_x (the margins exceed every rounding involved), so floor(p_x * 8), an exact
// power-of-two scaling, lies in the query's cell range.  The 5-NN list (5 smallest (d2, index)
// keys with d2 < 1.0) is a function of the scanned set once that set holds the true 5 nearest, so
// the neighbours are bit-identical to the grid search's (`test_knn_tile_is_bit_identical...`).
#include "fbr_gn.h"

namespace fbr {

namespace {
constexpr int kBinThreads = 256;
constexpr int kTilePts = 2048;     // map points per block tile (32 KB)
constexpr int kTileSide = 6;       // fine cells per side: the block's 4 + one on each side
constexpr int kTileCells = kTileSide * kTileSide * kTileSide;
constexpr float kFineInv = 8.0f;   // fine cell 0.125 m (= the grid's x cell; 4 per y / z cell)
}  // namespace

struct BinTileLds {
  float4 pts[kTilePts];               // the tile's points, by fine cell (w = map index bits)
  uint32_t cs[kTileCells];            // per-cell counts -> starts -> ends (cs[c] = end of cell c)
  int2 rows[9];                       // the 3 x 3 global rows of the load
  int rpre[10];                       // their running lengths
  uint32_t wsum[kBinThreads / 64];
};

__device__ __forceinline__ int fine8(float x) { return (int)floorf(x * kFineInv); }

// The query of slot (it, tid) at the job's current pose and its warm-start bound (the largest
// distance to its previous 5 neighbours; +inf without them): gn_knn_block's arithmetic.
struct BinQuery {
  float x0, y0, z0, bound;
  int32_t oid[5];
  bool have_prev;
};
__device__ __forceinline__ void bin_query(const GnArgs& a, int it, int tid, const int4& item, const GnState& g,
                                          BinQuery& q) {
  const int job = item.x;
  const bool corner = item.y == 0;
  const float4 p = corner ? a.cornerDS[job * a.capc + item.z + tid] : a.surfDS[job * a.caps + item.z + tid];
  const float* T = g.T;
  q.x0 = T[0] * p.x + T[1] * p.y + T[2] * p.z + T[3];
  q.y0 = T[4] * p.x + T[5] * p.y + T[6] * p.z + T[7];
  q.z0 = T[8] * p.x + T[9] * p.y + T[10] * p.z + T[11];
  const int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
  q.have_prev = o[0] >= 0;
  q.bound = __int_as_float(0x7f800000);
#pragma unroll
  for (int k = 0; k < 5; ++k) q.oid[k] = -1;
  if (q.have_prev) {
    const float4* by_id = corner ? a.mc.by_id : a.ms.by_id;
    float mx = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) q.oid[k] = o[k * kResThreads];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const float4 m = by_id[q.oid[k]];
      float dist = 0.0f, diff;
      diff = q.x0 - m.x; dist += diff * diff;
      diff = q.y0 - m.y; dist += diff * diff;
      diff = q.z0 - m.z; dist += diff * diff;
      mx = fmaxf(mx, dist);
    }
    q.bound = mx;
  }
}

// Fine-cell bound box of a query (absolute fine coordinates).
__device__ __forceinline__ void bin_box(const BinQuery& q, int* lo, int* hi) {
  const float r_up = sqrtf(q.bound) * 1.0078125f + 1e-6f * (1.0f + fabsf(q.x0) + fabsf(q.y0) + fabsf(q.z0));
  lo[0] = fine8(q.x0 - r_up); hi[0] = fine8(q.x0 + r_up);
  lo[1] = fine8(q.y0 - r_up); hi[1] = fine8(q.y0 + r_up);
  lo[2] = fine8(q.z0 - r_up); hi[2] = fine8(q.z0 + r_up);
}

// Blocks of a map grid along x (4 x cells each); y / z: one per grid cell.
__device__ __forceinline__ int bin_nbx(const MapGrid& m) { return (m.g.dims[0] + 3) >> 2; }

// The query's result: the neighbour map indices (slot 0 = -1: no correspondence) and the
// same-as-previous flag of the fit cache.
__device__ __forceinline__ void bin_write(const GnArgs& a, int it, int tid, const BinQuery& q, const Knn5& nn) {
  int32_t* o = a.nbr + (int64_t)it * 5 * kResThreads + tid;
  const bool ok = nn.k[4] < kKnnEmpty;
  int32_t ids[5];
  bool same = q.have_prev && ok && a.fit_cache;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    ids[k] = knn_id(nn.k[k]);
    same = same && ids[k] == q.oid[k];
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) o[k * kResThreads] = ok ? ids[k] : -1;
  a.nsame[(int64_t)it * kResThreads + tid] = same ? 1 : 0;
}

// Per-sub counters in iter_cnt: [2 mi] solve, [mi] queued queries, [mi] non-empty blocks.
__device__ __forceinline__ int32_t* fb_count(const GnArgs& a, int iter) {
  return a.iter_cnt + 2 * max(1, a.max_iter) + iter;
}
__device__ __forceinline__ int32_t* ne_count(const GnArgs& a, int iter) {
  return a.iter_cnt + 3 * max(1, a.max_iter) + iter;
}

// Queue the flagged lanes' slots for the grid search (one atomic per wave).
__device__ __forceinline__ void queue_fallback(const GnArgs& a, int iter, bool fb, int v) {
  const uint64_t m = __ballot(fb);
  if (!m) return;
  const int lane = threadIdx.x & 63, lead = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == lead) base = atomicAdd(fb_count(a, iter), __popcll(m));
  base = __shfl(base, lead);
  if (fb) a.fb_list[base + __popcll(m & ((1ull << lane) - 1ull))] = v;
}

// tile_stats (diagnostic, may be null): [queries, binned queries, tiles built, points in tiles,
// points scanned by the tile loads, tiles over capacity].
__global__ void __launch_bounds__(kBinThreads) k_bin_count(GnArgs a, int iter, float rmax2,
                                                          unsigned long long* tile_stats) {
  const int nitems = a.nitems[0];
  const int nb_c = a.nb_c;
  int32_t* cnt = a.bin;
  int32_t* ne = a.bin + 2 * (a.nb_c + a.nb_s);
  for (int64_t v0 = (int64_t)blockIdx.x * kBinThreads; v0 < (int64_t)nitems * kResThreads;
       v0 += (int64_t)gridDim.x * kBinThreads) {
    const int v = (int)v0 + (int)threadIdx.x;  // kBinThreads == kResThreads: v < nitems * 256
    const int it = v / kResThreads, tid = v % kResThreads;
    const int4 item = a.items[it];
    const GnState& g = a.gn[item.x];
    const bool has_q = g.active && tid < item.w;
    int blk = -1;
    if (has_q) {
      BinQuery q;
      bin_query(a, it, tid, item, g, q);
      if (q.have_prev && q.bound <= rmax2) {
        const bool corner = item.y == 0;
        const MapGrid& mg = corner ? a.mc : a.ms;
        int lo[3], hi[3];
        bin_box(q, lo, hi);
        const int ox = (int)mg.g.origin[0], oy = (int)mg.g.origin[1], oz = (int)mg.g.origin[2];
        // the block of the query's fine cell (grid-relative: x cells / 4, y / z cells)
        const int bx = (fine8(q.x0) - ox) >> 2, by = (fine8(q.y0) >> 2) - oy, bz = (fine8(q.z0) >> 2) - oz;
        const int nbx = bin_nbx(mg);
        const bool in_grid = bx >= 0 && bx < nbx && by >= 0 && by < mg.g.dims[1] && bz >= 0 && bz < mg.g.dims[2];
        const int fx0 = 4 * bx + ox, fy0 = 4 * (by + oy), fz0 = 4 * (bz + oz);  // the block's first fine cells
        const bool fits = lo[0] >= fx0 - 1 && hi[0] <= fx0 + 4 && lo[1] >= fy0 - 1 && hi[1] <= fy0 + 4 &&
                          lo[2] >= fz0 - 1 && hi[2] <= fz0 + 4;
        if (in_grid && fits) blk = (corner ? 0 : nb_c) + (bz * mg.g.dims[1] + by) * nbx + bx;
      }
    }
    a.qblk[v] = blk;
    if (blk >= 0 && atomicAdd(&cnt[blk], 1) == 0) ne[atomicAdd(ne_count(a, iter), 1)] = blk;
    queue_fallback(a, iter, has_q && blk < 0, v);
    if (tile_stats) {
      const uint64_t hq = __ballot(has_q), bq = __ballot(blk >= 0);
      if ((threadIdx.x & 63) == 0) {
        atomicAdd(&tile_stats[0], (unsigned long long)__popcll(hq));
        atomicAdd(&tile_stats[1], (unsigned long long)__popcll(bq));
      }
    }
  }
}

// Exclusive scan of the non-empty blocks' counts (one 1024-thread workgroup): cur[b] = first slot.
__global__ void __launch_bounds__(1024) k_bin_scan(GnArgs a, int iter) {
  __shared__ int32_t wsum[16];
  const int n = *ne_count(a, iter);
  const int32_t* cnt = a.bin;
  int32_t* cur = a.bin + (a.nb_c + a.nb_s);
  const int32_t* ne = a.bin + 2 * (a.nb_c + a.nb_s);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int carry = 0;
  for (int i0 = 0; i0 < n; i0 += 1024) {
    const int i = i0 + tid;
    const int b = i < n ? ne[i] : -1;
    const int c = b >= 0 ? cnt[b] : 0;
    int inc = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int pre = carry, tot = 0;
    for (int k = 0; k < 16; ++k) {
      if (k < w) pre += wsum[k];
      tot += wsum[k];
    }
    if (b >= 0) cur[b] = pre + inc - c;
    carry += tot;
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kBinThreads) k_bin_scatter(GnArgs a) {
  const int nitems = a.nitems[0];
  int32_t* cur = a.bin + (a.nb_c + a.nb_s);
  for (int64_t v = (int64_t)blockIdx.x * kBinThreads + threadIdx.x; v < (int64_t)nitems * kResThreads;
       v += (int64_t)gridDim.x * kBinThreads) {
    const int b = a.qblk[v];
    if (b >= 0) a.bin_list[atomicAdd(&cur[b], 1)] = (int32_t)v;
  }
}

// One workgroup per non-empty block: load its tile, serve its queries (every job's).
template <int R, int RX>
__global__ void __launch_bounds__(kBinThreads) k_bin_tile(GnArgs a, int iter, unsigned long long* tile_stats) {
  __shared__ BinTileLds T;
  const int n_ne = *ne_count(a, iter);
  int32_t* cnt = a.bin;
  const int32_t* cur = a.bin + (a.nb_c + a.nb_s);
  const int32_t* ne = a.bin + 2 * (a.nb_c + a.nb_s);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = blockIdx.x; i < n_ne; i += gridDim.x) {
    const int b = ne[i];
    const bool corner = b < a.nb_c;
    const MapGrid& mg = corner ? a.mc : a.ms;
    const int lb = corner ? b : b - a.nb_c;
    const int nbx = bin_nbx(mg), Y = mg.g.dims[1];
    const int bx = lb % nbx, by = (lb / nbx) % Y, bz = lb / (nbx * Y);
    const int nq = cnt[b], q0 = cur[b] - nq;  // the scatter advanced cur to the run's end
    const int ox = (int)mg.g.origin[0], oy = (int)mg.g.origin[1], oz = (int)mg.g.origin[2];
    const int X0 = 4 * bx + ox - 1, Y0 = 4 * (by + oy) - 1, Z0 = 4 * (bz + oz) - 1;  // tile fine box origin
    // ---- load: the 3 x 3 global rows around the block, x cells 4 bx - 1 .. 4 bx + 4 ----
    const int gx0 = max(4 * bx - 1, 0), gx1 = min(4 * bx + 4, mg.g.dims[0] - 1);
    if (tid < 9) {
      const int y = by - 1 + tid % 3, z = bz - 1 + tid / 3;
      int bb = 0, ee = 0;
      if (y >= 0 && y < Y && z >= 0 && z < mg.g.dims[2] && gx0 <= gx1) {
        const int rowbase = (z * Y + y) * mg.g.dims[0];
        bb = mg.cell_start[rowbase + gx0];
        ee = mg.cell_start[rowbase + gx1 + 1];
      }
      T.rows[tid] = make_int2(bb, ee);
    }
    for (int c = tid; c < kTileCells; c += kBinThreads) T.cs[c] = 0u;
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      T.rpre[0] = 0;
      for (int r = 0; r < 9; ++r) T.rpre[r + 1] = (s += T.rows[r].y - T.rows[r].x);
    }
    __syncthreads();
    const int L = T.rpre[9];
    // pass 1: counts per fine cell (every point of the box: the CropBox is per query)
    for (int t = tid; t < L; t += kBinThreads) {
      int j = 0;
      while (T.rpre[j + 1] <= t) ++j;
      const float4 p = mg.pts[T.rows[j].x + (t - T.rpre[j])];
      const int cx = fine8(p.x) - X0, cy = fine8(p.y) - Y0, cz = fine8(p.z) - Z0;
      if ((unsigned)cx < (unsigned)kTileSide && (unsigned)cy < (unsigned)kTileSide && (unsigned)cz < (unsigned)kTileSide)
        atomicAdd(&T.cs[cx + kTileSide * (cy + kTileSide * cz)], 1u);
    }
    __syncthreads();
    // exclusive starts over the 216 cells (one per thread)
    {
      const uint32_t c = tid < kTileCells ? T.cs[tid] : 0u;
      uint32_t inc = c;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
      }
      if (lane == 63) T.wsum[w] = inc;
      __syncthreads();
      uint32_t pre = 0;
      for (int k = 0; k < w; ++k) pre += T.wsum[k];
      if (tid < kTileCells) T.cs[tid] = pre + inc - c;
    }
    __syncthreads();
    const uint32_t total = T.wsum[0] + T.wsum[1] + T.wsum[2] + T.wsum[3];
    const bool tile_ok = total <= (uint32_t)kTilePts;
    if (tile_ok) {
      // pass 2: scatter (cs[c] ends as the end of cell c)
      for (int t = tid; t < L; t += kBinThreads) {
        int j = 0;
        while (T.rpre[j + 1] <= t) ++j;
        const float4 p = mg.pts[T.rows[j].x + (t - T.rpre[j])];
        const int cx = fine8(p.x) - X0, cy = fine8(p.y) - Y0, cz = fine8(p.z) - Z0;
        if ((unsigned)cx < (unsigned)kTileSide && (unsigned)cy < (unsigned)kTileSide && (unsigned)cz < (unsigned)kTileSide)
          T.pts[atomicAdd(&T.cs[cx + kTileSide * (cy + kTileSide * cz)], 1u)] = p;
      }
    }
    __syncthreads();
    if (tile_stats && tid == 0) {
      atomicAdd(&tile_stats[2], 1ull);
      atomicAdd(&tile_stats[3], (unsigned long long)total);
      atomicAdd(&tile_stats[4], (unsigned long long)L);
      if (!tile_ok) atomicAdd(&tile_stats[5], 1ull);
    }
    // ---- the block's queries, one per lane ----
    const float fc = 1.0f / kFineInv;
    for (int k0 = 0; k0 < nq; k0 += kBinThreads) {
      const int k = k0 + tid;
      if (k < nq) {
        const int v = a.bin_list[q0 + k];
        const int it = v / kResThreads, qt = v % kResThreads;
        const int4 item = a.items[it];
        const GnState& g = a.gn[item.x];
        BinQuery q;
        bin_query(a, it, qt, item, g, q);
        Knn5 nn;
#pragma unroll
        for (int t = 0; t < 5; ++t) nn.k[t] = kKnnEmpty;
        if (tile_ok) {
          int lo[3], hi[3];
          bin_box(q, lo, hi);  // within the tile (k_bin_count checked it, same arithmetic)
          const float bx0 = g.crop_min[0], by0 = g.crop_min[1], bz0 = g.crop_min[2];
          const float bx1 = g.crop_max[0], by1 = g.crop_max[1], bz1 = g.crop_max[2];
          // the tile inside the job's CropBox: no per-point test (edges exact: multiples of 1/8)
          const bool inside = (float)X0 * fc >= bx0 && (float)(X0 + kTileSide) * fc <= bx1 && (float)Y0 * fc >= by0 &&
                              (float)(Y0 + kTileSide) * fc <= by1 && (float)Z0 * fc >= bz0 &&
                              (float)(Z0 + kTileSide) * fc <= bz1;
          const int nyr = hi[1] - lo[1] + 1, nr = nyr * (hi[2] - lo[2] + 1);
          int r = 0, ii = 0, e = 0;
          while (true) {
            if (ii >= e) {
              if (r >= nr) break;
              const int y = lo[1] + r % nyr - Y0, z = lo[2] + r / nyr - Z0;
              const int base = kTileSide * (y + kTileSide * z);
              const int ca = base + (lo[0] - X0), cb = base + (hi[0] - X0);
              ii = ca ? (int)T.cs[ca - 1] : 0;
              e = (int)T.cs[cb];
              ++r;
              continue;
            }
            const float4 p = T.pts[ii++];
            bool out = false;
            if (!inside) out = (p.x < bx0) | (p.y < by0) | (p.z < bz0) | (p.x > bx1) | (p.y > by1) | (p.z > bz1);
            float dist = 0.0f, diff;
            diff = q.x0 - p.x; dist += diff * diff;  // flann::L2_Simple
            diff = q.y0 - p.y; dist += diff * diff;
            diff = q.z0 - p.z; dist += diff * diff;
            const unsigned hb = out ? 0x7f800000u : (unsigned)__float_as_int(dist);
            knn_insert<R>(nn, ((unsigned long long)hb << 32) | (unsigned)__float_as_int(p.w));
          }
        } else {  // the tile did not fit: the grid search
          unsigned ks[12] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
          knn5_grid<R, RX, false, false, 1>(mg, q.x0, q.y0, q.z0, g.crop_min, g.crop_max, q.bound, nn, ks);
          (void)ks;
        }
        bin_write(a, it, qt, q, nn);
      }
    }
    __syncthreads();
    if (tid == 0) cnt[b] = 0;  // the next iteration's counts start from zero
  }
}

// The grid search (knn5_grid, gn_knn_block's per-query body) for the query slots k_bin_count
// queued (fb_list[0, count): it * 256 + slot, in arrival order; each query's result depends on the
// query only).
template <int R, int RX>
__global__ void __launch_bounds__(256) k_gn_knn_list(GnArgs a, int iter) {
  const int n = *fb_count(a, iter);
  for (int k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const int v = a.fb_list[k];
    const int it = v / kResThreads, tid = v % kResThreads;
    const int4 item = a.items[it];
    const GnState& g = a.gn[item.x];
    BinQuery q;
    bin_query(a, it, tid, item, g, q);
    Knn5 nn;
    unsigned ks[12] = {1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    knn5_grid<R, RX, false, false, 1>(item.y == 0 ? a.mc : a.ms, q.x0, q.y0, q.z0, g.crop_min, g.crop_max, q.bound,
                                      nn, ks);
    (void)ks;
    bin_write(a, it, tid, q, nn);
  }
}

// FBR_KNN_TILE: 1 serves iterations >= 1 on dense 0.5 m x 0.125 m grids from the block tiles; 0
// (the default: the tiles measured slower than the grid search) keeps the grid
// search for every query.
bool knn_tile_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_KNN_TILE");
    return e ? std::atoi(e) != 0 : false;
  }();
  return v;
}

// The tiles apply to dense grids of 0.5 m y/z x 0.125 m x cells (the k_gn_knn<2, 8> layout).
bool knn_tile_applies(const GridDesc& gc, const GridDesc& gs) {
  return knn_tile_enabled() && !gc.sparse && !gs.sparse && gc.inv_x == 8.0f && gc.inv_cell == 2.0f &&
         gs.inv_x == 8.0f && gs.inv_cell == 2.0f;
}

int64_t knn_tile_blocks(const GridDesc& g) { return (int64_t)((g.dims[0] + 3) / 4) * g.dims[1] * g.dims[2]; }

unsigned long long* knn_tile_stats_buffer();

bool gn_knn_tile_applies(const GnArgs& a, int iter) {
  return iter > 0 && a.bin && knn_tile_applies(a.mc.g, a.ms.g);
}

bool launch_gn_knn_tile(hipStream_t s, const GnArgs& a, int grid, int iter) {
  if (!gn_knn_tile_applies(a, iter)) return false;
  const float rmax2 = 1.0f / (kFineInv * kFineInv);  // bounds up to one fine cell
  const int gq = std::max(1, std::min(grid, 16384));
  unsigned long long* st = knn_tile_stats_buffer();
  fbr_launch(k_bin_count, dim3(gq), dim3(kBinThreads), 0, s, a, iter, rmax2, st);
  fbr_launch(k_bin_scan, dim3(1), dim3(1024), 0, s, a, iter);
  fbr_launch(k_bin_scatter, dim3(gq), dim3(kBinThreads), 0, s, a);
  fbr_launch((k_bin_tile<2, 8>), dim3(gq), dim3(kBinThreads), 0, s, a, iter, st);
  fbr_launch((k_gn_knn_list<2, 8>), dim3(gq), dim3(256), 0, s, a, iter);
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

// [queries, binned queries, tiles built, points in tiles, points scanned by the tile loads, tiles
// over capacity, 0, 0] since the last reset; -1 when the counters are off (FBR_KNN_TILE_STATS unset).
extern "C" int fbr_diag_knn_tile_stats(unsigned long long* out, int reset) {
  unsigned long long* p = fbr::knn_tile_stats_buffer();
  if (!p) return -1;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out, p, sizeof(unsigned long long) * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  if (reset && hipMemset(p, 0, sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  return 0;
}
