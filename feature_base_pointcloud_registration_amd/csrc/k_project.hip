// k_project.hip — A2 projectPointCloud + A4 cloudExtraction on the device.
//
// Reference: /root/reference/src/imageProjection.cpp:583-640 (projection, first point wins a
// range-image cell) and :642-670 (ring-major compaction, start/endRingIndex).
//
// K1 k_project:   one lane per raw point.  Column/range arithmetic is bit-for-bit the
//                 reference's (fdlibm atan2f, float *180, double /M_PI, double round, x86 int
//                 conversion, float sqrt without FMA).  A passing point claims its cell with
//                 atomicMin(owner, input index): the minimum index is exactly the reference's
//                 "first point wins" (rangeMat != FLT_MAX test, :623).
// K2 k_rowcount / k_compact: one wave per (job, ring row); ballot + popcount compaction keeps the
//                 row-major (ring, column) order of cloudExtraction.  Range is recomputed from the
//                 owning point (same expression, same bits) instead of storing a range image.
//                 With an IMU deskew table (fbr_set_deskew) the gathered point goes through
//                 deskewPoint (:545-580) on the way: the range stays the raw point's (rangeMat is
//                 written before deskewPoint, :633-635), and transStartInverse comes from the first
//                 point deskewPoint sees, which is the minimum owner of the scan (the first point
//                 in input order that passes every check always wins its cell).
// Roofline: HBM-bound.  Algorithmic bytes: 24 B per raw point read (K1), 4 B/cell owner
// write+read, 24 B per valid point written (xyzi 16 + col 4 + range 4).
#include <algorithm>
#include <cstdlib>

#include "fbr_common.h"
#include "fbr_fdlibm.h"
#include "fbr_imu.h"
#include "fbr_kernels.h"

namespace fbr {

__device__ __forceinline__ bool project_xyzr(float x, float y, float z, int rowIdn, int H, int W, int& row, int& colo) {
  if (rowIdn < 0 || rowIdn >= H) return false;
  float horizonAngle = (float)((double)(fd_atan2f(x, y) * 180.0f) / M_PI);
  float ang_res_x = (float)(360.0 / (double)(float)W);
  int columnIdn = x86_cvt(-round(((double)horizonAngle - 90.0) / (double)ang_res_x) + (double)(W / 2));
  if (columnIdn >= W) columnIdn -= W;
  if (columnIdn < 0 || columnIdn >= W) return false;
  // range = sqrtf(x^2 + y^2 + z^2) < 1.0 (:618-621): a correctly rounded sqrt is below 1 exactly
  // when its argument is (the largest float below 1 has a square root that rounds below 1; a NaN
  // is not below 1 either way), so the test needs no square root here (k_compact recomputes the
  // stored range)
  if (x * x + y * y + z * z < 1.0f) return false;
  row = rowIdn;
  colo = columnIdn;
  return true;
}

__device__ __forceinline__ bool project_point(const fbr_point_xyzirt& q, int H, int W, int& row, int& colo) {
  return project_xyzr(q.x, q.y, q.z, q.ring, H, W, row, colo);
}

// K1: a 256-thread block owns a chunk of kProjChunk consecutive input points of one job.  In the
// sensor's firing order the chunk covers ~kProjChunk/H columns of every ring, so cells are first
// claimed in an LDS tile [H][tile_cols] (LDS atomicMin on the input index), then the tile's claimed
// cells are merged into the global owner image with row-contiguous atomicMin (consecutive lanes ->
// consecutive cells: a wave's atomics leave L2 as 4 line requests instead of 64 scattered ones).
// min is associative, so the result is the global first-wins claim for any input order; chunks
// whose column span exceeds the tile (the 0/W seam, shuffled input) claim directly in global.
constexpr int kProjThreads = 256, kProjPPT = 8, kProjChunk = kProjThreads * kProjPPT;

// The per-point (row, col) results are parked in LDS (packed row << 16 | col, -1 = rejected)
// rather than in registers across the claim phase: the column arithmetic (fdlibm atan2f, double
// conversions) then runs two points at a time and the kernel stays at a register count that lets
// 8 waves per SIMD hide the atomic latency.
// kPk: the batch's 16-B device records (ScanRec: x, y, z, ring bits in w; one dwordx4 per point)
// instead of the 24-B fbr_point_xyzirt (read whole by the cache lines, 8 of its bytes unused here).
// Claims are tagged with the call's owner generation (OwnerTag).
// (6 waves per SIMD: the LDS tile's limit; the 16-B record instance otherwise took 90 VGPRs, 5 waves)
template <bool kPk>
__global__ void __launch_bounds__(kProjThreads) __attribute__((amdgpu_waves_per_eu(6, 8)))
k_project(const void* __restrict__ src, const int64_t* __restrict__ nin, int64_t nmax, int H, int W,
          int tile_log2, int32_t* __restrict__ owner, int32_t* __restrict__ err, int64_t n_single, OwnerTag ot) {
  extern __shared__ int32_t tile[];  // [H][(1 << tile_log2) + 1]: the pad puts the consecutive rings of one
                                     // column (consecutive points in firing order) in distinct banks
  __shared__ int32_t cellk[kProjChunk];
  __shared__ int red[2][kProjThreads / 64];
  const int job = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // the job's feature-capacity flags start clear (k_features ORs into them; this saves the
  // single-scan path a 6 us fill dispatch on its critical path)
  if (err && blockIdx.x == 0 && tid == 0) err[job] = 0;
  const int tcols = 1 << tile_log2, tcells = H << tile_log2, tpitch = tcols + 1;
  const int64_t n = n_single >= 0 ? n_single : nin[job];  // single scans: the count as an argument
  const fbr_point_xyzirt* P = static_cast<const fbr_point_xyzirt*>(src) + (int64_t)job * nmax;
  const float4* PK = static_cast<const float4*>(src) + (int64_t)job * nmax;
  int32_t* O = owner + (int64_t)job * H * W;
  for (int64_t base = (int64_t)blockIdx.x * kProjChunk; base < n; base += (int64_t)gridDim.x * kProjChunk) {
    int cmin = INT_MAX, cmax = -1;
    // every load of the thread's points first (x, y | z | ring: 16 of the 24 B), then the
    // arithmetic: one memory round trip per chunk instead of two dependent ones per point
    float px[kProjPPT], py[kProjPPT], pz[kProjPPT];
    int pr[kProjPPT];
#pragma unroll
    for (int k = 0; k < kProjPPT; ++k) {
      const int64_t i = base + k * kProjThreads + tid;
      const int64_t ic = i < n ? i : n - 1;  // branch-free: every lane loads (base < n)
      if constexpr (kPk) {
        const float4 q = PK[ic];
        px[k] = q.x;
        py[k] = q.y;
        pz[k] = q.z;
        pr[k] = i < n ? __float_as_int(q.w) : -1;
      } else {
        const float2 xy = *reinterpret_cast<const float2*>(&P[ic].x);
        px[k] = xy.x;
        py[k] = xy.y;
        pz[k] = P[ic].z;
        pr[k] = i < n ? (int)P[ic].ring : -1;
      }
    }
#pragma unroll
    for (int k = 0; k < kProjPPT; ++k) {
      int row, col, v = -1;
      if (project_xyzr(px[k], py[k], pz[k], pr[k], H, W, row, col)) {
        v = (row << 16) | col;
        cmin = min(cmin, col);
        cmax = max(cmax, col);
      }
      cellk[k * kProjThreads + tid] = v;
    }
    for (int o = 32; o > 0; o >>= 1) {
      cmin = min(cmin, __shfl_xor(cmin, o));
      cmax = max(cmax, __shfl_xor(cmax, o));
    }
    if (lane == 0) {
      red[0][wv] = cmin;
      red[1][wv] = cmax;
    }
    __syncthreads();
    cmin = red[0][0];
    cmax = red[1][0];
    for (int w = 1; w < kProjThreads / 64; ++w) {
      cmin = min(cmin, red[0][w]);
      cmax = max(cmax, red[1][w]);
    }
    if (cmax >= 0 && cmax - cmin < tcols) {
      for (int e = tid; e < H * tpitch; e += kProjThreads) tile[e] = kEmptyOwner;
      __syncthreads();
      for (int k = 0; k < kProjPPT; ++k) {
        const int v = cellk[k * kProjThreads + tid];
        if (v >= 0)
          atomicMin(&tile[(v >> 16) * tpitch + ((v & 0xFFFF) - cmin)], (int32_t)(base + k * kProjThreads + tid));
      }
      __syncthreads();
      for (int e = tid; e < tcells; e += kProjThreads) {
        const int32_t v = tile[(e >> tile_log2) * tpitch + (e & (tcols - 1))];
        if (v != kEmptyOwner) atomicMin(&O[(e >> tile_log2) * W + cmin + (e & (tcols - 1))], (int32_t)(ot.bits | (uint32_t)v));
      }
    } else {
      for (int k = 0; k < kProjPPT; ++k) {
        const int v = cellk[k * kProjThreads + tid];
        if (v >= 0) atomicMin(&O[(v >> 16) * W + (v & 0xFFFF)], (int32_t)(ot.bits | (uint32_t)(base + k * kProjThreads + tid)));
      }
    }
    __syncthreads();
  }
}

// Compaction tiles (k_compact): HB rows x CG columns, HB * CG <= cells (512, 1024 or 2048, FBR_COMPACT_CELLS),
// HB <= 64, CG a power of two in [32, 256].  Chosen on the host and passed to both kernels.
struct CompactTile {
  int hb, cg;
};
inline CompactTile compact_tile(int H, int cells) {
  CompactTile t;
  t.hb = std::min(std::min(H, 64), cells / 32);
  t.cg = 32;
  while (t.cg < 256 && 2 * t.cg * t.hb <= cells) t.cg *= 2;
  return t;
}
__host__ __device__ inline int compact_nchunk(int cg, int W) { return (W + cg - 1) / cg; }

// One wave per (job, row): number of claimed cells in the row, the claimed cells of the row before
// each CG-column chunk (choff [job][row][chunk]), and, for deskew, the row's minimum owner.
__global__ void k_rowcount(const int32_t* __restrict__ owner, int H, int W, int cg, int32_t* __restrict__ rowcnt,
                           int32_t* __restrict__ rowmin, int32_t* __restrict__ choff, OwnerTag ot) {
  const int row = blockIdx.x, job = blockIdx.y, lane = threadIdx.x;
  const int32_t* O = owner + ((int64_t)job * H + row) * W;
  const int nch = compact_nchunk(cg, W);
  int32_t* CH = choff + ((int64_t)job * H + row) * nch;
  int run = 0, mn = kEmptyOwner;
  // four 64-column steps per round, their loads issued together (the row is one dependent chain
  // of ballots; a single scan's 64 row waves otherwise wait ~29 L2 round trips each)
  for (int c00 = 0; c00 < W; c00 += 256) {
    int32_t o4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c00 + 64 * q + lane;
      o4[q] = c < W ? O[c] : kEmptyOwner;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c0 = c00 + 64 * q;
      if (c0 >= W) break;  // wave-uniform
      const bool ok = owner_valid(o4[q], ot);
      const int32_t o = ok ? (int32_t)((uint32_t)o4[q] & ot.mask) : kEmptyOwner;
      mn = min(mn, o);
      const uint64_t m = __ballot(ok);
      // chunk starts inside this 64-column step (cg is a multiple of 32)
      if (lane == 0) {
        if (c0 % cg == 0) CH[c0 / cg] = run;
        if ((c0 + 32) % cg == 0 && c0 + 32 < W) CH[(c0 + 32) / cg] = run + __popcll(m & 0xFFFFFFFFull);
      }
      run += __popcll(m);
    }
  }
  if (rowmin)
    for (int off = 32; off > 0; off >>= 1) mn = min(mn, __shfl_xor(mn, off));
  if (lane == 0) {
    rowcnt[job * H + row] = run;
    if (rowmin) rowmin[job * H + row] = mn;
  }
}

// deskewPoint (imageProjection.cpp:545-580) of one kept point: findRotation at timeScanCur + the
// point's relative time, transBt = transStartInverse * getTransformation(0, 0, 0, rot).
__device__ __forceinline__ float4 deskew_point(const fbr_point_xyzirt& q, const fbr_deskew_table& T, const Rot3& Ls,
                                               const float ts[3]) {
  float rx, ry, rz;
  find_rotation(T, T.time_scan_cur + (double)q.time, &rx, &ry, &rz);
  Rot3 Rb;
  float tb[3], o[3];
  compose(Ls, ts, rot_rpy(rx, ry, rz), Rb, tb);
  apply_affine(Rb, tb, q.x, q.y, q.z, o);
  return make_float4(o[0], o[1], o[2], q.intensity);
}

// One workgroup per (job, HB-row block, CG-column chunk) tile.  The owner tile is read row by row
// (coalesced), the owning raw points are gathered column by column (in the sensor's firing order
// consecutive rings of one column are consecutive raw points, so a wave's gather is one contiguous
// span instead of 64 lines 1.5 KB apart), staged in LDS, and written out row by row at
// rowoff + choff + rank: ring-major (ring, column) order as cloudExtraction (:642-670).  Tiles of
// a job are dealt to one XCD (b % 8), so its raw points stay in that XCD's L2 (speed only).
// LDS (dynamic): xyzi [HB*CG] float4, owners [HB*CG] int32, and with deskew the raw ranges
// [HB*CG] float (without deskew the staged point is the raw point and the range is recomputed
// from it at the write, same expression, same bits): 20 KB per 1024-cell tile.
template <bool kDesk, bool kPk = false>
__global__ void __launch_bounds__(256)
k_compact(const fbr_point_xyzirt* __restrict__ pts, const float4* __restrict__ pk, int64_t nmax, int32_t* __restrict__ owner,
          const int32_t* __restrict__ rowcnt, const int32_t* __restrict__ choff, int B, int H, int W, int HB, int CG,
          float4* __restrict__ cloud, int32_t* __restrict__ col, float* __restrict__ range,
          int32_t* __restrict__ start_ring, int32_t* __restrict__ end_ring, int32_t* __restrict__ nvalid,
          DeskArgs desk, OwnerTag ot) {
  // [HB][CG + 1] arrays: the column-by-column gather has consecutive lanes on consecutive rows, and
  // the pad puts those in distinct banks (a CG-word pitch put a whole wave on one bank group:
  // 13.8 conflict cycles per LDS instruction, profiles/r05a_sq_decomp.txt)
  extern __shared__ float4 lds_c[];
  const int PC = CG + 1;
  float4* pxyz = lds_c;                                    // [HB][PC] gathered xyzi
  int32_t* own = reinterpret_cast<int32_t*>(pxyz + HB * PC);  // [HB][PC] owners of the tile
  float* prng = reinterpret_cast<float*>(own + HB * PC);   // [HB][PC] range (deskew only)
  __shared__ int32_t rowoff[64];    // output offset of each tile row before this chunk
  __shared__ int32_t scan[256];
  const int tid = threadIdx.x, lane = tid & 63;
  const int nch = compact_nchunk(CG, W);
  const int nrb = (H + HB - 1) / HB;
  const int tiles = nrb * nch;  // tiles per job
  // XCD-aware deal: job groups of 8, tile t of job (g*8 + x) at block (g*tiles + t)*8 + x
  const int b = blockIdx.x, x = b % 8, rest = b / 8, g = rest / tiles, t = rest % tiles;
  const int job = g * 8 + x;
  if (job >= B) return;
  const int rb = t / nch, ch = t % nch;
  const int r0 = rb * HB, c0 = ch * CG;
  const int nr = min(HB, H - r0), ncl = min(CG, W - c0);
  const int64_t HW = (int64_t)H * W;
  const int32_t* RC = rowcnt + job * H;
  // Every load the tile needs before its gather is issued first, branch-free: its owners (two cells
  // per thread, clamped to the tile's first cell), the row counts before the tile, the tile rows'
  // counts and chunk offsets.  One memory round trip for all of them and one barrier for the
  // prefix (the owner image is reset behind the read for the next scan: this tile is its last
  // reader, which replaces a separate memset launch per call).
  int32_t* O = owner + job * HW;
  int32_t o[2];
  int32_t* a[2];
  bool in[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = tid + 256 * q, r = i / CG, c = i % CG;
    in[q] = i < HB * CG && r < nr && c < ncl;
    a[q] = O + (int64_t)(r0 + (in[q] ? r : 0)) * W + c0 + (in[q] ? c : 0);
    o[q] = *a[q];
  }
  const int tr = min(tid, nr - 1);  // wave 0 holds the tile rows (nr <= HB <= 64)
  const int rcv = RC[r0 + tr];
  const int cho = choff[((int64_t)job * H + r0 + tr) * nch + ch];
  int before = 0;
  for (int r = tid; r < r0; r += 256) before += RC[r];
  for (int sh = 32; sh > 0; sh >>= 1) before += __shfl_xor(before, sh);
  if (lane == 0) scan[tid >> 6] = before;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int i = tid + 256 * q, r = i / CG, c = i % CG;
    const int32_t v = in[q] && owner_valid(o[q], ot) ? (int32_t)((uint32_t)o[q] & ot.mask) : kEmptyOwner;
    if (ot.reset && v != kEmptyOwner) *a[q] = kEmptyOwner;
    if (i < HB * CG) own[r * PC + c] = v;
  }
  for (int i = tid + 512; i < HB * CG; i += 256) {  // tiles above 512 cells (FBR_COMPACT_CELLS)
    const int r = i / CG, c = i % CG;
    int32_t v = kEmptyOwner;
    if (r < nr && c < ncl) {
      int32_t* p = O + (int64_t)(r0 + r) * W + c0 + c;
      v = *p;
      v = owner_valid(v, ot) ? (int32_t)((uint32_t)v & ot.mask) : kEmptyOwner;
      if (ot.reset && v != kEmptyOwner) *p = kEmptyOwner;
    }
    own[r * PC + c] = v;
  }
  __syncthreads();
  if (tid < 64) {
    // inclusive prefix of the tile rows' counts (lane r of wave 0), plus this chunk's offset
    const int base = scan[0] + scan[1] + scan[2] + scan[3];
    const int v = tid < nr ? rcv : 0;
    int inc = v;
    for (int sh = 1; sh < 64; sh <<= 1) {
      const int y = __shfl_up(inc, sh);
      if (lane >= sh) inc += y;
    }
    if (tid < nr) {
      const int roff = base + inc - v;
      rowoff[tid] = roff + cho;
      if (ch == 0) {
        start_ring[job * H + r0 + tid] = roff - 1 + 5;   // imageProjection.cpp:650
        end_ring[job * H + r0 + tid] = roff + v - 1 - 5;  // :668
        if (r0 + tid == H - 1) nvalid[job] = roff + v;
      }
    }
  }
  // deskew: transStartInverse from the scan's first deskewed point (the minimum owner)
  const fbr_point_xyzirt* P = pts + (int64_t)job * nmax;
  const bool dsk = kDesk && (desk.mode[job] & kDeskPoints);
  const fbr_deskew_table* DT = dsk ? desk.table + job : nullptr;
  Rot3 Ls;
  float ts[3] = {0.0f, 0.0f, 0.0f};
  if (dsk) {
    int mn = kEmptyOwner;
    for (int r = lane; r < H; r += 64) mn = min(mn, desk.rowmin[job * H + r]);
    for (int s = 32; s > 0; s >>= 1) mn = min(mn, __shfl_xor(mn, s));
    float rx = 0.0f, ry = 0.0f, rz = 0.0f;
    if (mn != kEmptyOwner) find_rotation(*DT, DT->time_scan_cur + (double)P[mn].time, &rx, &ry, &rz);
    affine_inverse(rot_rpy(rx, ry, rz), Ls, ts);
  }
  // gather, column by column (consecutive threads = consecutive rings of one column)
  if (kDesk) {
    for (int i = tid; i < HB * CG; i += 256) {
      const int c = i / HB, r = i % HB, k = r * PC + c;
      const int32_t o = own[k];
      if (o != kEmptyOwner) {
        const fbr_point_xyzirt q = P[o];
        pxyz[k] = dsk ? deskew_point(q, *DT, Ls, ts) : make_float4(q.x, q.y, q.z, q.intensity);
        prng[k] = sqrt_rn(q.x * q.x + q.y * q.y + q.z * q.z);
      }
    }
  } else {
    for (int i0 = tid; i0 < HB * CG; i0 += 512) {
      float4 v[2];
      int kk[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int i = i0 + 256 * q, c = i / HB, r = i % HB;
        kk[q] = r * PC + (i < HB * CG ? c : CG);  // past the tile: the row's pad column (never read)
        const int32_t o = i < HB * CG ? own[kk[q]] : kEmptyOwner;
        if constexpr (kPk) {  // 16-B records: (x, y, z, ring); the batch's clouds carry no intensity
          v[q] = pk[(int64_t)job * nmax + (o != kEmptyOwner ? o : 0)];
          v[q].w = 0.0f;
        } else {
          v[q] = *reinterpret_cast<const float4*>(&P[o != kEmptyOwner ? o : 0].x);  // (x, y, z, intensity)
        }
      }
      // stored unconditionally (an empty cell's slot is never read): no branch for the compiler to
      // sink the loads into
#pragma unroll
      for (int q = 0; q < 2; ++q) pxyz[kk[q]] = v[q];
    }
  }
  __syncthreads();
  // write out row by row: rank of each claimed cell among the row's claimed cells of the tile
  float4* C = cloud + job * HW;
  int32_t* CI = col + job * HW;
  float* R = range + job * HW;
  const int rpp = 256 / CG;                          // rows per pass, CG threads per row
  const int passes = (nr + rpp - 1) / rpp;             // the same for every thread (barriers below)
  for (int p = 0; p < passes; ++p) {
    const int r = p * rpp + tid / CG;
    int rank = 0;
    const int c = tid % CG;
    const int k = r * PC + c;
    const bool v = r < nr && own[k] != kEmptyOwner;
    // prefix over the CG cells of the row: ballots over the wave's 64 lanes (CG = 32: two rows per
    // wave; CG >= 64: a row spans CG / 64 waves, combined through LDS)
    const uint64_t m = __ballot(v);
    if (CG <= 32) {
      const int sh = lane & ~31;  // the row's half of the wave
      const uint64_t mm = (m >> sh) & 0xFFFFFFFFull;
      rank = __popcll(mm & ((1ull << (lane & 31)) - 1ull));
    } else {
      const int wv = tid >> 6, wrow = (tid % CG) >> 6;  // wave index inside the row
      scan[wv] = __popcll(m);
      __syncthreads();
      int prev = 0;
      for (int q = 0; q < wrow; ++q) prev += scan[wv - wrow + q];
      rank = prev + __popcll(m & ((1ull << lane) - 1ull));
      __syncthreads();
    }
    if (v) {
      const int dst = rowoff[r] + rank;
      const float4 p = pxyz[k];
      C[dst] = p;
      CI[dst] = c0 + c;
      R[dst] = kDesk ? prng[k] : sqrt_rn(p.x * p.x + p.y * p.y + p.z * p.z);
    }
  }
}

// K0 k_unpack_msg: sensor_msgs/PointCloud2 bytes (row-major, point_step / row_step strided
// records, as they arrive) -> the 24-B fbr_point_xyzirt scan buffer; pcl::fromROSMsg's field
// mapping was resolved on the host (fbr_msg.cpp), unmapped fields are 0.  One lane per point;
// dword loads when every offset and stride is aligned (the usual driver layouts), byte loads
// otherwise.  HBM-bound: point_step B read + 24 B written per point.
template <bool kAligned>
__device__ __forceinline__ float msg_f32(const uint8_t* p, int off) {
  if (off < 0) return 0.0f;
  if (kAligned) return *reinterpret_cast<const float*>(p + off);
  uint32_t u = (uint32_t)p[off] | ((uint32_t)p[off + 1] << 8) | ((uint32_t)p[off + 2] << 16) |
               ((uint32_t)p[off + 3] << 24);
  return __uint_as_float(u);
}

template <bool kAligned>
__global__ void __launch_bounds__(256)
k_unpack_msg(const uint8_t* __restrict__ data, MsgDev L, fbr_point_xyzirt* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= L.n) return;
  const int64_t r = i / L.width, c = i - r * L.width;
  const uint8_t* p = data + r * L.row_step + c * L.point_step;
  fbr_point_xyzirt q;
  q.x = msg_f32<kAligned>(p, L.off[0]);
  q.y = msg_f32<kAligned>(p, L.off[1]);
  q.z = msg_f32<kAligned>(p, L.off[2]);
  q.intensity = msg_f32<kAligned>(p, L.off[3]);
  const int orr = L.off[4];
  q.ring = orr < 0 ? 0
           : kAligned ? *reinterpret_cast<const uint16_t*>(p + orr)
                      : (uint16_t)(p[orr] | (p[orr + 1] << 8));
  q.pad_ = 0;
  q.time = msg_f32<kAligned>(p, L.off[5]);
  out[i] = q;
}

void launch_unpack_msg(hipStream_t s, const uint8_t* data, const MsgDev& L, fbr_point_xyzirt* out) {
  if (L.n <= 0) return;
  bool aligned = (L.point_step % 4 == 0) && (L.row_step % 4 == 0);
  for (int k = 0; k < 6; ++k)
    if (L.off[k] >= 0) aligned = aligned && (L.off[k] % (k == 4 ? 2 : 4) == 0);
  const dim3 grid((unsigned)((L.n + 255) / 256));
  if (aligned)
    fbr_launch(k_unpack_msg<true>, grid, dim3(256), 0, s, data, L, out);
  else
    fbr_launch(k_unpack_msg<false>, grid, dim3(256), 0, s, data, L, out);
}

// K0' k_expand_scans: the compact ingest records of fbr_process_batch -> the 24-B scan buffer.
// No deskew: the reference never reads `time` on this path (imageProjection.cpp:189-191), and a
// batch returns poses and statistics, which no point's intensity reaches (it rides along as the
// clouds' w channel: never in a key, a distance, a residual or a count), so neither is shipped.
// Job j's record (at byte offset off[j] of the stage) holds its n points as planes x[m], y[m],
// z[m] (f32, m = ingest_plane(n)), then the rings x n (u8 when rb = 1, u16 when rb = 2);
// intensity = time = 0.  Slots
// past n are not written (k_project reads n points).  HBM-bound: 12 + rb B read + 24 B written per
// point.
template <bool kPk>
__global__ void __launch_bounds__(256)
k_expand_scans(const uint8_t* __restrict__ stage, int64_t nmax, const int64_t* __restrict__ nin,
               const int64_t* __restrict__ off, int rb, void* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t job = blockIdx.y;
  const int64_t n = min(nin[job], nmax);
  if (i >= n) return;
  const uint8_t* r = stage + off[job];
  const float* pl = reinterpret_cast<const float*>(r);
  const int64_t m = ingest_plane(n);
  const uint16_t ring = rb == 1 ? (uint16_t)r[12 * m + i] : reinterpret_cast<const uint16_t*>(r + 12 * m)[i];
  if constexpr (kPk) {
    static_cast<float4*>(dst)[job * nmax + i] = make_float4(pl[i], pl[m + i], pl[2 * m + i], __int_as_float((int)ring));
  } else {
    fbr_point_xyzirt q;
    q.x = pl[i];
    q.y = pl[m + i];
    q.z = pl[2 * m + i];
    q.intensity = 0.0f;
    q.ring = ring;
    q.pad_ = 0;
    q.time = 0.0f;
    static_cast<fbr_point_xyzirt*>(dst)[job * nmax + i] = q;
  }
}

void launch_expand_scans(hipStream_t s, const uint8_t* stage, int64_t nmax, int B, const int64_t* nin,
                         const int64_t* off, int rb, void* out, bool pk) {
  if (B <= 0 || nmax <= 0) return;
  const dim3 grid((unsigned)((nmax + 255) / 256), B);
  if (pk)
    fbr_launch(k_expand_scans<true>, grid, dim3(256), 0, s, stage, nmax, nin, off, rb, out);
  else
    fbr_launch(k_expand_scans<false>, grid, dim3(256), 0, s, stage, nmax, nin, off, rb, out);
}

void launch_project(hipStream_t s, const fbr_point_xyzirt* pts, const int64_t* nin, int64_t nmax, int B, int H,
                    int W, int32_t* owner, int32_t* err, int64_t n_single, const float4* pk, const OwnerTag& ot) {
  int blocks = (int)((nmax + kProjChunk - 1) / kProjChunk);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  int tile_log2 = 6;  // 64 columns, shrunk so the tile stays <= 32 KB
  while (tile_log2 > 3 && ((int64_t)H << tile_log2) > 8192) --tile_log2;
  const size_t lds = sizeof(int32_t) * (size_t)H * ((1 << tile_log2) + 1);
  if (pk)
    fbr_launch(k_project<true>, dim3(blocks, B), dim3(kProjThreads), lds, s, (const void*)pk, nin, nmax, H, W,
               tile_log2, owner, err, n_single, ot);
  else
    fbr_launch(k_project<false>, dim3(blocks, B), dim3(kProjThreads), lds, s, (const void*)pts, nin, nmax, H, W,
               tile_log2, owner, err, n_single, ot);
}

// Compaction tile size in cells (FBR_COMPACT_CELLS: 512, 1024 or 2048).  512 since round 5: 10 KB of
// LDS per workgroup, twice the tiles in flight per CU; once the other kernels had shrunk, C2 B = 1024
// 114.5-114.9k -> 115.7-115.8k and C3 +0.9 % interleaved (profiles/r05ar_compact_cells_ab.txt; it was
// even with 1024 in round 4).
int compact_cells() {
  static const int v = [] {
    const char* e = std::getenv("FBR_COMPACT_CELLS");
    const int c = e ? std::atoi(e) : 512;
    return c >= 2048 ? 2048 : c >= 1024 ? 1024 : 512;
  }();
  return v;
}

void launch_extract(hipStream_t s, const fbr_point_xyzirt* pts, int64_t nmax, int32_t* owner, int B, int H,
                    int W, int32_t* rowcnt, int32_t* choff, float4* cloud, int32_t* col, float* range,
                    int32_t* start_ring, int32_t* end_ring, int32_t* nvalid, const DeskArgs& desk, const float4* pk,
                    const OwnerTag& ot) {
  const CompactTile T = compact_tile(H, compact_cells());
  fbr_launch(k_rowcount, dim3(H, B), dim3(64), 0, s, owner, H, W, T.cg, rowcnt, desk.mode ? desk.rowmin : nullptr,
             choff, ot);
  const int tiles = ((H + T.hb - 1) / T.hb) * compact_nchunk(T.cg, W);
  const int groups = (B + 7) / 8;
  const dim3 grid((unsigned)(groups * 8 * tiles));
  const size_t cells = (size_t)T.hb * (T.cg + 1);  // padded pitch (k_compact)
  if (desk.mode)
    fbr_launch(k_compact<true>, grid, dim3(256), (uint32_t)(cells * 24), s, pts, pk, nmax, owner, rowcnt, choff, B,
               H, W, T.hb, T.cg, cloud, col, range, start_ring, end_ring, nvalid, desk, ot);
  else if (pk)
    fbr_launch(k_compact<false, true>, grid, dim3(256), (uint32_t)(cells * 20), s, pts, pk, nmax, owner, rowcnt,
               choff, B, H, W, T.hb, T.cg, cloud, col, range, start_ring, end_ring, nvalid, desk, ot);
  else
    fbr_launch(k_compact<false>, grid, dim3(256), (uint32_t)(cells * 20), s, pts, pk, nmax, owner, rowcnt, choff, B,
               H, W, T.hb, T.cg, cloud, col, range, start_ring, end_ring, nvalid, desk, ot);
}

}  // namespace fbr
