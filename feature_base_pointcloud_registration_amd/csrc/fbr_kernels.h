// fbr_kernels.h — argument blocks and host launchers of the device kernels.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>

#include "fbr_common.h"

namespace fbr {

// ---- kernel timing (fbr_set_profiling) ----
// When a launcher runs under a kernel timer (fbr_api.hip TIMED_ON), its kernels are dispatched with
// hipExtLaunchKernel and the timer's events: the first kernel's dispatch records the start event
// with its own start timestamp and every kernel records the stop event with its end timestamp, so
// the measured interval is the launcher's kernels' execution (the timestamps rocprofv3's kernel
// trace reports), not the time the stream spends waiting for CUs the other streams hold.
struct LaunchTimer {
  hipEvent_t start = nullptr, stop = nullptr;
  int launched = 0;
};
inline LaunchTimer& launch_timer() {
  static thread_local LaunchTimer t;
  return t;
}

// Diagnostic counters (fbr_debug_counters): kernel launches, blocking host synchronisations
// (stream syncs and synchronous copies of the boundary code) and Gauss-Newton flag polls.
struct DebugCounters {
  std::atomic<long long> launches{0}, host_syncs{0}, flag_polls{0};
  // host wall time (ns) of the single-scan calls: [0] scan upload (staging copy + enqueue),
  // [1] enqueue of the stages (launches, GN flag polls), [2] result wait, [3] whole call
  std::atomic<long long> host_ns[4] = {0, 0, 0, 0};
  // batch calls: [0] fbr_batch_launch wall time, [1] of it spent waiting for GN iteration flags
  std::atomic<long long> batch_ns[2] = {0, 0};
  // host waits on device results (fbr_diag_wait_stats): fallbacks, waits > 1 ms, longest wait (ns),
  // stream queries
  std::atomic<long long> flag_fallbacks{0}, waits_over_1ms{0}, wait_max_ns{0}, stream_queries{0};
};
inline DebugCounters& debug_counters() {
  static DebugCounters c;
  return c;
}

template <typename F, typename... Args>
inline void fbr_launch(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
  debug_counters().launches.fetch_add(1, std::memory_order_relaxed);
  LaunchTimer& t = launch_timer();
  if (t.stop) {
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, t.launched ? nullptr : t.start, t.stop, 0, args...);
    t.launched++;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
  }
}

// ---- A2+A4 (k_project.hip) ----
// Device copy of the resolved PointCloud2 layout (fbr_msg.h): offsets x, y, z, intensity, ring,
// time (-1 = unmapped).
struct MsgDev {
  int64_t n, width, row_step, point_step;
  int32_t off[6];
};
void launch_unpack_msg(hipStream_t s, const uint8_t* data, const MsgDev& L, fbr_point_xyzirt* out);
// Compact ingest records (fbr_process_batch without deskew tables): job j's record, at byte offset
// off[j] of the stage (16-B aligned, back to back as the staging chunks lay them out), holds its n
// points as planes [x f32 x m][y f32 x m][z f32 x m][ring x n], m = ingest_plane(n) (16-B aligned
// planes, for the packers' streaming stores), the rings as u8 when the sensor has at most 256 rings
// (rb = 1), else u16 (rb = 2).  ingest_region_bytes(nmax) bounds one record, padding included.
__host__ __device__ inline int64_t ingest_plane(int64_t n) { return (n + 3) & ~(int64_t)3; }
inline int64_t ingest_region_bytes(int64_t nmax) { return (14 * nmax + 48 + 15) & ~(int64_t)15; }
// Batch scans may live on the device as 16-B records (ScanRec): float4 (x, y, z, ring as int bits
// in w), one dwordx4 per point where the 24-B fbr_point_xyzirt costs 24 B of cache lines for the 16
// projection and extraction read.  pk = the records (null: the 24-B scans); intensity and time are
// not carried, so launches that deskew keep the 24-B scans.
// out: fbr_point_xyzirt records, or with pk the 16-B ones.
void launch_expand_scans(hipStream_t s, const uint8_t* stage, int64_t nmax, int B, const int64_t* nin,
                         const int64_t* off, int rb, void* out, bool pk);
// Generation-tagged owner image: a claim is (tag << ib) | input index, where the tag of call g is
// (kEmptyOwner >> ib) - g, so a later call's claims win atomicMin against every stale one, and a cell
// belongs to this call only when its tag bits equal `bits`.  The image is then never reset between
// calls (only when the generations run out).  bits = 0, mask = 0x7FFFFFFF: untagged, k_compact
// resets the claimed cells behind its read (owner images of > 2^24-point scans).
struct OwnerTag {
  uint32_t bits, mask;
  bool reset;  // untagged: k_compact writes kEmptyOwner back
};
__host__ __device__ inline bool owner_valid(int32_t o, const OwnerTag& t) {
  return o != 0x7F7F7F7F && ((uint32_t)o & ~t.mask) == t.bits;
}
void launch_project(hipStream_t s, const fbr_point_xyzirt* pts, const int64_t* nin, int64_t nmax, int B, int H,
                    int W, int32_t* owner,
                    int32_t* err, int64_t n_single, const float4* pk, const OwnerTag& ot);
// Optional IMU deskew of the kept points (deskewPoint, imageProjection.cpp:545-580): desk_mode
// [B] (kDesk* bits, fbr_imu.h) and desk [B] tables, both null when no job deskews; rowmin [B][H]
// receives each row's minimum owner (the scan's first deskewed point is the minimum over rows).
struct DeskArgs {
  const int32_t* mode;
  const fbr_deskew_table* table;
  int32_t* rowmin;
};
// choff: [B][H][ceil(W / 32)] scratch (claimed cells of a row before each compaction tile)
void launch_extract(hipStream_t s, const fbr_point_xyzirt* pts, int64_t nmax, int32_t* owner, int B, int H,
                    int W, int32_t* rowcnt, int32_t* choff, float4* cloud, int32_t* col, float* range,
                    int32_t* start_ring, int32_t* end_ring, int32_t* nvalid, const DeskArgs& desk,
                    const float4* pk, const OwnerTag& ot);

// ---- A6-A8 (k_features.hip) ----
struct FeatArgs {
  int B, H, W;
  const float4* cloud;
  const int32_t* col;
  const float* range;
  const int32_t* start_ring;
  const int32_t* end_ring;
  const int32_t* nvalid;
  float edge_thr, surf_thr;
  StreamState* stream;   // [B]
  int8_t* label;         // [B][H*W]
  float4* corner_slot;   // [B][H][120]
  int32_t* corner_cnt;   // [B][H]
  int32_t* err;          // [B]
  int lcap, segcap;      // LDS capacities (window length, segment length)
  int kseg;              // segment sort capacity: next power of two >= segcap - 1 (<= 1024)
  int nwcap;             // 64-bit words per window bit array
  unsigned char* gscratch;  // [B*H][gslot_bytes] sorted-path buffers (stale-slot segment, ties)
  int64_t gslot_bytes;
  unsigned long long* stamps;  // diagnostic builds only: [B*H][12] phase cycle sums
  // 0 (independent batch jobs): the surf walk is resolved only as far as it reaches the next
  // segment (its picks' suppression past ep), since nothing else of it is observable there: the
  // per-ring VoxelGrid takes label <= 0 (picked surf -1 and 0 alike, featureExtraction.h:279-284)
  // and no label leaves a batch.  1 (single scans: cloudLabel is an output): the whole walk.
  int surf_full = 1;
  // Stream mode (single scans): cloudLabel[0..4] and cloudNeighborPicked[0..4] carry to the next
  // scan, so with surf_full = 0 the segments starting at index <= 9 (whose members reach them) still
  // run the whole walk.
  int carry = 0;
  // Batch jobs start from a fresh node: labels at indices < 5 are written even when 0 (no stale
  // value to keep), so the label buffer needs no clearing between launches.
  int fresh = 0;
};
size_t features_lds_bytes(const FeatArgs& a, int nwv);  // nwv: waves per ring
size_t features_gslot_bytes(const FeatArgs& a);
void launch_features(hipStream_t s, const FeatArgs& a);

// ---- A9 VoxelGrid over segments (k_voxel.hip) ----
struct VgSet {               // nseg segments of one cloud family, one leaf size
  const float4* in;
  int64_t stride_in;         // input segment stride (points)
  const int32_t* cnt_in;     // per-segment input counts
  int64_t cap;               // max points per segment (counts are clamped to it)
  float4* out;
  int64_t stride_out;
  int32_t* cnt_out;
  uint32_t* scratch;         // global mode: [nseg][kVgScratch][cap]
  float leaf;
  int nseg;
  int morton;                // 1: emit voxels in Morton order of (i,j,k) instead of PCL key order
  int exact;                 // 1: PCL's point order inside voxels (std::sort's, fbr_introsort.h;
                             // fbr_params.exact_voxel_order), 0: index order
  // Optional precomputed bounds (k_concat's ring boxes): segment seg's box k at
  // box + seg * box_stride + k * kRingBox, k < box_n, each {min xyz, max xyz}; null: from the points
  const float* box;
  int box_n;
  int64_t box_stride;
};
// Per-point u32 slots of a VoxelGrid segment's global scratch: keys / indices ping-pong (4) and
// the std::sort emulation's frame lists (1).
constexpr int64_t kVgScratch = 5;
struct VgArgs {
  VgSet s[2];                // segments of set 0, then of set 1 (set 1 may be empty)
  // per-segment error words (segment j of either set = job j): k_voxel_grid_split ORs
  // kVgErrLookback into them when the bounded look-back of any part gives up.  A middle part that
  // gives up skips its emit while the last part may still see every flag and write a full count,
  // so callers must check the error word, not only the count (the batch jobs' error words, the
  // single-cloud callers' own word).  With err null a lost last part writes -1.
  int32_t* err = nullptr;
};
constexpr int32_t kVgErrLookback = 16;
constexpr int64_t kVgLdsCap = 4096;  // segments up to this size sort entirely in LDS
void launch_voxel_grid(hipStream_t s, const VgArgs& a);

// Device scratch of the set-up paths (map VoxelGrid, kNN grid builds): one hipMalloc'd block per
// context, grown when a call needs more (after draining the stream that used it) and carved by a
// bump allocator.  Every user runs on the context's stream, so a call that fits reuses the block
// in stream order without a host synchronisation.
struct DevArena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
};
inline size_t arena_bytes(size_t b) { return (std::max<size_t>(b, 1) + 255) & ~(size_t)255; }
// Room for `bytes` (the sum of arena_bytes of every slice the call takes); carving restarts at 0.
inline hipError_t arena_reserve(DevArena& a, size_t bytes, hipStream_t s) {
  a.used = 0;
  if (bytes <= a.cap) return hipSuccess;
  hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return e;
  if (a.base) (void)hipFree(a.base);
  a.base = nullptr;
  a.cap = 0;
  const size_t nc = std::max(bytes + bytes / 4, (size_t)1 << 20);
  e = hipMalloc((void**)&a.base, nc);
  if (e == hipSuccess) a.cap = nc;
  return e;
}
template <typename T>
T* arena_take(DevArena& a, size_t bytes) {
  const size_t b = arena_bytes(bytes);
  if (!a.base || a.used + b > a.cap) return nullptr;
  T* p = reinterpret_cast<T*>(a.base + a.used);
  a.used += b;
  return p;
}
inline void arena_free(DevArena& a) {
  if (a.base) (void)hipFree(a.base);
  a = DevArena{};
}

// One large cloud on the whole device (rocprim stable radix sort); *d_nout gets the voxel count.
constexpr int64_t kVgLargeMin = 32768;  // below this the one-workgroup kernel is faster
int voxel_grid_large(hipStream_t s, DevArena& ar, const float4* in, int64_t n, float leaf, int morton, int exact,
                     float4* out, int32_t* d_nout);

// Per-ring surf filter reading the projected cloud + label mask directly (no candidate copy).
struct VgRing {
  const float4* cloud;       // [B][H*W] projected cloud
  const int8_t* label;       // [B][H*W] cloudLabel
  const int32_t* start_ring; // [B][H]
  const int32_t* end_ring;   // [B][H]
  int B, H;
  int64_t HW;
  int64_t cap;               // Horizon_SCAN (max points per ring, <= 4096)
  float leaf;
  float4* out;               // [B*H][stride_out]
  int64_t stride_out;
  int32_t* cnt_out;          // [B*H]
  int dbg;                   // diagnostic phase cut (FBR_VR_DBG; 0 = full kernel)
  int kernel = -1;           // default order: -1 by launch size, 0 the 512-thread kernel, 2 four waves
                             // per ring (fbr_diag_ring_filter: tests compare the two)
  int exact;                 // 1: PCL's point order inside voxels (std::sort's, fbr_introsort.h)
  unsigned long long* stamps;  // diagnostic builds (FBR_VR_STAMPS) only: [B*H][12]
};
void launch_voxel_ring(hipStream_t s, const VgRing& a);

// Concatenate per-ring corner slots / per-ring surf DS outputs into per-job clouds (the
// cornerCloud / surfaceCloud push_back order of featureExtraction.h:219,292).  ring_box (may be
// null): per (job, ring) the corner then the surf points' {min xyz, max xyz} (kRingBox floats;
// empty rings +FLT_MAX / -FLT_MAX), so the mapping DS need not read its clouds for the bounds.
constexpr int kRingBox = 12;
void launch_concat(hipStream_t s, int B, int H, int W, const float4* corner_slot, const int32_t* corner_cnt,
                   const float4* surf_ring, const int32_t* surf_ring_cnt, float4* corner_all, int64_t capc,
                   int32_t* n_corner, float4* surf_all, int64_t caps, int32_t* n_surf, float* ring_box);

// ---- A10-A18 (k_register.hip) ----
struct MapGrid {
  const float4* pts;          // sorted by cell; w = bit pattern of the map index
  const int32_t* cell_start;  // dense: [n_cells+1]; sparse: [chunks][kChunkX + 1]
  GridDesc g;
  const float4* by_id;        // the same points in map-index order (neighbour gathers by index)
  const unsigned long long* hkeys;  // sparse: [hmask + 1] chunk keys (kChunkEmpty = free)
  const int32_t* hvals;             // sparse: [hmask + 1] chunk ids
};

// A map's kNN grid in HBM (fbr_set_map, the keyframe local map): built on the device from the
// map points in map-index order.  Dense when the occupied box has at most kDenseGridCells cells,
// hashed chunks otherwise (or when FBR_GRID_SPARSE=1).
struct DevGrid {
  float4* pts = nullptr;              // [0, n): sorted by cell; [n, 2n): by map index
  int32_t* cs = nullptr;
  unsigned long long* hkeys = nullptr;
  int32_t* hvals = nullptr;
  GridDesc g{};
  MapGrid view() const { return MapGrid{pts, cs, g, pts + g.n_points, hkeys, hvals}; }
};
constexpr int64_t kDenseGridCells = (int64_t)1 << 26;
void free_grid(DevGrid& d);
// Build `out` over n points (device, map-index order) with cells of 1/invx (x) and 1/inv (y, z).
int grid_build_device(hipStream_t s, DevArena& ar, const float4* pts, int64_t n, float invx, float inv,
                      bool force_sparse, DevGrid& out);

struct JobResult;
struct GnArgs {
  int B, max_iter;
  // one_item: the plain kNN / residual launches run one work item per workgroup over
  // [0, grid) (no grid-stride loop: the loop's carried state took k_gn_residual from 64 to 108
  // VGPRs, the flat kNN from 54 to 68), and a loop launch picks up items past the grid
  // (one_item = 2: the host has seen the run's item count fit the grid, no loop launch)
  int one_item;
  int rest_grid;  // workgroups of that loop launch (few when the grid was sized from a previous count)
  int one_part;   // 0: both launches; 1: the one-item launch only; 2: the loop launch only (timed apart)
  const float4* cornerDS;
  int64_t capc;
  const int32_t* ncds;
  const float4* surfDS;
  int64_t caps;
  const int32_t* nsds;
  MapGrid mc, ms;
  GnState* gn;               // [B]
  const float* guess;        // [B][6]
  int4* items;               // work items {job, type, start, count}
  int32_t* nitems;           // [1]
  int32_t* item_range;       // [B][2] first / end item of each job
  double* partial;           // [max_items][32]
  int max_items;
  int edge_min, surf_min;
  float crop_half[3];
  float rot_tol, z_tol;
  float* pose_out;           // [B][6]
  fbr_reg_stats* stats;      // [B]
  float* trace;              // [B][max_iter][6] or null
  int32_t* nbr;              // [max_items][5][256] kNN-5 map indices of each query (-1 = rejected)
  float* fitc;               // [max_items][6][256] fit cache: line / plane of each query's neighbours
  int8_t* fits;              // [max_items][256] fit cache state (0 none, 1 fitted, 2 rejected)
  int8_t* nsame;             // [max_items][256] 1: this iteration's neighbours equal the previous ones
  int fit_cache;             // reuse cached fits (FBR_FIT_CACHE, default 1)
  unsigned long long* iter_flags;  // host-mapped [max_iter]: (generation << 32) | jobs still active
  unsigned long long* items_flag;  // host-mapped: (generation << 32) | work items (k_gn_solve, iteration 0)
  int32_t* iter_cnt;         // [max_iter][2] active-job count / finished workgroups, then [max_iter]
                             // queued-query and [max_iter] non-empty-block counts of the block
                             // tiles (k_knn_tile.hip; all zeroed by k_gn_init)
  int32_t* fb_list;          // block tiles: [max_items][256] query slots left to the grid search
  int32_t* bin_list;         // block tiles: [max_items][256] binned query slots, by block
  int32_t* qblk;             // block tiles: [max_items][256] block of each query slot (-1: none)
  int32_t* bin;              // block tiles: [3][nb_c + nb_s] counts, cursors, non-empty list; null: off
  int nb_c, nb_s;            // blocks of the corner / surf grids
  const int32_t* desk_mode;  // [B] kDesk* bits or null (transformUpdate's IMU slerp, :1447-1474)
  const fbr_deskew_table* desk;  // [B]
  int nocrop;                // 1: keyframe local map, no CropBox (scan2MapOptimization on it)
  int deg_carry;             // isDegenerate before the first LMOptimization (the member carried
                             // across registration() calls, mapOptmization.h:137); 0 for batch jobs
  unsigned long long* knn_stats;  // diagnostic builds (FBR_KNN_STATS): the kNN counters, else null
  // Single scans (fbr_process_scan): the k_gn_solve that ends the run (no job active, or the last
  // iteration) also runs transformUpdate and packs each job's JobResult into host-mapped memory
  // (`direct`, pad = direct_gen), so the host reads the result without a finalize launch, a pack
  // launch and a copy.  null: the host enqueues k_gn_finalize and k_pack_results.
  JobResult* direct;
  int32_t* direct_done;      // [1] the ending solve's claim (zeroed by k_gn_init)
  int32_t direct_gen;
  const int32_t* nvalid;     // the pack's inputs: [B] valid points, corner / surf features, the
  const int32_t* ncorner;    // features' capacity flags, CropBox counts [B][2]
  const int32_t* nsurf;
  const int32_t* ferr;
  const int32_t* cropcnt;
};
#ifdef FBR_KNN_STATS
unsigned long long* knn_stats_buffer();
#endif
// iterations >= 1 on dense maps: the wave-tile search (k_knn_tile.hip); false = not applicable
bool launch_gn_knn_tile(hipStream_t s, const GnArgs& a, int grid, int iter);
bool gn_knn_tile_applies(const GnArgs& a, int iter);
bool knn_tile_applies(const GridDesc& gc, const GridDesc& gs);
int64_t knn_tile_blocks(const GridDesc& g);
void launch_gn_init(hipStream_t s, const GnArgs& a);
// fused: kNN + residual row + item partial in one launch (launch_gn_residual is then skipped)
void launch_gn_knn(hipStream_t s, const GnArgs& a, int grid, int iter, bool fused);
void launch_gn_residual(hipStream_t s, const GnArgs& a, int grid);
void launch_gn_solve(hipStream_t s, const GnArgs& a, int iter_idx, unsigned long long gen);
void launch_gn_finalize(hipStream_t s, const GnArgs& a);
// Everything the host reads back per job, packed by one kernel so a single copy returns it.
struct JobResult {
  float pose[6];
  fbr_reg_stats st;
  int32_t err;  // k_features capacity error of the job
  int32_t pad;
};
// with_reg = 0: the registration did not run (interval gate): stats hold only the cloud counts.
// guess (batch calls): a job with a features capacity error gets it as pose, status
// FBR_REG_FEATURE_CAPACITY; null: the caller fails the call on any error instead
void launch_pack_results(hipStream_t s, int B, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                         const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf, const int32_t* cropcnt,
                         const int32_t* err, const float* guess, JobResult* out);
// laserCloud{Corner,Surf}FromMapDSNum: CropBox counts of the global map per job.
void launch_export_records(hipStream_t s, int B, const float* pose_out, const fbr_reg_stats* stats, const int32_t* err,
                           const float* guess, float* dst);
// (accumulated in `work` [B][2], this launch's work slot, then copied to `counts` [B][2]: a
// recomputation never exposes a partial count to a reader of the same staged batch's counts)
void launch_crop_count(hipStream_t s, const GnArgs& a, const float4* corner_pts, int64_t n_corner,
                       const float4* surf_pts, int64_t n_surf, int32_t* work, int32_t* counts);

// ---- keyframe local map (k_keyframe.hip) ----
struct KfSeg {               // one selected keyframe cloud: pool[src .. src+count) -> out[dst ..]
  int64_t src, dst, count;
  float T[12];               // pcl::getTransformation of the key pose, row-major 3x4
};
void launch_kf_transform(hipStream_t s, const float4* pool, const KfSeg* segs, int nseg, int64_t max_count, float4* out);

}  // namespace fbr
