// fbr_api.hip — the extern "C" boundary (include/fbr.h) and the device pipeline orchestration.
//
// One fbr_ctx = one HIP device + one stream + the HBM buffers for a batch of up to max_batch
// scans.  A batch runs entirely on the device:
//   memset owners -> k_project -> k_rowcount/k_compact        (imageProjection.cpp:583-670)
//   -> k_features (per ring) -> k_voxel_grid (per ring surf)  (featureExtraction.h:109-294)
//   -> k_concat -> k_voxel_grid x2 (downsampleCurrentScan)    (mapOptmization.h:981-993)
//   -> k_gn_init -> [k_gn_knn -> k_gn_residual -> k_gn_solve] x max_iter
//                                                             (mapOptmization.h:1403-1442)
//   -> k_gn_finalize                                          (transformUpdate, :1444-1479)
// with no host round trip between stages (converged jobs drop out on the device).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "fbr_common.h"
#include "fbr_imu.h"
#include "fbr_kernels.h"
#include "fbr_msg.h"

using namespace fbr;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "fbr: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return FBR_ERR_HIP;                                                            \
    }                                                                                \
  } while (0)

namespace {

// Host wall time since t0 into DebugCounters::host_ns[k] (fbr_diag_host_times).
void host_time(int k, std::chrono::steady_clock::time_point t0) {
  const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  debug_counters().host_ns[k].fetch_add((long long)ns, std::memory_order_relaxed);
}

// Blocking host synchronisations, counted (fbr_debug_counters).
hipError_t fbr_sync(hipStream_t s) {
  debug_counters().host_syncs.fetch_add(1, std::memory_order_relaxed);
  return hipStreamSynchronize(s);
}
hipError_t fbr_memcpy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
  debug_counters().host_syncs.fetch_add(1, std::memory_order_relaxed);
  return hipMemcpy(dst, src, bytes, kind);
}

struct KernelTimer {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  double total_ms = 0.0;
  int64_t launches = 0;
};

template <typename T>
int dalloc(T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  CK(hipMalloc((void**)p, sizeof(T) * count));
  return FBR_OK;
}

}  // namespace

constexpr int kMaxSub = 8;  // sub-batch streams per launch (FBR_NSUB); more than 3 pays only with
                             // GPU_MAX_HW_QUEUES above HIP's default of 4 (one hardware queue per stream)

// Host ingest of fbr_process_batch: the caller's (pageable) scans are packed into a ring of pinned
// staging chunks by host threads and copied to HBM on a copy stream, into the input slot the
// running device batch does not read; batch k+1's upload overlaps batch k's compute.
struct Ingest {
  static constexpr int kChunks = 4;
  hipStream_t cstream = nullptr;
  hipStream_t xstream = nullptr;     // k_expand_scans, off the copy stream (FBR_INGEST_XSTREAM=0: on it)
  hipEvent_t copied_ev = nullptr;    // the copies of the current upload are done (on cstream)
  hipEvent_t up_ev[2] = {};          // the upload of input slot s is complete (on xstream / cstream)
  hipEvent_t chunk_ev[kChunks] = {};  // the copies out of chunk k are complete
  bool chunk_used[kChunks] = {};
  int next_chunk = 0;
  uint8_t* h_stage = nullptr;        // kChunks x chunk_bytes, pinned
  int64_t chunk_bytes = 0;
  fbr_point_xyzirt* d_pts_slot[2] = {};  // slot 0 = the context's scan buffer, slot 1 allocated here
  int nthreads = 8;                  // packing threads per chunk
  double h2d_bytes = 0.0;            // bytes copied host -> device by the last fbr_process_batch
  // Compact records (no deskew tables set: `time` is never read): per scan the x, y, z planes
  // (f32) and the rings (u8 below 256 rings), 13 B per point instead of 24, expanded on the device
  // by k_expand_scans (the batch returns poses and statistics, which no point's intensity or time
  // reaches).
  uint8_t* d_stage[2] = {};          // per input slot: [Bcap][ingest_region_bytes(NMAX)] (one per
                                     // slot, so slot s's expand overlaps slot s^1's copies)
  int64_t* d_nin = nullptr;          // [2][2][Bcap] per input slot: the staged scans' point counts,
                                     // then their records' byte offsets in d_stage (copy stream)
  int64_t* h_nin = nullptr;          // [2][2][Bcap] pinned
  bool compact_used = false;         // the last fbr_process_batch used compact records
  bool pk_slot[2] = {};              // input slot s holds 16-B device records (launch_expand_scans pk)
};

// A contiguous sub-batch of jobs driven on one stream.  j0 is the first job of the sub-batch's
// work buffers (every per-job intermediate array, and the Gauss-Newton work-item arrays at
// j0 * items_per_job); in0 the first job of its inputs (raw scans, counts, guesses, deskew tables,
// CropBox statistics).  A batch launch in work slot s has j0 = s * max_batch + in0, so two launches
// in flight never share intermediates.  k indexes the sub-batch's GN flags / counters.
struct Sub {
  int j0, B, k;  // first work job, job count, GN flag index (< kMaxSub)
  hipStream_t st;
  bool stream_mode = false;  // single-scan call (carries stream state) vs independent batch jobs
  int in0 = 0;               // first input job
};

// The Gauss-Newton iterations of one launch that the host has still to enqueue.  The host stays
// `lag` (gn_lag) iterations ahead of each sub-batch and stops once its k_gn_solve reports that no job is
// active (flags in host-mapped memory), so a launch's tail cannot be enqueued before the device
// has run most of it; two launches in flight are advanced together (fbr_batch_launch).
struct GnRun {
  bool pending = false;
  bool trace = false;
  int nsub = 0;
  unsigned long long gen = 0;
  Sub subs[kMaxSub];
  GnArgs a[kMaxSub];
  bool live[kMaxSub] = {}, watch[kMaxSub] = {}, done[kMaxSub] = {};
  int lag = 2;               // gn_lag: iterations enqueued ahead of the latest flag read
  int active[kMaxSub] = {};  // jobs still iterating `lag` iterations ago (an upper bound now)
  int it[kMaxSub] = {};      // next iteration to enqueue
  long polls[kMaxSub] = {};  // unanswered flag reads of the current wait
  std::chrono::steady_clock::time_point wait0[kMaxSub];  // start of the current wait
  int64_t next_query[kMaxSub] = {};  // ns into the current wait of the next stream query
};

// A flag wait asks the runtime whether the stream drained (flags not visible although the work
// is done) only once it has lasted several times longer than the waits of its kind usually do:
// hipStreamQuery puts a marker into the stream, and a marker between two iterations' kernels cost
// ~5.7 us on the device (every launch enqueued after a wait had one).  The bound is 4x the
// smoothed duration of the completed waits of that kind (GN flags of batch runs, of single-scan
// runs, single-scan direct results), within [kQueryMinNs, kQueryMaxNs]; queries repeat at most
// every half bound.  (Round 5 used a fixed 2 ms, which a late-visible flag turned into a 2 ms scan.)
// The floor stays above the longest normal single-scan wait (0.44 ms measured, r06c): at 150 us
// about one wait per scan queried its stream, and each query is a marker before the next kernel.
constexpr int64_t kQueryMinNs = 500000, kQueryMaxNs = 2000000;
struct WaitBound {
  double ema_ns = 0.0;
  int64_t after() const {
    return ema_ns <= 0.0 ? kQueryMaxNs : std::min<int64_t>(kQueryMaxNs, std::max<int64_t>(kQueryMinNs, (int64_t)(4.0 * ema_ns)));
  }
  void done(int64_t ns) { ema_ns = ema_ns <= 0.0 ? (double)ns : 0.875 * ema_ns + 0.125 * (double)ns; }
};
enum { kWaitBatchFlag = 0, kWaitScanFlag = 1, kWaitDirect = 2 };
// Every completed wait into the process-wide wait statistics (fbr_diag_wait_stats).
void wait_stat(int64_t ns) {
  DebugCounters& d = debug_counters();
  if (ns > 1000000) d.waits_over_1ms.fetch_add(1, std::memory_order_relaxed);
  long long m = d.wait_max_ns.load(std::memory_order_relaxed);
  while (ns > m && !d.wait_max_ns.compare_exchange_weak(m, ns, std::memory_order_relaxed)) {
  }
}

struct fbr_ctx {
  fbr_params P;
  int dev = 0;
  hipStream_t stream = nullptr;   // primary stream (single-scan calls, batch sub-batch 0, export)
  hipStream_t xstream[kMaxSub] = {};  // extra streams of batch sub-batches 1.. (index 0 unused)
  hipEvent_t xev[kMaxSub] = {};       // fork / join events
  WaitBound wait_bound[3];            // kWaitBatchFlag / kWaitScanFlag / kWaitDirect
  int nsub_pref = 3;                  // sub-batches per batch launch (FBR_NSUB overrides): 3 unpipelined (at
                                      // B = 128: 2 -> 76.1k, 3 -> 78.5k, 4 -> 46.7k scans/s), 1 pipelined
  int H = 0, W = 0, Bcap = 0;
  // Batch launches rotate over nslot work slots (fbr_params.pipeline_depth, default 3; 1 when max_batch = 1): the
  // next launch's projection / features overlap the previous ones' Gauss-Newton tails.  Work arrays
  // hold Bwork = nslot * Bcap jobs; inputs hold Bcap.
  static constexpr int kMaxSlots = 3;
  int nslot = 1;
  int64_t Bwork = 0;
  GnRun run[kMaxSlots];
  int64_t launch_seq = 0;     // batch launches so far
  int last_slot = -1;         // slot of the latest launch (-1: none since the last stage)
  int64_t slot_launch[kMaxSlots] = {-1, -1, -1};  // launch number of each slot's latest launch
  bool batch_full_masks = false;            // fbr_batch_set_full_masks: launches compute whole masks
  bool slot_full_masks[kMaxSlots] = {};     // ... and which slots' latest launch did
  int64_t exported = -1;      // latest launch whose records fbr_batch_export_ready exported
  int64_t first_valid = 0;    // launches below this id belong to a dropped batch (fbr_batch_allgather)
  int diag_err_job = -1;      // diagnostic (fbr_diag_force_capacity_error): batch job flagged over capacity
  int diag_ring_filter = -1;  // diagnostic (fbr_diag_ring_filter): per-ring surf filter kernel, -1 = by size
  hipEvent_t ev_staged = nullptr;  // the staged inputs are on the device (recorded on stream)
  hipEvent_t ev_fork = nullptr;    // single-scan side-stream fork
  hipEvent_t ev_ext = nullptr;     // a caller's stream, waited on before an export (fbr_batch_export_ready)
  int items_per_job = 0;
  int64_t HW = 0, NMAX = 0;
  // inputs
  fbr_point_xyzirt* d_pts = nullptr;
  // the staged batch's 16-B device records (fbr_kernels.h: x, y, z, ring bits), null = the 24-B
  // scans in d_pts; d_pk backs them for fbr_batch_stage (fbr_process_batch expands into its slots)
  float4* d_pk = nullptr;
  const float4* staged_pk = nullptr;
  bool staged_24 = false;  // d_pts holds the staged batch's 24-B scans (a deskewing launch needs them)
  int64_t* d_nin = nullptr;
  int64_t single_n = -1;  // the single-scan path's point count (k_project's argument, no copy)
  float* d_guess = nullptr;
  // projection
  // owner image generations (OwnerTag, fbr_kernels.h): owner_ib index bits, owner_tmax the last
  // generation before the image is refilled (0: untagged, reset by k_compact)
  int owner_ib = 0;
  int gn_items_hint = 0, gn_items_hint_B = 0;  // the last batch run's work items and its job count
  uint32_t owner_gen = 0, owner_tmax = 0;
  int32_t *d_owner = nullptr, *d_rowcnt = nullptr, *d_col = nullptr, *d_start = nullptr, *d_end = nullptr,
          *d_nvalid = nullptr;
  float4* d_cloud = nullptr;
  float* d_range = nullptr;
  // features
  StreamState* d_sstate = nullptr;    // [Bcap] batch (zeroed per batch)
  StreamState* d_sstream = nullptr;   // [1]   stream mode (persistent)
  int8_t* d_label = nullptr;          // [Bcap][HW]
  int8_t* d_label_stream = nullptr;   // [HW]   stream mode (persistent)
  float4* d_corner_slot = nullptr;
  int32_t* d_corner_cnt = nullptr;
  float4* d_surf_ring = nullptr;
  int32_t* d_surf_ring_cnt = nullptr;
  float* d_ring_box = nullptr;  // [B][H][kRingBox]: k_concat's per-ring cloud bounds
  bool ring_box_valid = false;  // d_corner_all / d_surf_all came from k_concat (not upload_cloud)
  int32_t* d_err = nullptr;
  float4 *d_corner_all = nullptr, *d_surf_all = nullptr, *d_cornerDS = nullptr, *d_surfDS = nullptr;
  int32_t *d_ncorner = nullptr, *d_nsurf = nullptr, *d_ncds = nullptr, *d_nsds = nullptr;
  uint32_t* d_vg_scratch = nullptr;
  int64_t vg_scratch_elems = 0;
  // registration
  GnState* d_gn = nullptr;
  int4* d_items = nullptr;
  int32_t *d_nitems = nullptr, *d_item_range = nullptr, *d_cropcnt = nullptr;
  int32_t* d_cropwork = nullptr;  // [Bwork][2]: a launch's CropBox counts while they accumulate
  double* d_partial = nullptr;
  int32_t* d_nbr = nullptr;
  float* d_fitc = nullptr;     // [max_items][6][256] per-query fit cache (k_gn_residual)
  int8_t* d_fits = nullptr;    // [max_items][256]
  int8_t* d_nsame = nullptr;   // [max_items][256]
  // block-tile kNN (k_knn_tile.hip), allocated by build_map_grids when the map's grids take it:
  int32_t* d_fb_list = nullptr;  // [3][max_items][256] queued / binned query slots, query blocks
  int32_t* d_bin = nullptr;      // [kMaxSub][3][bin_nb] per-block counts, cursors, non-empty list
  int64_t bin_nb = 0, bin_nb_c = 0;
  unsigned long long* h_iter_flags = nullptr;  // host-mapped, written by k_gn_solve
  unsigned long long* d_iter_flags = nullptr;  // its device address
  unsigned long long gn_gen = 0;
  std::set<std::string> profile_only;  // empty: time every kernel
  int32_t* d_iter_cnt = nullptr;
  unsigned char* d_feat_scratch = nullptr;  // k_features sorted-path slots [B*H][gslot_bytes]
  uint8_t* d_msg = nullptr;                 // raw PointCloud2 bytes of the last *_msg call (grown on demand)
  uint64_t msg_cap = 0;
  bool crop_cached = false;  // d_cropcnt holds the staged batch's CropBox statistics
  bool crop_join = false;    // single scan: copy_results takes the CropBox counts from h_crop (side stream)
  int32_t* h_crop = nullptr;  // pinned [2]: the single-scan CropBox counts
  float* h_guess = nullptr;   // pinned [6]: the single-scan guess (queue_guess)
  int max_items = 0;
  float* d_pose_out = nullptr;
  fbr_reg_stats* d_stats = nullptr;
  float* d_trace = nullptr;
  // map
  bool has_map = false;
  DevGrid grid_c, grid_s;  // kNN grids of the corner / surf maps (k_grid.hip)
  std::vector<fbr_point_xyzi> map_c_host, map_s_host;
  // state
  bool have_projection = false;
  int staged_B = 0;
  std::vector<int64_t> staged_nin;
  double time_last = -1.0;
  bool profiling = false;
  std::map<std::string, KernelTimer> timers;
  std::vector<int32_t> last_iters, last_q, last_n, last_m;
  // Work items of the previous single scan: the next one's Gauss-Newton grids are sized from it
  // (2x, at least 16 workgroups) instead of from the capacity bound.  The kernels loop over the
  // items whatever the grid, so the hint only moves time: the C2 bound of ~900 items launched
  // ~870 workgroups (x 8 in the wide kNN mode) that found no item.
  int items_hint = 0;
  unsigned long long* d_feat_stamps = nullptr;  // diagnostic builds (FBR_FEAT_STAMPS) only
  // IMU deskew (fbr_set_deskew)
  fbr_deskew_table* d_desk = nullptr;  // [Bcap] tables (allocated on first use)
  int32_t* d_desk_mode = nullptr;      // [Bcap] kDesk* bits per job
  int32_t* d_rowmin = nullptr;         // [Bcap][H] minimum owner per row
  int32_t* d_choff = nullptr;          // [Bcap][H][W / 32 + 1] compaction tile offsets
  DevArena arena;                      // scratch of the set-up paths (map VoxelGrid, grid builds)
  bool desk_any = false;               // some job has a non-zero mode
  bool no_time_call = false;           // the current call's PointCloud2 has no "time" field
  // LIO-SAM keyframe store (fbr_keyframes_*) and the local map built from it
  std::vector<fbr_keypose> kf_poses;
  std::vector<int64_t> kf_c_off, kf_c_cnt, kf_s_off, kf_s_cnt;
  float4 *d_kf_c = nullptr, *d_kf_s = nullptr;  // lidar-frame keyframe clouds, appended
  int64_t kf_c_cap = 0, kf_s_cap = 0, kf_c_used = 0, kf_s_used = 0;
  float4 *d_kraw_c = nullptr, *d_kraw_s = nullptr;  // concatenated transformed clouds
  int64_t kraw_c_cap = 0, kraw_s_cap = 0;
  float4 *d_kds_c = nullptr, *d_kds_s = nullptr;    // their VoxelGrids (laserCloud*FromMapDS)
  int64_t kds_c_n = 0, kds_s_n = 0;
  KfSeg* d_kf_segs = nullptr;
  int64_t kf_segs_cap = 0;
  int* d_bounds = nullptr;
  bool map_nocrop = false;  // the registration map is a keyframe local map
  int stream_degenerate = 0;  // mapOptimization::isDegenerate across single-scan registrations
  JobResult* d_result = nullptr;          // [Bcap] packed per-job results
  JobResult* h_result = nullptr;          // [Bcap] pinned
  fbr_point_xyzirt* h_scan = nullptr;     // [NMAX] pinned staging of single-scan uploads
  int64_t* h_nin = nullptr;               // pinned scalar
  uint8_t* h_msg = nullptr;               // pinned staging of raw PointCloud2 bytes (grown on demand)
  uint64_t h_msg_cap = 0;
  Ingest ing;                 // fbr_process_batch host ingest (allocated on first use)
  // fbr_process_scan's direct result (GnArgs::direct): the ending k_gn_solve packs the job's
  // result into h_direct (host-mapped); the host spins on its generation word instead of
  // enqueueing finalize + pack + copy and synchronising.  The no-op iterations the host had
  // enqueued ahead of the last flag may still be queued when the call returns (tail_pending):
  // the next single-scan call is ordered after them on the stream, every other entry point
  // synchronises the stream first (enter).
  JobResult* h_direct = nullptr;
  JobResult* d_direct = nullptr;
  int32_t* d_direct_done = nullptr;
  int32_t direct_gen = 0;     // generation of the current single-scan run (0: direct off)
  int32_t direct_gen_seq = 0;
  bool tail_pending = false;
};

namespace {

// Single scans take their result from the ending solve (FBR_DIRECT=0: finalize + pack + copy).
bool direct_results() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_DIRECT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// Every public entry point: the context's device, and no single-scan tail left on the stream
// unless the call is a single scan itself (keep_tail: its work is ordered after the tail).
hipError_t enter(fbr_ctx* c, bool keep_tail = false) {
  hipError_t e = hipSetDevice(c->dev);
  if (e == hipSuccess && c->tail_pending && !keep_tail) {
    e = fbr_sync(c->stream);
    c->tail_pending = false;
  }
  return e;
}

void timer_begin(fbr_ctx* c, hipStream_t st, const char* name, hipEvent_t* ev_end) {
  *ev_end = nullptr;
  if (!c->profiling) return;
  if (!c->profile_only.empty() && c->profile_only.count(name) == 0) return;
  KernelTimer& t = c->timers[name];
  std::pair<hipEvent_t, hipEvent_t> pr;
  if (!t.pool.empty()) {
    pr = t.pool.back();
    t.pool.pop_back();
  } else {
    (void)hipEventCreate(&pr.first);
    (void)hipEventCreate(&pr.second);
  }
  t.pending.push_back(pr);
  *ev_end = pr.second;
  // the launcher's kernels carry the events in their dispatches (fbr_launch, fbr_kernels.h)
  launch_timer() = LaunchTimer{pr.first, pr.second, 0};
}
void timer_end(hipStream_t st, hipEvent_t ev_end) {
  if (!ev_end) return;
  LaunchTimer& t = launch_timer();
  if (!t.launched) {  // nothing dispatched (empty input): a zero-length interval on the stream
    (void)hipEventRecord(t.start, st);
    (void)hipEventRecord(t.stop, st);
  }
  t = LaunchTimer{};
}

// Kernel launch timed by its dispatches' own start / end timestamps (when profiling).
#define TIMED_ON(ctx, st, name, launch)   \
  do {                                    \
    hipEvent_t ev_;                       \
    timer_begin(ctx, st, name, &ev_);     \
    launch;                               \
    timer_end(st, ev_);                   \
  } while (0)
#define TIMED(ctx, name, launch) TIMED_ON(ctx, (ctx)->stream, name, launch)

int64_t seg_cap(int W) { return W / 6 + 8; }

// LDS / scratch capacities of k_features for a Horizon_SCAN of W.
void feat_caps(int W, FeatArgs& a);
int64_t feat_slot_bytes(int W) {
  FeatArgs a{};
  feat_caps(W, a);
  return a.gslot_bytes;
}
void feat_caps(int W, FeatArgs& a) {
  a.lcap = W + 16;
  a.segcap = (int)seg_cap(W);
  a.kseg = 1;
  while (a.kseg < a.segcap - 1) a.kseg <<= 1;
  a.nwcap = (a.lcap + 63) / 64 + 1;
  a.gslot_bytes = (int64_t)features_gslot_bytes(a);
}

int check_params(const fbr_params* p) {
  if (!p) return FBR_ERR_INVALID_ARG;
  if (p->n_scan <= 0 || p->horizon_scan <= 0 || p->horizon_scan > kMaxW) return FBR_ERR_UNSUPPORTED;
  if (p->max_points_per_scan <= 0 || p->max_batch <= 0 || p->max_iterations <= 0) return FBR_ERR_INVALID_ARG;
  if (!(p->odometry_surf_leaf_size > 0 && p->mapping_corner_leaf_size > 0 && p->mapping_surf_leaf_size > 0))
    return FBR_ERR_INVALID_ARG;
  return FBR_OK;
}

// ---------------------------------------------------------------------------------------------
// map grid (built once per fbr_set_map; see k_register.hip for why this replaces the KD-trees)
// ---------------------------------------------------------------------------------------------
// kNN grid cell sizes (powers of two, so cell coordinates and edges are exact), chosen from the
// map density the mapping leaf implies (one point per leaf voxel at most): 1 m along y and z and
// 0.25 m along x for surf leaves >= 0.3 m (the 0.4 m default), 0.5 m / 0.125 m for denser maps
// (measured).  FBR_KNN_CELL / FBR_KNN_CELL_X override; both maps share them.
void grid_cell_sizes(const fbr_params& P, float* inv_yz, float* inv_x) {
  const bool sparse = P.mapping_surf_leaf_size >= 0.3f;
  auto pick = [](const char* name, float def, float lo, float hi) {
    float inv = def;
    if (const char* e = std::getenv(name)) {
      const float cell = std::strtof(e, nullptr);
      if (cell > 0.0f) inv = std::min(hi, std::max(lo, std::exp2(-std::round(std::log2(cell)))));
    }
    return inv;
  };
  *inv_yz = pick("FBR_KNN_CELL", sparse ? 1.0f : 2.0f, 0.5f, 4.0f);  // 2 m .. 0.25 m
  *inv_x = pick("FBR_KNN_CELL_X", sparse ? 4.0f : 8.0f, 0.5f, 8.0f);  // 2 m .. 0.125 m
}

// Clouds at least this large take the device-wide VoxelGrid (FBR_VG_LARGE_MIN overrides; tests
// use it to compare both kernels on the same input).
int64_t vg_large_min() {
  static const int64_t v = [] {
    const char* e = std::getenv("FBR_VG_LARGE_MIN");
    return e ? std::max<int64_t>(1, std::atoll(e)) : kVgLargeMin;
  }();
  return v;
}

// One-segment device VoxelGrid with temporary buffers (map start-up filter, fbr_voxel_grid).
int voxel_grid_once(fbr_ctx* c, const fbr_point_xyzi* in, int64_t n, float leaf, std::vector<fbr_point_xyzi>& out) {
  out.clear();
  if (n <= 0) return FBR_OK;
  // a host cloud with a non-finite point is not dense: PCL's VoxelGrid (and getMinMax3D) skip such
  // points (voxel_grid.cpp, is_dense false), which is the filter over the finite points alone
  for (int64_t i = 0; i < n; ++i)
    if (!(std::isfinite(in[i].x) && std::isfinite(in[i].y) && std::isfinite(in[i].z))) {
      std::vector<fbr_point_xyzi> fin;
      fin.reserve(n);
      for (int64_t j = 0; j < n; ++j)
        if (std::isfinite(in[j].x) && std::isfinite(in[j].y) && std::isfinite(in[j].z)) fin.push_back(in[j]);
      return voxel_grid_once(c, fin.data(), (int64_t)fin.size(), leaf, out);
    }
  if (n > INT32_MAX / 4) return FBR_ERR_CAPACITY;
  float4 *d_in = nullptr, *d_out = nullptr;
  int32_t* d_cnt = nullptr;
  uint32_t* d_sc = nullptr;
  int rc = FBR_OK;
  const bool large = n >= vg_large_min();
  // d_cnt: {input count, output count, look-back error word (k_voxel_grid_split: a part that gave
  // up its look-back flags it, whichever part writes the count)}
  if (dalloc(&d_in, n) || dalloc(&d_out, n) || dalloc(&d_cnt, 3) || (!large && dalloc(&d_sc, kVgScratch * n))) {
    rc = FBR_ERR_HIP;
  } else {
    int32_t nn = (int32_t)n;
    if (hipMemcpyAsync(d_in, in, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(d_cnt, &nn, sizeof(int32_t), hipMemcpyHostToDevice, c->stream) != hipSuccess) {
      rc = FBR_ERR_HIP;
    } else if (large) {
      rc = voxel_grid_large(c->stream, c->arena, d_in, n, leaf, 0, c->P.exact_voxel_order ? 1 : 0, d_out, d_cnt + 1);
      int32_t nout = 0;
      if (!rc && (hipMemcpyAsync(&nout, d_cnt + 1, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                  fbr_sync(c->stream) != hipSuccess))
        rc = FBR_ERR_HIP;
      if (!rc) {
        out.resize(nout);
        if (nout && fbr_memcpy_sync(out.data(), d_out, sizeof(float4) * nout, hipMemcpyDeviceToHost) != hipSuccess)
          rc = FBR_ERR_HIP;
      }
    } else {
      VgArgs a{};
      a.s[0].in = d_in;
      a.s[0].stride_in = n;
      a.s[0].cnt_in = d_cnt;
      a.s[0].cap = n;
      a.s[0].out = d_out;
      a.s[0].stride_out = n;
      a.s[0].cnt_out = d_cnt + 1;
      a.s[0].scratch = d_sc;
      a.s[0].leaf = leaf;
      a.s[0].nseg = 1;
      a.s[0].exact = c->P.exact_voxel_order ? 1 : 0;
      a.err = d_cnt + 2;
      int32_t ce[2] = {0, 0};  // output count, error word
      if (hipMemsetAsync(d_cnt + 2, 0, sizeof(int32_t), c->stream) != hipSuccess) rc = FBR_ERR_HIP;
      if (!rc) launch_voxel_grid(c->stream, a);
      if (rc || hipMemcpyAsync(ce, d_cnt + 1, sizeof(ce), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
          fbr_sync(c->stream) != hipSuccess || ce[0] < 0 || ce[1] != 0) {
        rc = FBR_ERR_HIP;
      } else {
        const int32_t nout = ce[0];
        out.resize(nout);
        if (nout && fbr_memcpy_sync(out.data(), d_out, sizeof(float4) * nout, hipMemcpyDeviceToHost) != hipSuccess)
          rc = FBR_ERR_HIP;
      }
    }
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_cnt);
  (void)hipFree(d_sc);
  return rc;
}

// ---------------------------------------------------------------------------------------------
// pipeline stages
// ---------------------------------------------------------------------------------------------
// Sub-batches (struct Sub above) share the context's buffers without overlapping: the stages offset
// every per-job work array by j0 and every input array by in0.

// Generation-tagged owner images (fbr_kernels.h OwnerTag; FBR_OWNER_TAGS=0: untagged images reset
// by k_compact, for A/B).
bool owner_tags_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_OWNER_TAGS");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// The next owner generation of a projection call.  When the tags run out, every owner image is
// refilled once the device is idle (a call of the previous tag may still be running on another stream).
int next_owner_tag(fbr_ctx* c, OwnerTag* ot) {
  if (!c->owner_tmax) {
    *ot = OwnerTag{0u, 0x7FFFFFFFu, true};
    return FBR_OK;
  }
  if (c->owner_gen >= c->owner_tmax) {
    CK(hipDeviceSynchronize());
    CK(hipMemset(c->d_owner, 0x7F, sizeof(int32_t) * (int64_t)c->Bwork * c->HW));
    CK(hipDeviceSynchronize());
    c->owner_gen = 0;
  }
  const uint32_t g = ++c->owner_gen;
  *ot = OwnerTag{(((uint32_t)kEmptyOwner >> c->owner_ib) - g) << c->owner_ib, (1u << c->owner_ib) - 1u, false};
  return FBR_OK;
}

// The single-scan sub-batch: job slot 0 on the primary stream, stream mode (the state the
// reference's stage objects keep between scans is carried between calls).
Sub single_sub(fbr_ctx* c) { return Sub{0, 1, 0, c->stream, true}; }

int stage_project(fbr_ctx* c, const Sub& sb) {
  const int64_t j0 = sb.j0, i0 = sb.in0;
  DeskArgs desk{nullptr, nullptr, nullptr};
  if (c->desk_any && !c->no_time_call)  // deskewFlag == -1 without a "time" field (:296-297, :548)
    desk = DeskArgs{c->d_desk_mode + i0, c->d_desk + i0, c->d_rowmin + j0 * c->H};
  // batch jobs read the 16-B device records when the staged batch has them and nothing deskews
  const float4* pk = (!sb.stream_mode && !desk.mode && c->staged_pk) ? c->staged_pk + i0 * c->NMAX : nullptr;
  if (!sb.stream_mode && !pk && !c->staged_24) return FBR_ERR_STATE;  // deskew tables set after a 16-B upload
  int32_t* owner = c->d_owner + j0 * c->HW;
  OwnerTag ot;
  const int trc = next_owner_tag(c, &ot);
  if (trc) return trc;
  TIMED_ON(c, sb.st, "project", launch_project(sb.st, c->d_pts + i0 * c->NMAX, c->d_nin + i0, c->NMAX, sb.B, c->H,
                                               c->W, owner, c->d_err + j0, sb.stream_mode ? c->single_n : -1, pk, ot));
  TIMED_ON(c, sb.st, "extract",
           launch_extract(sb.st, c->d_pts + i0 * c->NMAX, c->NMAX, owner, sb.B, c->H, c->W, c->d_rowcnt + j0 * c->H,
                          c->d_choff + j0 * c->H * (c->W / 32 + 1),
                          c->d_cloud + j0 * c->HW, c->d_col + j0 * c->HW, c->d_range + j0 * c->HW,
                          c->d_start + j0 * c->H, c->d_end + j0 * c->H, c->d_nvalid + j0, desk, pk, ot));
  return FBR_OK;
}

// Batch scans as 16-B device records (fbr_kernels.h; FBR_PACKED_SCANS=0: the 24-B scans, for A/B).
bool packed_scans_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_PACKED_SCANS");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// Batch jobs resolve the surf walk only within reach of each segment's end (FeatArgs::surf_full;
// FBR_FEAT_SURF_WINDOW=0: the whole walk, for A/B).
bool feat_surf_window() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_FEAT_SURF_WINDOW");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// err_clear: stage_project has just cleared the jobs' feature-capacity flags (k_project).
// labels_out: cloudLabel is an output of the call (fbr_extract_features), so every surf walk runs
// whole; otherwise only the picks that reach something observable are resolved (FeatArgs).
int stage_features(fbr_ctx* c, const Sub& sb, bool stream_mode, bool err_clear = false, bool labels_out = false) {
  const int64_t j0 = sb.j0, HW = c->HW, H = c->H;
  FeatArgs a{};
  a.B = sb.B;
  a.H = c->H;
  a.W = c->W;
  a.cloud = c->d_cloud + j0 * HW;
  a.col = c->d_col + j0 * HW;
  a.range = c->d_range + j0 * HW;
  a.start_ring = c->d_start + j0 * H;
  a.end_ring = c->d_end + j0 * H;
  a.nvalid = c->d_nvalid + j0;
  a.edge_thr = c->P.edge_threshold;
  a.surf_thr = c->P.surf_threshold;
  if (stream_mode) {
    a.stream = c->d_sstream;
    a.label = c->d_label_stream;
  } else {
    CK(hipMemsetAsync(c->d_sstate + j0, 0, sizeof(StreamState) * sb.B, sb.st));
    a.stream = c->d_sstate + j0;
    a.label = c->d_label + j0 * HW;
  }
  a.corner_slot = c->d_corner_slot + j0 * H * kCornerPerRing;
  a.corner_cnt = c->d_corner_cnt + j0 * H;
  a.err = c->d_err + j0;
  a.surf_full = labels_out || !feat_surf_window() ? 1 : 0;
  a.carry = stream_mode ? 1 : 0;
  a.fresh = stream_mode ? 0 : 1;
  feat_caps(c->W, a);
  a.gscratch = c->d_feat_scratch + j0 * H * a.gslot_bytes;
  a.stamps = c->d_feat_stamps ? c->d_feat_stamps + j0 * H * 12 : nullptr;
  if (!err_clear) CK(hipMemsetAsync(c->d_err + j0, 0, sizeof(int32_t) * sb.B, sb.st));
  TIMED_ON(c, sb.st, "features", launch_features(sb.st, a));
  if (!stream_mode && c->diag_err_job >= sb.in0 && c->diag_err_job < sb.in0 + sb.B)
    CK(hipMemsetD32Async((hipDeviceptr_t)(c->d_err + j0 + (c->diag_err_job - sb.in0)), 1, 1, sb.st));
  VgRing v{};
  v.cloud = a.cloud;
  v.label = a.label;
  v.start_ring = a.start_ring;
  v.end_ring = a.end_ring;
  v.B = sb.B;
  v.H = c->H;
  v.HW = HW;
  v.cap = c->W;
  v.leaf = c->P.odometry_surf_leaf_size;
  v.out = c->d_surf_ring + j0 * HW;
  v.stride_out = c->W;
  v.cnt_out = c->d_surf_ring_cnt + j0 * H;
  v.dbg = std::getenv("FBR_VR_DBG") ? std::atoi(std::getenv("FBR_VR_DBG")) : 0;
  v.exact = c->P.exact_voxel_order ? 1 : 0;
  v.stamps = a.stamps;
  v.kernel = c->diag_ring_filter;
  TIMED_ON(c, sb.st, "voxel_ring", launch_voxel_ring(sb.st, v));
  TIMED_ON(c, sb.st, "concat",
           launch_concat(sb.st, sb.B, c->H, c->W, a.corner_slot, a.corner_cnt, v.out, v.cnt_out,
                         c->d_corner_all + j0 * HW, HW, c->d_ncorner + j0, c->d_surf_all + j0 * HW, HW,
                         c->d_nsurf + j0, c->d_ring_box + j0 * H * kRingBox));
  c->ring_box_valid = true;
  return FBR_OK;
}

GnArgs gn_args(fbr_ctx* c, const Sub& sb, bool trace) {
  const int64_t j0 = sb.j0, HW = c->HW, ib = j0 * c->items_per_job;
  const int mi = std::max(1, c->P.max_iterations);
  GnArgs a{};
#ifdef FBR_KNN_STATS
  a.knn_stats = knn_stats_buffer();
#endif
  a.B = sb.B;
  a.max_iter = c->P.max_iterations;
  a.cornerDS = c->d_cornerDS + j0 * HW;
  a.capc = HW;
  a.ncds = c->d_ncds + j0;
  a.surfDS = c->d_surfDS + j0 * HW;
  a.caps = HW;
  a.nsds = c->d_nsds + j0;
  a.mc = c->grid_c.view();
  a.ms = c->grid_s.view();
  a.gn = c->d_gn + j0;
  a.guess = c->d_guess + (int64_t)sb.in0 * 6;
  a.items = c->d_items + ib;
  a.nitems = c->d_nitems + sb.k;
  a.item_range = c->d_item_range + j0 * 2;
  a.partial = c->d_partial + ib * 32;
  a.max_items = sb.B * c->items_per_job;
  a.edge_min = c->P.edge_feature_min_valid_num;
  a.surf_min = c->P.surf_feature_min_valid_num;
  for (int k = 0; k < 3; ++k) a.crop_half[k] = c->P.crop_half[k];
  a.rot_tol = c->P.rotation_tollerance;
  a.z_tol = c->P.z_tollerance;
  a.pose_out = c->d_pose_out + j0 * 6;
  a.stats = c->d_stats + j0;
  a.trace = trace ? c->d_trace + j0 * c->P.max_iterations * 6 : nullptr;
  a.nbr = c->d_nbr + ib * 5 * 256;
  a.fitc = c->d_fitc + ib * 6 * 256;
  a.fits = c->d_fits + ib * 256;
  a.nsame = c->d_nsame + ib * 256;
  static const int fit_cache = [] {
    const char* e = std::getenv("FBR_FIT_CACHE");
    return e ? std::atoi(e) : 1;
  }();
  a.fit_cache = fit_cache;
  a.iter_flags = c->d_iter_flags + (int64_t)sb.k * mi;
  a.items_flag = c->d_iter_flags + (int64_t)kMaxSub * mi + sb.k;  // after every sub-batch's iteration flags
  a.iter_cnt = c->d_iter_cnt + (int64_t)sb.k * 4 * mi;  // [2 * mi] solve, [mi] queued, [mi] blocks
  if (c->d_bin) {
    const int64_t slots = (int64_t)c->max_items * 256;
    a.fb_list = c->d_fb_list + ib * 256;
    a.bin_list = c->d_fb_list + slots + ib * 256;
    a.qblk = c->d_fb_list + 2 * slots + ib * 256;
    a.bin = c->d_bin + (int64_t)sb.k * 3 * c->bin_nb;
    a.nb_c = (int)c->bin_nb_c;
    a.nb_s = (int)(c->bin_nb - c->bin_nb_c);
  }
  a.desk_mode = c->desk_any ? c->d_desk_mode + sb.in0 : nullptr;
  a.desk = c->desk_any ? c->d_desk + sb.in0 : nullptr;
  a.nocrop = c->map_nocrop ? 1 : 0;
  a.deg_carry = sb.stream_mode ? c->stream_degenerate : 0;
  if (c->direct_gen && sb.stream_mode && sb.B == 1 && c->d_direct) {
    a.direct = c->d_direct;
    a.direct_done = c->d_direct_done;
    a.direct_gen = c->direct_gen;
    a.nvalid = c->d_nvalid + j0;
    a.ncorner = c->d_ncorner + j0;
    a.nsurf = c->d_nsurf + j0;
    a.ferr = c->d_err + j0;
    a.cropcnt = c->d_cropcnt + (int64_t)sb.in0 * 2;
  }
  return a;
}

// Registration of the clouds in d_corner_all / d_surf_all (counts d_ncorner / d_nsurf) from d_guess.
// Single-scan entry points reuse job slot 0 of the device buffers: a staged batch is dropped
// (fbr_batch_launch then reports FBR_ERR_STATE until the next fbr_batch_stage).
int batch_quiesce(fbr_ctx* c);
int drop_staged_batch(fbr_ctx* c) {
  const int rc = batch_quiesce(c);
  c->staged_B = 0;
  c->staged_pk = nullptr;
  c->staged_24 = false;
  c->crop_cached = false;
  c->last_slot = -1;
  // launch ids only grow: every launch made so far belongs to the dropped batch (or its slot was
  // overwritten by a single-scan call), so fbr_batch_export_ready must never hand one of them out
  c->exported = c->launch_seq - 1;
  c->first_valid = c->launch_seq;
  return rc;
}

int crop_stats(fbr_ctx* c, const Sub& sb) {
  GnArgs a = gn_args(c, sb, false);
  int32_t* cnt = c->d_cropcnt + (int64_t)sb.in0 * 2;
  if (c->map_nocrop) {  // keyframe local map: laserCloud*FromMapDSNum = the whole DS map
    std::vector<int32_t> v(2 * sb.B);
    for (int j = 0; j < sb.B; ++j) {
      v[2 * j] = (int32_t)c->grid_c.g.n_points;
      v[2 * j + 1] = (int32_t)c->grid_s.g.n_points;
    }
    CK(hipMemcpyAsync(cnt, v.data(), sizeof(int32_t) * 2 * sb.B, hipMemcpyHostToDevice, sb.st));
    CK(fbr_sync(sb.st));
    return FBR_OK;
  }
  TIMED_ON(c, sb.st, "crop", launch_crop_count(sb.st, a, c->grid_c.pts, c->grid_c.g.n_points, c->grid_s.pts,
                                                c->grid_s.g.n_points, c->d_cropwork + (int64_t)sb.j0 * 2, cnt));
  return FBR_OK;
}

// downsampleCurrentScan (mapOptmization.h:981-993) + the Gauss-Newton set-up of a sub-batch.
int register_prepare(fbr_ctx* c, const Sub& sb, bool trace) {
  const int64_t j0 = sb.j0, HW = c->HW;
  // corner and surf filters in one launch; Morton voxel order (internal clouds: spatially compact
  // query order for the kNN waves)
  VgArgs v{};
  const int64_t ccap = std::min<int64_t>(HW, (int64_t)kCornerPerRing * c->H);
  v.s[0] = VgSet{c->d_surf_all + j0 * HW, HW, c->d_nsurf + j0, HW, c->d_surfDS + j0 * HW, HW, c->d_nsds + j0,
                 c->d_vg_scratch + j0 * kVgScratch * HW, c->P.mapping_surf_leaf_size, sb.B, 1, c->P.exact_voxel_order ? 1 : 0};
  v.s[1] = VgSet{c->d_corner_all + j0 * HW, HW, c->d_ncorner + j0, ccap, c->d_cornerDS + j0 * HW, HW, c->d_ncds + j0,
                 c->d_vg_scratch + c->Bwork * kVgScratch * HW + j0 * kVgScratch * ccap, c->P.mapping_corner_leaf_size,
                 sb.B, 1, c->P.exact_voxel_order ? 1 : 0};
  if (c->ring_box_valid) {  // the clouds' bounds from k_concat: the filter reads each cloud twice, not 3 times
    const float* rb = c->d_ring_box + j0 * c->H * kRingBox;
    for (int k = 0; k < 2; ++k) {
      v.s[k].box = rb + (k == 0 ? 6 : 0);  // set 0 = surf (box floats 6-11), set 1 = corner (0-5)
      v.s[k].box_n = c->H;
      v.s[k].box_stride = (int64_t)c->H * kRingBox;
    }
  }
  v.err = c->d_err + j0;  // a failed split look-back flags the job (FBR_REG_FEATURE_CAPACITY / error)
  TIMED_ON(c, sb.st, "voxel_scan", launch_voxel_grid(sb.st, v));
  GnArgs a = gn_args(c, sb, trace);
  if (trace) CK(hipMemsetAsync(a.trace, 0, sizeof(float) * sb.B * c->P.max_iterations * 6, sb.st));
  TIMED_ON(c, sb.st, "gn_init", launch_gn_init(sb.st, a));  // also zeroes a.iter_cnt
  // map-in-box statistics (from the kNN grid, every launch; the single-scan path runs them on a side
  // stream beside its front end, the keyframe map's are host constants set at staging)
  if (!c->crop_cached) {
    const int rc = crop_stats(c, sb);
    if (rc) return rc;
  }
  return FBR_OK;
}

// Workgroups of the per-iteration GN kernels (each loops over the work items; FBR_GN_GRID overrides).
// 16384 covers the ~11k items of a C2 launch of 341 jobs with one workgroup each (8192 left a second
// round of items to half the workgroups: flat gn_knn -4 % per step, r05q).
int gn_grid_cap() {
  static const int v = [] {
    const char* e = std::getenv("FBR_GN_GRID");
    return e ? std::max(1, std::atoi(e)) : 16384;
  }();
  return v;
}


// One work item per workgroup in the batch kNN / residual launches (GnArgs::one_item;
// FBR_GN_ONE_ITEM=0: grid-stride loops, for A/B).
bool gn_one_item() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_GN_ONE_ITEM");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

bool gn_tail_one_item() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_GN_TAIL_ONE_ITEM");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// Tail mode: once at most 1/FBR_GN_TAIL of a sub-batch's jobs are still iterating (default 8),
// its iterations run fused (kNN + residual in one launch) on a smaller grid: the few remaining
// jobs' work is latency-bound, so one launch less per iteration and fewer idle workgroups
// matter more than the fused kernel's register cost (0 disables).
int gn_tail_div() {
  static const int v = [] {
    const char* e = std::getenv("FBR_GN_TAIL");
    return e ? std::max(0, std::atoi(e)) : 8;
  }();
  return v;
}

// Iterations the host enqueues ahead of a sub-batch's latest flag (FBR_GN_LAG, default 2).  Three
// for single scans (~40 us iterations, a ~5.7 us host gap before each from the third on) measured
// no better: C2 latency p50 0.719 / 0.746 ms against 0.716 / 0.716 with 2 (profiles/r04v_*).
int gn_lag(int jobs) {
  static const int v = [] {
    const char* e = std::getenv("FBR_GN_LAG");
    return e ? std::max(1, std::min(8, std::atoi(e))) : 0;
  }();
  (void)jobs;
  return v ? v : 2;
}

void gn_run_start(fbr_ctx* c, GnRun& r, const Sub* subs, int nsub, bool trace) {
  r = GnRun{};
  r.pending = true;
  r.trace = trace;
  r.nsub = nsub;
  r.gen = ++c->gn_gen;
  int jobs = 0;
  for (int k = 0; k < nsub; ++k) jobs += subs[k].B;
  r.lag = gn_lag(jobs);
  for (int k = 0; k < nsub; ++k) {
    r.subs[k] = subs[k];
    r.a[k] = gn_args(c, subs[k], trace);
    r.live[k] = true;
    r.active[k] = subs[k].B;
    r.watch[k] = c->h_iter_flags != nullptr;
  }
}

// The run's work-item count once iteration 0's solve has published it (GnArgs::items_flag), else -1.
int items_known(fbr_ctx* c, const GnRun& r, int k) {
  if (!c->h_iter_flags) return -1;
  const int mi = std::max(1, c->P.max_iterations);
  const volatile unsigned long long* f = c->h_iter_flags + (int64_t)kMaxSub * mi + r.subs[k].k;
  const unsigned long long v = *f;
  return (v >> 32) == (r.gen & 0xFFFFFFFFull) ? (int)(uint32_t)v : -1;
}

// Workgroups of a one-item launch before the run's item count is known (FBR_GN_ONE_GRID; a C2
// launch of 1,024 jobs has ~25.6k items); the loop launch behind it takes any items past them.
int gn_one_grid() {
  static const int v = [] {
    const char* e = std::getenv("FBR_GN_ONE_GRID");
    return e ? std::max(1, std::atoi(e)) : 32768;
  }();
  return v;
}

// One pass over the run's sub-batches: each enqueues its next iteration if the flag it needs is
// visible (block: wait for it).  A sub-batch whose jobs all stopped, or that reached
// max_iterations, gets its transformUpdate.  *progress: something was enqueued.
int gn_run_pass(fbr_ctx* c, GnRun& r, bool block, bool* progress) {
  const int mi = std::max(1, c->P.max_iterations);
  const unsigned long long g32 = r.gen & 0xFFFFFFFFull;
  bool all_done = true;
  for (int k = 0; k < r.nsub; ++k) {
    if (r.done[k]) continue;
    const Sub& sb = r.subs[k];
    const int it = r.it[k];
    if (r.live[k] && it < c->P.max_iterations && r.watch[k] && it >= r.lag) {
      volatile unsigned long long* f = c->h_iter_flags + (int64_t)sb.k * mi + (it - r.lag);
      unsigned long long v = *f;
      const auto tspin = std::chrono::steady_clock::now();
      if (r.polls[k] == 0) {
        r.wait0[k] = tspin;
        r.next_query[k] = c->wait_bound[sb.stream_mode ? kWaitScanFlag : kWaitBatchFlag].after();
      }
      while ((v >> 32) != g32) {
        if ((++r.polls[k] & 1023) == 1023) {
          const int64_t waited =
              std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - r.wait0[k]).count();
          if (waited > r.next_query[k]) {
            r.next_query[k] = waited + std::max<int64_t>(kQueryMinNs, r.next_query[k] / 2);
            debug_counters().stream_queries.fetch_add(1, std::memory_order_relaxed);
            const hipError_t q = hipStreamQuery(sb.st);
            if (q != hipSuccess && q != hipErrorNotReady) return FBR_ERR_HIP;
            if (q == hipSuccess && ((v = *f) >> 32) != g32) {
              // the stream drained but the host-mapped flag is not visible: the solve's count is in
              // device memory (iter_cnt[2 i]), final once the stream is idle; read it and go on
              // watching (round 5 enqueued every remaining iteration here)
              int32_t cnt = 0;
              if (hipMemcpyAsync(&cnt, r.a[k].iter_cnt + 2 * (it - r.lag), sizeof(cnt), hipMemcpyDeviceToHost, sb.st) !=
                      hipSuccess ||
                  fbr_sync(sb.st) != hipSuccess)
                return FBR_ERR_HIP;
              v = (g32 << 32) | (unsigned long long)(uint32_t)cnt;
              debug_counters().flag_fallbacks.fetch_add(1, std::memory_order_relaxed);
              break;
            }
          }
        }
        if (!block) break;
        v = *f;
      }
      if ((v >> 32) == g32) {  // the wait's duration (from its first poll) into the bound and the stats
        const int64_t waited =
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - r.wait0[k]).count();
        c->wait_bound[sb.stream_mode ? kWaitScanFlag : kWaitBatchFlag].done(waited);
        wait_stat(waited);
      }
      if (block || (v >> 32) == g32 || !r.watch[k])
        debug_counters().batch_ns[1].fetch_add(
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tspin).count(),
            std::memory_order_relaxed);
      if (r.watch[k] && (v >> 32) != g32) {  // not yet (non-blocking pass)
        all_done = false;
        continue;
      }
      r.polls[k] = 0;
      debug_counters().flag_polls.fetch_add(1, std::memory_order_relaxed);
      if (r.watch[k]) r.active[k] = (int)(v & 0xFFFFFFFFull);
      if (r.watch[k] && r.active[k] == 0) r.live[k] = false;
    }
    if (!r.live[k] || it >= c->P.max_iterations) {
      if (!r.a[k].direct) TIMED_ON(c, sb.st, "gn_finalize", launch_gn_finalize(sb.st, r.a[k]));
      CK(hipEventRecord(c->xev[sb.k], sb.st));  // the sub-batch's last work (batch_quiesce joins it)
      r.done[k] = true;
      *progress = true;
      continue;
    }
    all_done = false;
    const bool tail = gn_tail_div() > 0 && (int64_t)r.active[k] * gn_tail_div() <= sb.B;
    // the batch tail also one item per workgroup (the grid then covers the items of the jobs that
    // stopped too, which return at once); FBR_GN_TAIL_ONE_ITEM=0: a 1,024-workgroup loop
    const bool tail_one = tail && !sb.stream_mode && gn_one_item() && gn_tail_one_item();
    int grid = std::max(1, std::min(r.a[k].max_items, tail && !tail_one ? std::min(gn_grid_cap(), 1024) : gn_grid_cap()));
    if (sb.stream_mode && c->items_hint > 0) grid = std::min(grid, std::max(16, 2 * c->items_hint));
    // one-item launches: one workgroup per item once the count is known (no loop launch), before
    // that a grid of gn_one_grid() workgroups and the loop launch behind it
    // (single scans: once the count is known, iteration 2 on; before that the loop over the
    // previous scan's grid, so no second launch sits on their critical path)
    const int nk = gn_one_item() && (!tail || tail_one || sb.stream_mode) ? items_known(c, r, k) : -1;
    const bool one = gn_one_item() && (!tail || tail_one) && (!sb.stream_mode || nk >= 0);
    int one_mode = 0, rest_grid = 0;
    if (one) {
      if (nk >= 0) {
        grid = std::max(1, nk);
        one_mode = 2;
        c->gn_items_hint = nk;  // the next run's first grids
        c->gn_items_hint_B = sb.B;
      } else if (c->gn_items_hint > 0 && c->gn_items_hint_B == sb.B) {
        // a previous run of this many jobs: its count + 25 % + 256, and a small loop launch behind
        grid = std::max(1, std::min(r.a[k].max_items, c->gn_items_hint + c->gn_items_hint / 4 + 256));
        one_mode = 1;
        rest_grid = 64;
      } else {
        grid = std::max(1, std::min(r.a[k].max_items, gn_one_grid()));
        one_mode = 1;
      }
    }
    if (tail) {  // kNN and residual in one launch (whole runs fused: 4 % slower at round 6, r06b)
      GnArgs a1 = r.a[k];
      a1.one_item = one_mode;
      a1.rest_grid = rest_grid;
      // the one-item launch and the loop launch behind it timed apart (rocprof: k_gn_knn / k_gn_loop_*)
      a1.one_part = one_mode == 1 ? 1 : 0;
      TIMED_ON(c, sb.st, "gn_knn", launch_gn_knn(sb.st, a1, grid, it, true));
      if (one_mode == 1) {
        a1.one_part = 2;
        TIMED_ON(c, sb.st, "gn_loop", launch_gn_knn(sb.st, a1, grid, it, true));
      }
    } else {
      GnArgs a1 = r.a[k];
      a1.one_item = one_mode;
      a1.rest_grid = rest_grid;
      a1.one_part = one_mode == 1 ? 1 : 0;
      TIMED_ON(c, sb.st, "gn_knn", launch_gn_knn(sb.st, a1, grid, it, false));
      if (one_mode == 1) {
        a1.one_part = 2;
        TIMED_ON(c, sb.st, "gn_loop", launch_gn_knn(sb.st, a1, grid, it, false));
        a1.one_part = 1;
      }
      TIMED_ON(c, sb.st, "gn_residual", launch_gn_residual(sb.st, a1, grid));
      if (one_mode == 1) {
        a1.one_part = 2;
        TIMED_ON(c, sb.st, "gn_loop", launch_gn_residual(sb.st, a1, grid));
      }
    }
    TIMED_ON(c, sb.st, "gn_solve", launch_gn_solve(sb.st, r.a[k], it, r.gen));
    r.it[k] = it + 1;
    *progress = true;
  }
  if (all_done) r.pending = false;
  return FBR_OK;
}

// Enqueue the rest of a run, waiting for its flags.
int gn_run_finish(fbr_ctx* c, GnRun& r) {
  while (r.pending) {
    bool p = false;
    const int rc = gn_run_pass(c, r, true, &p);
    if (rc) return rc;
  }
  return FBR_OK;
}

// Advance the batch launches in flight together (non-blocking passes; spin while neither can
// progress) until run[target] is fully enqueued (target -1: every run).
int advance_runs(fbr_ctx* c, int target) {
  auto busy = [&] {
    if (target >= 0) return c->run[target].pending;
    for (int q = 0; q < fbr_ctx::kMaxSlots; ++q)
      if (c->run[q].pending) return true;
    return false;
  };
  auto tw = std::chrono::steady_clock::now();
  bool waiting = false;
  while (busy()) {
    bool p = false;
    for (int s = 0; s < fbr_ctx::kMaxSlots; ++s)
      if (c->run[s].pending) {
        const int rc = gn_run_pass(c, c->run[s], false, &p);
        if (rc) return rc;
      }
    if (p && waiting) {
      debug_counters().batch_ns[1].fetch_add(
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tw).count(),
          std::memory_order_relaxed);
      waiting = false;
    } else if (!p && !waiting) {
      waiting = true;
      tw = std::chrono::steady_clock::now();
    }
    if (!p) __builtin_ia32_pause();
  }
  return FBR_OK;
}

// Every batch launch fully enqueued, and the primary stream ordered after all of them (on the
// device): the caller may then overwrite the inputs or use job slot 0 on the primary stream.
int batch_quiesce(fbr_ctx* c) {
  const int rc = advance_runs(c, -1);
  if (rc) return rc;
  for (int s = 0; s < fbr_ctx::kMaxSlots; ++s)
    for (int k = 0; k < c->run[s].nsub; ++k)
      if (c->run[s].subs[k].st != c->stream) CK(hipStreamWaitEvent(c->stream, c->xev[c->run[s].subs[k].k], 0));
  return FBR_OK;
}

// The Gauss-Newton iterations of sub-batches enqueued to the end (single-scan calls).
int register_iterate(fbr_ctx* c, const Sub* subs, int nsub, bool trace) {
  GnRun r;
  gn_run_start(c, r, subs, nsub, trace);
  return gn_run_finish(c, r);
}

int stage_register(fbr_ctx* c, const Sub& sb, bool trace) {
  if (!c->has_map) return FBR_ERR_NO_MAP;
  int rc = register_prepare(c, sb, trace);
  if (!rc) rc = register_iterate(c, &sb, 1, trace);
  return rc;
}

// Per-job results of the last B jobs, packed on the device and returned by one copy (then one
// host synchronisation): poses (when poses_out), stats, and the features' capacity errors
// (FBR_ERR_UNSUPPORTED if any job has one).  with_reg = false: the registration was gated off.
// A single scan's direct result (GnArgs::direct): spin on its generation word; false when the
// stream drained without it (then the caller takes the enqueued path).
int wait_direct(fbr_ctx* c, bool* got) {
  volatile int32_t* gen = &c->h_direct->pad;
  *got = false;
  const auto t0 = std::chrono::steady_clock::now();
  int64_t next_query = c->wait_bound[kWaitDirect].after();
  for (int64_t polls = 1;; ++polls) {
    if (*gen == c->direct_gen) break;
    if ((polls & 1023) == 0) {
      const int64_t waited =
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
      if (waited > next_query) {
        next_query = waited + std::max<int64_t>(kQueryMinNs, next_query / 2);
        debug_counters().stream_queries.fetch_add(1, std::memory_order_relaxed);
        const hipError_t q = hipStreamQuery(c->stream);
        if (q != hipSuccess && q != hipErrorNotReady) return FBR_ERR_HIP;
        if (q == hipSuccess && *gen != c->direct_gen) {  // the caller copies the enqueued results
          debug_counters().flag_fallbacks.fetch_add(1, std::memory_order_relaxed);
          wait_stat(waited);
          return FBR_OK;
        }
      }
    }
    __builtin_ia32_pause();
  }
  {
    const int64_t waited =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    c->wait_bound[kWaitDirect].done(waited);
    wait_stat(waited);
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  std::memcpy(c->h_result, (const void*)c->h_direct, sizeof(JobResult));
  *got = true;
  return FBR_OK;
}

int copy_results(fbr_ctx* c, int B, fbr_reg_stats* stats, float* poses_out, bool with_reg = true, int64_t w0 = 0,
                 bool per_job = false) {
  const auto tw = std::chrono::steady_clock::now();
  bool direct = false;
  if (c->direct_gen && with_reg && B == 1 && w0 == 0 && !per_job) {
    const int rc = wait_direct(c, &direct);
    if (rc) return rc;
    // the stream may still run the no-op iterations enqueued ahead of the last flag (tail_pending)
    if (direct) c->tail_pending = true;
    else TIMED(c, "gn_finalize", launch_gn_finalize(c->stream, gn_args(c, single_sub(c), false)));
  }
  if (!direct) {
    launch_pack_results(c->stream, B, with_reg ? 1 : 0, c->d_pose_out + w0 * 6, c->d_stats + w0, c->d_nvalid + w0,
                        c->d_ncorner + w0, c->d_nsurf + w0, c->d_cropcnt, c->d_err + w0, per_job ? c->d_guess : nullptr,
                        c->d_result);
    CK(hipMemcpyAsync(c->h_result, c->d_result, sizeof(JobResult) * B, hipMemcpyDeviceToHost, c->stream));
    CK(fbr_sync(c->stream));
  }
  if (c->crop_join) {  // the single-scan CropBox statistics: their own copy on the side stream (no
    c->crop_join = false;  // cross-stream dependency on the device; that stream finished long ago)
    CK(fbr_sync(c->xstream[1]));
    c->h_result[0].st.n_corner_map = c->h_crop[0];
    c->h_result[0].st.n_surf_map = c->h_crop[1];
  }
  host_time(2, tw);
  // Single scans: a capacity error (features truncated) fails the call before anything is written
  // (pose_inout keeps the guess, as the reference leaves the pose on a failed scan).  Batches: the
  // failed jobs carry FBR_REG_FEATURE_CAPACITY and their guesses (k_pack_results), the rest their
  // results.
  if (!per_job)
    for (int j = 0; j < B; ++j)
      if (c->h_result[j].err) return FBR_ERR_UNSUPPORTED;
  if (with_reg) {
    c->last_iters.resize(B);
    c->last_q.resize(B);
    c->last_n.resize(B);
    c->last_m.resize(B);
  }
  for (int j = 0; j < B; ++j) {
    const JobResult& r = c->h_result[j];
    if (with_reg) {
      c->last_iters[j] = r.st.iterations;
      c->last_q[j] = r.st.n_corner_ds + r.st.n_surf_ds;
      c->last_n[j] = r.st.n_points;
      c->last_m[j] = r.st.n_corner_map + r.st.n_surf_map;
    }
    if (stats) stats[j] = r.st;
    if (poses_out && with_reg)
      for (int k = 0; k < 6; ++k) poses_out[6 * j + k] = r.pose[k];
  }
  return FBR_OK;
}

int copy_stats(fbr_ctx* c, int B, fbr_reg_stats* stats) { return copy_results(c, B, stats, nullptr, true); }

// Host copy workers of the single-scan uploads, alive for the process (spawning threads per call
// cost ~30 us each).  run(fn) calls fn(p) on participants p = 0..kCopyWorkers (the caller is 0)
// and returns when all are done.  Idle workers spin briefly on the generation counter (back-to-back
// scans find them awake), then sleep on the condition variable.
class CopyPool {
 public:
  // + the caller: 4 host copies of a single-scan upload (7 workers and 256 KB chunks measured
  // slower: latency p50 0.72 -> 0.75 ms, profiles/r04z_latency_8_copiers.txt)
  static constexpr int kWorkers = 3;
  CopyPool() {
    for (int t = 1; t <= kWorkers; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  void run(const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> serial(run_mu_);  // one upload at a time (contexts may share it)
    // adaptive spin: 4x the smoothed interval between uploads, within [1 ms, spin_ns()]
    const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (last_run_ns_ > 0) {
      const double dt = (double)(now - last_run_ns_);
      ema_ns_ = ema_ns_ > 0.0 ? 0.8 * ema_ns_ + 0.2 * dt : dt;
      const int64_t cap = spin_ns();
      spin_cur_.store(std::min<int64_t>(cap, std::max<int64_t>(std::min<int64_t>(cap, 1000000), (int64_t)(4.0 * ema_ns_))));
    }
    last_run_ns_ = now;
    fn_ = &fn;
    pending_.store(kWorkers);
    {
      std::lock_guard<std::mutex> g(mu_);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    fn(0);
    while (pending_.load() != 0) __builtin_ia32_pause();
  }

 private:
  // Idle workers spin after an upload for 4x the smoothed interval between uploads, at least 1 ms
  // and at most spin_us (FBR_COPY_SPIN_US, default 5000 us), so a pose-chained scan stream
  // (one call every ~0.7-0.9 ms, the caller's own work included) finds them awake while a sensor-
  // rate stream (a scan every 100 ms) holds the cores for at most 5 % of the time; then they sleep
  // on the condition variable.  0 = never spin.  A fixed 1000 us spin let late calls find the
  // workers asleep, and the futex wake-up put ms-scale outliers into the upload (p99 3.9 ms).
  static int64_t spin_ns() {
    static const int64_t v = [] {
      const char* e = std::getenv("FBR_COPY_SPIN_US");
      return (int64_t)(e ? std::max(0, std::atoi(e)) : 5000) * 1000;
    }();
    return v;
  }
  void loop(int id) {
    uint64_t seen = 0;
    while (true) {
      uint64_t g = gen_.load();
      const int64_t spin = spin_cur_.load();
      if (g == seen && spin > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; g == seen; ++k) {
          __builtin_ia32_pause();
          g = gen_.load();
          if ((k & 255) == 255 &&
              std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > spin)
            break;
        }
      }
      if (g == seen) {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return gen_.load() != seen; });
        g = gen_.load();
      }
      seen = g;
      if (stop_.load()) return;
      (*fn_)(id);
      pending_.fetch_sub(1);
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  const std::function<void(int)>* fn_ = nullptr;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> spin_cur_{spin_ns()};
  int64_t last_run_ns_ = 0;
  double ema_ns_ = 0.0;
};

CopyPool& copy_pool() {
  static CopyPool* pool = new CopyPool();  // never destroyed: workers may outlive static teardown
  return *pool;
}

// Host bytes -> pinned staging -> device, pipelined: the participants copy 512 KB chunks
// round-robin and each enqueues its chunk's DMA on `st` as soon as the chunk is staged, so the
// copy engine runs while the rest is still being copied (a 64x1800 scan is 2.6 MB).  The chunks
// are disjoint, so their order on the stream does not matter; the caller enqueues the consumer
// after this returns.
hipError_t pinned_upload_async(int dev, void* d_dst, void* h_stage, const void* src, size_t bytes, hipStream_t st) {
  constexpr size_t kChunk = 512 << 10;
  if (bytes <= kChunk) {
    std::memcpy(h_stage, src, bytes);
    return hipMemcpyAsync(d_dst, h_stage, bytes, hipMemcpyHostToDevice, st);
  }
  const size_t nchunk = (bytes + kChunk - 1) / kChunk;
  std::atomic<int> err{(int)hipSuccess};
  const std::function<void(int)> fn = [&](int p) {
    thread_local int cur_dev = -1;  // pool workers serve every context: the stream's device
    if (p > 0 && cur_dev != dev) {
      (void)hipSetDevice(dev);
      cur_dev = dev;
    }
    for (size_t k = (size_t)p; k < nchunk; k += CopyPool::kWorkers + 1) {
      const size_t b = k * kChunk, e = std::min(bytes, b + kChunk);
      std::memcpy((uint8_t*)h_stage + b, (const uint8_t*)src + b, e - b);
      const hipError_t r = hipMemcpyAsync((uint8_t*)d_dst + b, (uint8_t*)h_stage + b, e - b, hipMemcpyHostToDevice, st);
      if (r != hipSuccess) err.store((int)r);
    }
  };
  copy_pool().run(fn);
  return (hipError_t)err.load();
}

// Single-scan uploads stage through our own pinned buffer with a threaded host copy (default;
// 1.00 vs 1.07 ms per pose-chained C2 scan) or hand the caller's pageable buffer to the runtime's
// staging copy (FBR_PINNED_UPLOAD=0).
bool pinned_upload() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_PINNED_UPLOAD");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// A single scan into job slot `job` with no host synchronisation of its own: a copy from pageable
// memory returns once the runtime has staged the source, and the pinned staging buffer is only
// rewritten by the next call, after this call's results came back.
// A single-scan call at `stamp` registers (the mapping_process_interval gate, mapOptmization.h:279).
bool will_register(const fbr_ctx* c, double stamp) { return stamp - c->time_last >= c->P.mapping_process_interval; }

// The registration guess of a single-scan call, queued on the stream ahead of the scan's chunks
// (pinned, so the 24-B DMA runs while the host still copies the first chunk).
hipError_t queue_guess(fbr_ctx* c, const float* guess) {
  if (!guess) return hipSuccess;
  std::memcpy(c->h_guess, guess, sizeof(float) * 6);
  return hipMemcpyAsync(c->d_guess, c->h_guess, sizeof(float) * 6, hipMemcpyHostToDevice, c->stream);
}

int upload_scan(fbr_ctx* c, int job, const fbr_point_xyzirt* pts, int64_t n, const float* guess = nullptr) {
  if (n < 0 || n > c->NMAX) return FBR_ERR_CAPACITY;
  c->no_time_call = false;
  // staging free: a no-op after the previous call's result copy; after a direct result the stream
  // may still hold that call's no-op iterations, which read no staging buffer (the scan's DMA ran
  // before its projection), and this call's work is ordered after them
  if (c->tail_pending) c->tail_pending = false;
  else CK(fbr_sync(c->stream));
  CK(queue_guess(c, guess));
  if (n && pinned_upload()) {
    CK(pinned_upload_async(c->dev, c->d_pts + job * c->NMAX, c->h_scan, pts, sizeof(fbr_point_xyzirt) * n, c->stream));
  } else if (n) {
    CK(hipMemcpyAsync(c->d_pts + job * c->NMAX, pts, sizeof(fbr_point_xyzirt) * n, hipMemcpyHostToDevice, c->stream));
  }
  c->single_n = n;  // k_project takes it as an argument (no 8-B copy ahead of it on the stream)
  (void)job;
  return FBR_OK;
}

// The raw PointCloud2 goes to HBM as it is; k_unpack_msg writes job 0's scan buffer
// (cachePointCloud's fromROSMsg, imageProjection.cpp:253, on the device).
int upload_msg(fbr_ctx* c, const fbr_pointcloud2* msg, int32_t* msg_flags, const float* guess = nullptr) {
  MsgLayout L;
  int rc = resolve_msg(msg, &L);
  if (rc) return rc;
  if (L.n > c->NMAX) return FBR_ERR_CAPACITY;
  if (c->tail_pending) c->tail_pending = false;  // as upload_scan
  else CK(fbr_sync(c->stream));
  CK(queue_guess(c, guess));
  if (L.bytes > c->msg_cap) {
    if (c->d_msg) CK(hipFree(c->d_msg));
    c->d_msg = nullptr;
    c->msg_cap = 0;
    CK(hipMalloc(&c->d_msg, L.bytes));
    c->msg_cap = L.bytes;
  }
  if (L.bytes > c->h_msg_cap) {
    if (c->h_msg) CK(hipHostFree(c->h_msg));
    c->h_msg = nullptr;
    c->h_msg_cap = 0;
    CK(hipHostMalloc((void**)&c->h_msg, L.bytes, hipHostMallocDefault));
    c->h_msg_cap = L.bytes;
  }
  if (L.bytes) {
    CK(pinned_upload_async(c->dev, c->d_msg, c->h_msg, msg->data, L.bytes, c->stream));
  }
  MsgDev D;
  D.n = L.n;
  D.width = L.width;
  D.row_step = L.row_step;
  D.point_step = L.point_step;
  for (int k = 0; k < kMsgFields; ++k) D.off[k] = L.off[k];
  TIMED(c, "unpack_msg", launch_unpack_msg(c->stream, c->d_msg, D, c->d_pts));
  c->single_n = L.n;
  if (msg_flags) *msg_flags = L.flags;
  c->no_time_call = (L.flags & FBR_MSG_NO_TIME) != 0;
  return FBR_OK;
}

int check_err(fbr_ctx* c, int B) {
  std::vector<int32_t> e(B);
  CK(hipMemcpyAsync(e.data(), c->d_err, sizeof(int32_t) * B, hipMemcpyDeviceToHost, c->stream));
  CK(fbr_sync(c->stream));
  for (int j = 0; j < B; ++j)
    if (e[j]) return FBR_ERR_UNSUPPORTED;
  return FBR_OK;
}

int upload_cloud(fbr_ctx* c, float4* dst, int32_t* dcnt, const fbr_point_xyzi* src, int64_t n) {
  if (n < 0 || n > c->HW) return FBR_ERR_CAPACITY;
  if (n && !src) return FBR_ERR_INVALID_ARG;
  c->ring_box_valid = false;  // clouds from the host: the mapping DS takes their bounds from the points
  if (n) CK(hipMemcpyAsync(dst, src, sizeof(float4) * n, hipMemcpyHostToDevice, c->stream));
  int32_t nn = (int32_t)n;
  CK(hipMemcpyAsync(dcnt, &nn, sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  CK(fbr_sync(c->stream));
  return FBR_OK;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// keyframe local map helpers (fbr_extract_surrounding_keyframes)
// ---------------------------------------------------------------------------------------------
namespace {

// Grow a device array to hold `need` elements (keeping `keep` of them).
template <typename T>
int grow(T** p, int64_t* cap, int64_t need, int64_t keep, hipStream_t st) {
  if (need <= *cap) return FBR_OK;
  const int64_t ncap = std::max<int64_t>(need, *cap * 2 + 1024);
  T* q = nullptr;
  CK(hipMalloc((void**)&q, sizeof(T) * ncap));
  if (*p && keep > 0) CK(hipMemcpyAsync(q, *p, sizeof(T) * keep, hipMemcpyDeviceToDevice, st));
  CK(fbr_sync(st));
  if (*p) CK(hipFree(*p));
  *p = q;
  *cap = ncap;
  return FBR_OK;
}

// One-segment device VoxelGrid of a device-resident cloud into a device buffer of n points.
int voxel_grid_dev(fbr_ctx* c, const float4* d_in, int64_t n, float leaf, float4* d_out, int64_t* n_out) {
  *n_out = 0;
  if (n <= 0) return FBR_OK;
  if (n > INT32_MAX / 4) return FBR_ERR_CAPACITY;
  int32_t* d_cnt = nullptr;
  uint32_t* d_sc = nullptr;
  int rc = FBR_OK;
  if (n >= vg_large_min()) {
    int32_t nout = 0;
    if (dalloc(&d_cnt, 1)) return FBR_ERR_HIP;
    rc = voxel_grid_large(c->stream, c->arena, d_in, n, leaf, 0, c->P.exact_voxel_order ? 1 : 0, d_out, d_cnt);
    if (!rc && (hipMemcpyAsync(&nout, d_cnt, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                fbr_sync(c->stream) != hipSuccess))
      rc = FBR_ERR_HIP;
    *n_out = nout;
    (void)hipFree(d_cnt);
    return rc;
  }
  if (dalloc(&d_cnt, 3) || dalloc(&d_sc, kVgScratch * n)) {  // input count, output count, error word
    rc = FBR_ERR_HIP;
  } else {
    int32_t nn = (int32_t)n, ce[2] = {0, 0};
    VgArgs a{};
    a.s[0].in = d_in;
    a.s[0].stride_in = n;
    a.s[0].cnt_in = d_cnt;
    a.s[0].cap = n;
    a.s[0].out = d_out;
    a.s[0].stride_out = n;
    a.s[0].cnt_out = d_cnt + 1;
    a.s[0].scratch = d_sc;
    a.s[0].leaf = leaf;
    a.s[0].nseg = 1;
    a.s[0].exact = c->P.exact_voxel_order ? 1 : 0;
    a.err = d_cnt + 2;  // a lost look-back part flags it, whichever part writes the count
    if (hipMemcpyAsync(d_cnt, &nn, sizeof(int32_t), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemsetAsync(d_cnt + 2, 0, sizeof(int32_t), c->stream) != hipSuccess) {
      rc = FBR_ERR_HIP;
    } else {
      launch_voxel_grid(c->stream, a);
      if (hipMemcpyAsync(ce, d_cnt + 1, sizeof(ce), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
          fbr_sync(c->stream) != hipSuccess || ce[0] < 0 || ce[1] != 0)
        rc = FBR_ERR_HIP;
      *n_out = rc ? 0 : ce[0];
    }
  }
  (void)hipFree(d_cnt);
  (void)hipFree(d_sc);
  return rc;
}

// Both kNN grids of a map (corner, surf) on the device, with one cell size and one layout (the
// kNN kernel is specialised on both): the shared cell sizes of grid_cell_sizes, dense unless a
// map's occupied box is too large, then hashed chunks for both.
int build_map_grids(fbr_ctx* c, const float4* d_corner, int64_t nc, const float4* d_surf, int64_t ns) {
  float inv, invx;
  grid_cell_sizes(c->P, &inv, &invx);
  int rc = grid_build_device(c->stream, c->arena, d_corner, nc, invx, inv, false, c->grid_c);
  if (!rc) rc = grid_build_device(c->stream, c->arena, d_surf, ns, invx, inv, c->grid_c.g.sparse != 0, c->grid_s);
  if (!rc && c->grid_s.g.sparse && !c->grid_c.g.sparse)
    rc = grid_build_device(c->stream, c->arena, d_corner, nc, invx, inv, true, c->grid_c);
  // block-tile kNN buffers (dense 0.5 m x 0.125 m grids only): per-block arrays for every stream
  // a sub-batch may run on, zeroed once (k_bin_tile re-zeroes the counts it used)
  (void)hipFree(c->d_bin);
  c->d_bin = nullptr;
  c->bin_nb = c->bin_nb_c = 0;
  if (!rc && knn_tile_applies(c->grid_c.g, c->grid_s.g)) {
    c->bin_nb_c = knn_tile_blocks(c->grid_c.g);
    c->bin_nb = c->bin_nb_c + knn_tile_blocks(c->grid_s.g);
    const int64_t slots = (int64_t)c->max_items * 256;
    const bool ok = c->bin_nb < (int64_t)1 << 30 &&
                    (c->d_fb_list || hipMalloc(&c->d_fb_list, sizeof(int32_t) * 3 * slots) == hipSuccess) &&
                    hipMalloc(&c->d_bin, sizeof(int32_t) * kMaxSub * 3 * c->bin_nb) == hipSuccess &&
                    hipMemsetAsync(c->d_bin, 0, sizeof(int32_t) * kMaxSub * 3 * c->bin_nb, c->stream) == hipSuccess;
    if (!ok) {  // the grid search serves every query
      (void)hipGetLastError();
      (void)hipFree(c->d_bin);
      c->d_bin = nullptr;
      c->bin_nb = c->bin_nb_c = 0;
    }
  }
  return rc;
}

// pointDistance (utility.h:312-315) of two key poses
float key_distance(const fbr_keypose& a, const fbr_keypose& b) {
  return std::sqrt((a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z));
}

}  // namespace

// =============================================================================================
extern "C" {

void fbr_params_default(fbr_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->n_scan = 16;
  p->horizon_scan = 1800;
  p->edge_threshold = 1.0f;
  p->surf_threshold = 0.1f;
  p->edge_feature_min_valid_num = 10;
  p->surf_feature_min_valid_num = 100;
  p->odometry_surf_leaf_size = 0.4f;
  p->mapping_corner_leaf_size = 0.2f;
  p->mapping_surf_leaf_size = 0.4f;
  p->z_tollerance = 1000.0f;
  p->rotation_tollerance = 1000.0f;
  p->number_of_cores = 4;
  p->mapping_process_interval = 0.15;
  p->crop_half[0] = 30.0f;
  p->crop_half[1] = 30.0f;
  p->crop_half[2] = 10.0f;
  p->max_iterations = 30;
  p->max_points_per_scan = p->n_scan * p->horizon_scan;
  p->max_batch = 1;
}

const char* fbr_strerror(int s) {
  switch (s) {
    case FBR_OK: return "ok";
    case FBR_ERR_INVALID_ARG: return "invalid argument";
    case FBR_ERR_HIP: return "HIP runtime error";
    case FBR_ERR_NO_MAP: return "no map set (call fbr_set_map first)";
    case FBR_ERR_CAPACITY: return "input exceeds the context capacity";
    case FBR_ERR_UNSUPPORTED: return "configuration not supported by the device kernels";
    case FBR_ERR_NO_DEVICE: return "no HIP device available";
    case FBR_ERR_STATE: return "call order violated";
    case FBR_ERR_MSG: return "point cloud message rejected (not dense, or no ring field)";
    default: return "unknown status";
  }
}

int fbr_abi_version(void) { return FBR_ABI_VERSION; }

int fbr_device_count(int* count) {
  if (!count) return FBR_ERR_INVALID_ARG;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return FBR_OK;
}

int fbr_create(fbr_ctx** out, const fbr_params* p, int hip_device) {
  if (!out) return FBR_ERR_INVALID_ARG;
  *out = nullptr;
  int rc = check_params(p);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FBR_ERR_NO_DEVICE;
  if (hip_device < 0 || hip_device >= ndev) return FBR_ERR_INVALID_ARG;
  CK(hipSetDevice(hip_device));
  fbr_ctx* c = new fbr_ctx();
  c->P = *p;
  c->dev = hip_device;
  c->H = p->n_scan;
  c->W = p->horizon_scan;
  c->HW = (int64_t)c->H * c->W;
  c->Bcap = p->max_batch;
  c->NMAX = p->max_points_per_scan;
  if (const char* e = std::getenv("FBR_NSUB")) c->nsub_pref = std::max(1, std::min(kMaxSub, std::atoi(e)));
  // launch slots (fbr_params.pipeline_depth: 0 = the default 3)
  const int pipe = p->pipeline_depth <= 0 ? 3 : std::min(fbr_ctx::kMaxSlots, p->pipeline_depth);
  c->nslot = p->max_batch > 1 ? pipe : 1;
  // Pipelined, one sub-batch per launch is best at every batch size (the two launches in flight
  // overlap as the sub-batches did): B = 128 / 256 / 1024 give 91.8k / 96.7k / 97.4k scans/s
  // against 83.2k / 93.1k / 96.7k with 3 sub-batches (profiles/r04f_pipe_nsub_sweep.txt).  Three
  // slots (the default) against two: B = 128 / 256 96.8k / 100.1k vs 92.6k / 97.8k, B = 1024 equal
  // (profiles/r04n_mfma_pipe_cell_ab.txt).
  if (c->nslot > 1) c->nsub_pref = std::getenv("FBR_NSUB") ? std::min(c->nsub_pref, kMaxSub / c->nslot) : 1;
  c->Bwork = (int64_t)c->nslot * c->Bcap;
  const int64_t B = c->Bcap, Bw = c->Bwork, HW = c->HW, H = c->H;
  // streams of the sub-batches this context can use, per slot (each stream takes a hardware queue:
  // unused ones are not created, so they cannot share a queue with a busy one)
  const int nstreams = std::max(2, c->nslot * c->nsub_pref);
  bool sfail = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess;
  for (int k = 0; k < nstreams && !sfail; ++k) {
    if (k > 0) sfail = hipStreamCreateWithFlags(&c->xstream[k], hipStreamNonBlocking) != hipSuccess;
    if (!sfail) sfail = hipEventCreateWithFlags(&c->xev[k], hipEventDisableTiming) != hipSuccess;
  }
  if (!sfail) sfail = hipEventCreateWithFlags(&c->ev_staged, hipEventDisableTiming) != hipSuccess ||
                     hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
                     hipEventCreateWithFlags(&c->ev_ext, hipEventDisableTiming) != hipSuccess;
  if (sfail) {
    fbr_destroy(c);
    return FBR_ERR_HIP;
  }
  c->items_per_job = (int)(2 * ((HW + 255) / 256 + 1));
  c->max_items = (int)(Bw * c->items_per_job);
  c->vg_scratch_elems = kVgScratch * Bw * (HW + std::min<int64_t>(HW, (int64_t)kCornerPerRing * H));
  // inputs: B jobs; work arrays: Bw jobs (nslot launch slots)
  bool fail = dalloc(&c->d_pts, B * c->NMAX) || dalloc(&c->d_nin, B) || dalloc(&c->d_guess, B * 6) ||
              dalloc(&c->d_owner, Bw * HW) || dalloc(&c->d_rowcnt, Bw * H) || dalloc(&c->d_col, Bw * HW) ||
              dalloc(&c->d_start, Bw * H) || dalloc(&c->d_end, Bw * H) || dalloc(&c->d_nvalid, Bw) ||
              dalloc(&c->d_cloud, Bw * HW) || dalloc(&c->d_range, Bw * HW) || dalloc(&c->d_sstate, Bw) ||
              dalloc(&c->d_sstream, 1) || dalloc(&c->d_label, Bw * HW) || dalloc(&c->d_label_stream, HW) ||
              dalloc(&c->d_corner_slot, Bw * H * kCornerPerRing) || dalloc(&c->d_corner_cnt, Bw * H) ||
              dalloc(&c->d_surf_ring, Bw * HW) ||
              dalloc(&c->d_surf_ring_cnt, Bw * H) || dalloc(&c->d_ring_box, Bw * H * kRingBox) || dalloc(&c->d_err, Bw) ||
              dalloc(&c->d_corner_all, Bw * HW) ||
              dalloc(&c->d_surf_all, Bw * HW) || dalloc(&c->d_cornerDS, Bw * HW) || dalloc(&c->d_surfDS, Bw * HW) ||
              dalloc(&c->d_ncorner, Bw) || dalloc(&c->d_nsurf, Bw) || dalloc(&c->d_ncds, Bw) || dalloc(&c->d_nsds, Bw) ||
              dalloc(&c->d_vg_scratch, c->vg_scratch_elems) ||
              dalloc(&c->d_gn, Bw) || dalloc(&c->d_items, c->max_items) || dalloc(&c->d_nitems, kMaxSub) ||
              dalloc(&c->d_item_range, 2 * Bw) || dalloc(&c->d_cropcnt, 2 * B) || dalloc(&c->d_cropwork, 2 * Bw) ||
              dalloc(&c->d_partial, (int64_t)c->max_items * 32) ||
              dalloc(&c->d_nbr, (int64_t)c->max_items * 5 * 256) ||
              dalloc(&c->d_fitc, (int64_t)c->max_items * 6 * 256) || dalloc(&c->d_fits, (int64_t)c->max_items * 256) ||
              dalloc(&c->d_nsame, (int64_t)c->max_items * 256) ||
              dalloc(&c->d_iter_cnt, kMaxSub * 4 * std::max(1, p->max_iterations)) ||
              dalloc(&c->d_feat_scratch, Bw * H * feat_slot_bytes(c->W)) ||
              hipHostMalloc((void**)&c->h_iter_flags, sizeof(unsigned long long) * kMaxSub * (std::max(1, p->max_iterations) + 1),
                            hipHostMallocMapped) != hipSuccess ||
              hipHostGetDevicePointer((void**)&c->d_iter_flags, c->h_iter_flags, 0) != hipSuccess || dalloc(&c->d_pose_out, Bw * 6) ||
              dalloc(&c->d_stats, Bw) || dalloc(&c->d_trace, Bw * p->max_iterations * 6) ||
              dalloc(&c->d_desk_mode, B) || dalloc(&c->d_rowmin, Bw * H) || dalloc(&c->d_result, B) ||
              dalloc(&c->d_choff, Bw * H * (c->W / 32 + 1)) ||
              hipHostMalloc((void**)&c->h_result, sizeof(JobResult) * B, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&c->h_scan, sizeof(fbr_point_xyzirt) * std::max<int64_t>(c->NMAX, 1),
                            hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&c->h_nin, sizeof(int64_t), hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&c->h_crop, sizeof(int32_t) * 2, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&c->h_guess, sizeof(float) * 6, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&c->h_direct, sizeof(JobResult), hipHostMallocMapped) != hipSuccess ||
              hipHostGetDevicePointer((void**)&c->d_direct, c->h_direct, 0) != hipSuccess ||
              dalloc(&c->d_direct_done, 1);
  if (fail) {
    fbr_destroy(c);
    return FBR_ERR_HIP;
  }
  std::memset(c->h_iter_flags, 0, sizeof(unsigned long long) * kMaxSub * (std::max(1, p->max_iterations) + 1));
  std::memset(c->h_direct, 0, sizeof(JobResult));
  if (hipMemset(c->d_sstream, 0, sizeof(StreamState)) != hipSuccess ||
      hipMemset(c->d_label_stream, 0, HW) != hipSuccess || hipMemset(c->d_col, 0, sizeof(int32_t) * Bw * HW) != hipSuccess ||
      hipMemset(c->d_range, 0, sizeof(float) * Bw * HW) != hipSuccess ||
      hipMemset(c->d_desk_mode, 0, sizeof(int32_t) * B) != hipSuccess ||
      hipMemset(c->d_owner, 0x7F, sizeof(int32_t) * Bw * HW) != hipSuccess) {  // OwnerTag: refilled when the tags run out
    fbr_destroy(c);
    return FBR_ERR_HIP;
  }
  // index bits of the owner claims; tagged while at least 2^6 generations fit (scans up to 2^24 points)
  c->owner_ib = 1;
  while (((int64_t)1 << c->owner_ib) < c->NMAX) ++c->owner_ib;
  c->owner_tmax = (owner_tags_enabled() && c->owner_ib <= 24) ? ((uint32_t)kEmptyOwner >> c->owner_ib) - 1 : 0;
  if (const char* e = std::getenv("FBR_OWNER_TMAX"))  // tests: refill the images every few calls
    if (c->owner_tmax && std::atoi(e) > 0) c->owner_tmax = std::min<uint32_t>(c->owner_tmax, (uint32_t)std::atoi(e));
  *out = c;
  return FBR_OK;
}

int fbr_destroy(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)fbr_sync(c->stream);
  for (int k = 1; k < kMaxSub; ++k)
    if (c->xstream[k]) (void)fbr_sync(c->xstream[k]);
  void* ptrs[] = {c->d_pts, c->d_nin, c->d_guess, c->d_owner, c->d_rowcnt, c->d_col, c->d_start, c->d_end,
                  c->d_nvalid, c->d_cloud, c->d_range, c->d_sstate, c->d_sstream, c->d_label, c->d_label_stream,
                  c->d_corner_slot, c->d_corner_cnt, c->d_surf_ring, c->d_surf_ring_cnt, c->d_ring_box,
                  c->d_err, c->d_corner_all, c->d_surf_all, c->d_cornerDS, c->d_surfDS, c->d_ncorner, c->d_nsurf,
                  c->d_ncds, c->d_nsds, c->d_vg_scratch, c->d_gn, c->d_items, c->d_nitems,
                  c->d_item_range, c->d_cropcnt, c->d_cropwork, c->d_partial, c->d_pose_out, c->d_stats, c->d_trace, c->d_nbr, c->d_fitc, c->d_fits, c->d_nsame, c->d_fb_list, c->d_bin, c->d_iter_cnt, c->d_feat_scratch, c->d_msg,
                  c->d_desk, c->d_desk_mode, c->d_rowmin, c->d_choff,
                  c->d_kf_c, c->d_kf_s, c->d_kraw_c, c->d_kraw_s, c->d_kds_c, c->d_kds_s, c->d_kf_segs, c->d_bounds, c->d_direct_done, c->d_pk};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_iter_flags) (void)hipHostFree(c->h_iter_flags);
  free_grid(c->grid_c);
  free_grid(c->grid_s);
  arena_free(c->arena);
  for (void* h : {(void*)c->h_result, (void*)c->h_scan, (void*)c->h_nin, (void*)c->h_msg, (void*)c->h_crop, (void*)c->h_guess,
                  (void*)c->h_direct})
    if (h) (void)hipHostFree(h);
  if (c->d_result) (void)hipFree(c->d_result);
  if (c->ing.cstream) (void)fbr_sync(c->ing.cstream);
  if (c->ing.xstream) (void)fbr_sync(c->ing.xstream);
  if (c->ing.h_stage) (void)hipHostFree(c->ing.h_stage);
  if (c->ing.d_pts_slot[1]) (void)hipFree(c->ing.d_pts_slot[1]);
  for (uint8_t* d : c->ing.d_stage)
    if (d) (void)hipFree(d);
  if (c->ing.copied_ev) (void)hipEventDestroy(c->ing.copied_ev);
  if (c->ing.d_nin) (void)hipFree(c->ing.d_nin);
  if (c->ing.h_nin) (void)hipHostFree(c->ing.h_nin);
  for (auto& e : c->ing.up_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->ing.chunk_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->ing.cstream) (void)hipStreamDestroy(c->ing.cstream);
  if (c->ing.xstream) (void)hipStreamDestroy(c->ing.xstream);
  for (auto& kv : c->timers) {
    for (auto& pr : kv.second.pending) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
    for (auto& pr : kv.second.pool) {
      (void)hipEventDestroy(pr.first);
      (void)hipEventDestroy(pr.second);
    }
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (int k = 0; k < kMaxSub; ++k) {
    if (c->xstream[k]) (void)hipStreamDestroy(c->xstream[k]);
    if (c->xev[k]) (void)hipEventDestroy(c->xev[k]);
  }
  if (c->ev_staged) (void)hipEventDestroy(c->ev_staged);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_ext) (void)hipEventDestroy(c->ev_ext);
  delete c;
  return FBR_OK;
}

int fbr_set_map(fbr_ctx* c, const fbr_point_xyzi* corner, int64_t n_corner, const fbr_point_xyzi* surf,
                int64_t n_surf) {
  if (!c || n_corner < 0 || n_surf < 0 || (n_corner && !corner) || (n_surf && !surf)) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  c->crop_cached = false;
  c->map_nocrop = false;
  int rc = voxel_grid_once(c, corner, n_corner, c->P.mapping_corner_leaf_size, c->map_c_host);
  if (!rc) rc = voxel_grid_once(c, surf, n_surf, c->P.mapping_surf_leaf_size, c->map_s_host);
  // the DS maps (map-index order) go to HBM once; the grids are built there
  float4 *d_c = nullptr, *d_s = nullptr;
  const int64_t nc = (int64_t)c->map_c_host.size(), ns = (int64_t)c->map_s_host.size();
  if (!rc && (dalloc(&d_c, std::max<int64_t>(nc, 1)) || dalloc(&d_s, std::max<int64_t>(ns, 1)))) rc = FBR_ERR_HIP;
  if (!rc && nc && hipMemcpy(d_c, c->map_c_host.data(), sizeof(float4) * nc, hipMemcpyHostToDevice) != hipSuccess)
    rc = FBR_ERR_HIP;
  if (!rc && ns && hipMemcpy(d_s, c->map_s_host.data(), sizeof(float4) * ns, hipMemcpyHostToDevice) != hipSuccess)
    rc = FBR_ERR_HIP;
  if (!rc) rc = build_map_grids(c, d_c, nc, d_s, ns);
  if (d_c) (void)hipFree(d_c);
  if (d_s) (void)hipFree(d_s);
  c->has_map = rc == FBR_OK;
  return rc;
}

int fbr_map_grid_info(fbr_ctx* c, int64_t info[8]) {
  if (!c || !info) return FBR_ERR_INVALID_ARG;
  if (!c->has_map) return FBR_ERR_NO_MAP;
  const GridDesc& g = c->grid_s.g;
  info[0] = g.sparse;
  info[1] = g.dims[0];
  info[2] = g.dims[1];
  info[3] = g.dims[2];
  info[4] = (int64_t)g.dims[0] * g.dims[1] * g.dims[2];  // cells of the occupied box
  info[5] = g.sparse ? (int64_t)c->grid_c.g.n_cells + g.n_cells : info[4];  // chunks (sparse) / cells
  info[6] = c->grid_c.g.n_points;
  info[7] = g.n_points;
  return FBR_OK;
}

int fbr_get_map(fbr_ctx* c, int64_t* n_corner, int64_t* n_surf, fbr_point_xyzi* corner, fbr_point_xyzi* surf) {
  if (!c) return FBR_ERR_INVALID_ARG;
  if (!c->has_map) return FBR_ERR_NO_MAP;
  if (c->map_nocrop) {  // keyframe local map (device-resident)
    CK(enter(c));
    if (n_corner) *n_corner = c->kds_c_n;
    if (n_surf) *n_surf = c->kds_s_n;
    if (corner && c->kds_c_n) CK(fbr_memcpy_sync(corner, c->d_kds_c, sizeof(float4) * c->kds_c_n, hipMemcpyDeviceToHost));
    if (surf && c->kds_s_n) CK(fbr_memcpy_sync(surf, c->d_kds_s, sizeof(float4) * c->kds_s_n, hipMemcpyDeviceToHost));
    return FBR_OK;
  }
  if (n_corner) *n_corner = (int64_t)c->map_c_host.size();
  if (n_surf) *n_surf = (int64_t)c->map_s_host.size();
  if (corner) std::memcpy(corner, c->map_c_host.data(), sizeof(fbr_point_xyzi) * c->map_c_host.size());
  if (surf) std::memcpy(surf, c->map_s_host.data(), sizeof(fbr_point_xyzi) * c->map_s_host.size());
  return FBR_OK;
}

namespace {
// fbr_project after the scan is in job 0's buffer
int project_uploaded(fbr_ctx* c, int32_t* start_ring, int32_t* end_ring, int32_t* col_ind, float* range,
                     fbr_point_xyzi* cloud, int64_t* n_out);
// fbr_process_scan after the scan is in job 0's buffer
int process_uploaded(fbr_ctx* c, double stamp, float pose_inout[6], fbr_reg_stats* stats);
}  // namespace

int fbr_project(fbr_ctx* c, const fbr_point_xyzirt* points, int64_t n_in, int32_t* start_ring, int32_t* end_ring,
                int32_t* col_ind, float* range, fbr_point_xyzi* cloud, int64_t* n_out) {
  if (!c || (n_in && !points)) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  int rc = drop_staged_batch(c);
  if (rc) return rc;
  rc = upload_scan(c, 0, points, n_in);
  if (rc) return rc;
  return project_uploaded(c, start_ring, end_ring, col_ind, range, cloud, n_out);
}

int fbr_project_msg(fbr_ctx* c, const fbr_pointcloud2* msg, int32_t* start_ring, int32_t* end_ring, int32_t* col_ind,
                    float* range, fbr_point_xyzi* cloud, int64_t* n_out, int32_t* msg_flags) {
  if (!c || !msg) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  int rc = drop_staged_batch(c);
  if (rc) return rc;
  rc = upload_msg(c, msg, msg_flags);
  if (rc) return rc;
  return project_uploaded(c, start_ring, end_ring, col_ind, range, cloud, n_out);
}

namespace {
int project_uploaded(fbr_ctx* c, int32_t* start_ring, int32_t* end_ring, int32_t* col_ind, float* range,
                     fbr_point_xyzi* cloud, int64_t* n_out) {
  int rc = stage_project(c, single_sub(c));
  if (rc) return rc;
  int32_t n = 0;
  CK(hipMemcpyAsync(&n, c->d_nvalid, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  CK(fbr_sync(c->stream));
  if (start_ring) CK(fbr_memcpy_sync(start_ring, c->d_start, sizeof(int32_t) * c->H, hipMemcpyDeviceToHost));
  if (end_ring) CK(fbr_memcpy_sync(end_ring, c->d_end, sizeof(int32_t) * c->H, hipMemcpyDeviceToHost));
  if (col_ind && n) CK(fbr_memcpy_sync(col_ind, c->d_col, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (range && n) CK(fbr_memcpy_sync(range, c->d_range, sizeof(float) * n, hipMemcpyDeviceToHost));
  if (cloud && n) CK(fbr_memcpy_sync(cloud, c->d_cloud, sizeof(float4) * n, hipMemcpyDeviceToHost));
  if (n_out) *n_out = n;
  c->have_projection = true;
  return FBR_OK;
}
}  // namespace

int fbr_extract_features(fbr_ctx* c, int8_t* label, fbr_point_xyzi* corner, int64_t* n_corner, fbr_point_xyzi* surf,
                         int64_t* n_surf) {
  if (!c) return FBR_ERR_INVALID_ARG;
  if (!c->have_projection) return FBR_ERR_STATE;
  CK(enter(c));
  int rc = stage_features(c, single_sub(c), true, false, true);
  if (rc) return rc;
  rc = check_err(c, 1);
  if (rc) return rc;
  int32_t n = 0, nc = 0, ns = 0;
  CK(fbr_memcpy_sync(&n, c->d_nvalid, sizeof(int32_t), hipMemcpyDeviceToHost));
  CK(fbr_memcpy_sync(&nc, c->d_ncorner, sizeof(int32_t), hipMemcpyDeviceToHost));
  CK(fbr_memcpy_sync(&ns, c->d_nsurf, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (label && n) CK(fbr_memcpy_sync(label, c->d_label_stream, (size_t)n, hipMemcpyDeviceToHost));
  if (corner && nc) CK(fbr_memcpy_sync(corner, c->d_corner_all, sizeof(float4) * nc, hipMemcpyDeviceToHost));
  if (surf && ns) CK(fbr_memcpy_sync(surf, c->d_surf_all, sizeof(float4) * ns, hipMemcpyDeviceToHost));
  if (n_corner) *n_corner = nc;
  if (n_surf) *n_surf = ns;
  return FBR_OK;
}

int fbr_register_trace(fbr_ctx* c, const fbr_point_xyzi* corner, int64_t n_corner, const fbr_point_xyzi* surf,
                       int64_t n_surf, float pose_inout[6], fbr_reg_stats* stats, float* trace) {
  if (!c || !pose_inout) return FBR_ERR_INVALID_ARG;
  if (!c->has_map) return FBR_ERR_NO_MAP;
  CK(enter(c));
  int rc = drop_staged_batch(c);
  if (!rc) rc = upload_cloud(c, c->d_corner_all, c->d_ncorner, corner, n_corner);
  if (!rc) rc = upload_cloud(c, c->d_surf_all, c->d_nsurf, surf, n_surf);
  if (rc) return rc;
  CK(hipMemcpyAsync(c->d_guess, pose_inout, sizeof(float) * 6, hipMemcpyHostToDevice, c->stream));
  CK(hipMemsetAsync(c->d_nvalid, 0, sizeof(int32_t), c->stream));
  CK(hipMemsetAsync(c->d_err, 0, sizeof(int32_t), c->stream));  // no feature stage in this call
  rc = stage_register(c, single_sub(c), trace != nullptr);
  if (rc) return rc;
  CK(hipMemcpyAsync(pose_inout, c->d_pose_out, sizeof(float) * 6, hipMemcpyDeviceToHost, c->stream));
  if (trace)
    CK(hipMemcpyAsync(trace, c->d_trace, sizeof(float) * 6 * c->P.max_iterations, hipMemcpyDeviceToHost, c->stream));
  fbr_reg_stats st;
  rc = copy_stats(c, 1, &st);
  if (rc) return rc;
  c->stream_degenerate = st.degenerate;
  st.n_points = 0;
  st.n_corner = (int32_t)n_corner;
  st.n_surf = (int32_t)n_surf;
  if (stats) *stats = st;
  return FBR_OK;
}

int fbr_register(fbr_ctx* c, const fbr_point_xyzi* corner, int64_t n_corner, const fbr_point_xyzi* surf,
                 int64_t n_surf, float pose_inout[6], fbr_reg_stats* stats) {
  return fbr_register_trace(c, corner, n_corner, surf, n_surf, pose_inout, stats, nullptr);
}

int fbr_process_scan(fbr_ctx* c, const fbr_point_xyzirt* points, int64_t n_in, double stamp, float pose_inout[6],
                     fbr_reg_stats* stats) {
  if (!c || !pose_inout || (n_in && !points)) return FBR_ERR_INVALID_ARG;
  const auto t0 = std::chrono::steady_clock::now();
  CK(enter(c, true));
  int rc = drop_staged_batch(c);
  if (rc) return rc;
  rc = upload_scan(c, 0, points, n_in, will_register(c, stamp) ? pose_inout : nullptr);
  if (rc) return rc;
  host_time(0, t0);
  rc = process_uploaded(c, stamp, pose_inout, stats);
  host_time(3, t0);
  return rc;
}

int fbr_process_msg(fbr_ctx* c, const fbr_pointcloud2* msg, double stamp, float pose_inout[6], fbr_reg_stats* stats,
                    int32_t* msg_flags) {
  if (!c || !msg || !pose_inout) return FBR_ERR_INVALID_ARG;
  CK(enter(c, true));
  int rc = drop_staged_batch(c);
  if (rc) return rc;
  rc = upload_msg(c, msg, msg_flags, will_register(c, stamp) ? pose_inout : nullptr);
  if (rc) return rc;
  return process_uploaded(c, stamp, pose_inout, stats);
}

namespace {
// The scan is already queued into job slot 0.  Everything up to the pose runs on the stream with
// no host round trip (the features' capacity error is checked with the results); one packed copy
// and one synchronisation return pose and stats.
int process_uploaded(fbr_ctx* c, double stamp, float pose_inout[6], fbr_reg_stats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  c->crop_join = false;
  const bool run = stamp - c->time_last >= c->P.mapping_process_interval;  // mapOptmization.h:279
  if (run && !c->has_map) return FBR_ERR_NO_MAP;
  int rc = FBR_OK;
  if (run) {
    // the guess went to the device ahead of the scan (queue_guess); the CropBox statistics, which
    // depend only on it, run on a side stream forked here, beside the front end, and copy_results
    // joins them
    CK(hipEventRecord(c->ev_fork, c->stream));
    CK(hipStreamWaitEvent(c->xstream[1], c->ev_fork, 0));
    rc = crop_stats(c, Sub{0, 1, 0, c->xstream[1], true});
    if (rc) return rc;
    CK(hipMemcpyAsync(c->h_crop, c->d_cropcnt, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, c->xstream[1]));
    c->crop_join = true;
  }
  rc = stage_project(c, single_sub(c));
  if (!rc) rc = stage_features(c, single_sub(c), true, true);
  if (rc) return rc;
  c->have_projection = true;
  fbr_reg_stats st;
  std::memset(&st, 0, sizeof(st));
  float pose[6];
  if (run) {
    c->crop_cached = true;
    c->direct_gen = direct_results() ? (c->direct_gen_seq = c->direct_gen_seq % 0x7fffffff + 1) : 0;
    rc = stage_register(c, single_sub(c), false);
    c->crop_cached = false;
    if (rc) {
      c->direct_gen = 0;
      return rc;
    }
  }
  host_time(1, t0);
  rc = copy_results(c, 1, &st, pose, run);
  c->direct_gen = 0;
  if (rc) return rc;  // capacity error: the pose stays the guess, the time gate is not consumed
  if (run) {
    c->time_last = stamp;
    for (int k = 0; k < 6; ++k) pose_inout[k] = pose[k];
    c->stream_degenerate = st.degenerate;
    c->items_hint = (st.n_corner_ds + 255) / 256 + (st.n_surf_ds + 255) / 256;  // 256-query items (k_gn_init)
  }
  if (stats) *stats = st;
  return FBR_OK;
}
}  // namespace

int fbr_reset_stream(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  CK(hipMemsetAsync(c->d_sstream, 0, sizeof(StreamState), c->stream));
  CK(hipMemsetAsync(c->d_label_stream, 0, c->HW, c->stream));
  CK(hipMemsetAsync(c->d_col, 0, sizeof(int32_t) * c->HW, c->stream));
  CK(hipMemsetAsync(c->d_range, 0, sizeof(float) * c->HW, c->stream));
  CK(fbr_sync(c->stream));
  c->time_last = -1.0;
  c->have_projection = false;
  c->stream_degenerate = 0;
  return FBR_OK;
}

int fbr_batch_stage(fbr_ctx* c, const fbr_point_xyzirt* const* scans, const int64_t* n_in, int n_jobs,
                    const float* poses_in) {
  if (!c || !scans || !n_in || !poses_in || n_jobs <= 0) return FBR_ERR_INVALID_ARG;
  if (n_jobs > c->Bcap) return FBR_ERR_CAPACITY;
  // every job is validated before anything is copied: a rejected batch leaves the previous one's
  // buffers untouched, and nothing stays staged after a failure
  for (int j = 0; j < n_jobs; ++j) {
    if (n_in[j] < 0 || n_in[j] > c->NMAX) return FBR_ERR_CAPACITY;
    if (n_in[j] && !scans[j]) return FBR_ERR_INVALID_ARG;
  }
  CK(enter(c));
  int rc = drop_staged_batch(c);  // launches in flight read the inputs: they are enqueued first
  if (rc) return rc;
  c->no_time_call = false;
  auto q = [&](hipError_t e) {
    if (e != hipSuccess && !rc) rc = FBR_ERR_HIP;
  };
  // Without deskew tables the scans go over as 16-B device records (x, y, z, ring bits; packed by
  // host threads, as fbr_process_batch's compact records are); a deskewing batch keeps the 24-B
  // scans, whose time deskewPoint reads.
  const bool pk = packed_scans_enabled() && !c->desk_any;
  if (pk) {
    if (!c->d_pk && dalloc(&c->d_pk, (int64_t)c->Bcap * c->NMAX)) return FBR_ERR_HIP;
    std::vector<float4> rec;
    for (int j0 = 0; j0 < n_jobs && !rc; j0 += 64) {  // 64 scans per host buffer (~118 MB for C2)
      const int j1 = std::min(n_jobs, j0 + 64);
      std::vector<int64_t> at(j1 - j0 + 1, 0);
      for (int j = j0; j < j1; ++j) at[j - j0 + 1] = at[j - j0] + n_in[j];
      rec.resize((size_t)at.back());
      const int nt = std::max(1, std::min(16, j1 - j0));
      auto pack = [&](int t) {
        for (int j = j0 + t; j < j1; j += nt) {
          const fbr_point_xyzirt* P = scans[j];
          float4* o = rec.data() + at[j - j0];
          for (int64_t i = 0; i < n_in[j]; ++i) {
            float4 v;
            v.x = P[i].x;
            v.y = P[i].y;
            v.z = P[i].z;
            const int32_t ring = P[i].ring;
            std::memcpy(&v.w, &ring, 4);
            o[i] = v;
          }
        }
      };
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back(pack, t);
      pack(0);
      for (auto& x : th) x.join();
      for (int j = j0; j < j1 && !rc; ++j)
        if (n_in[j])
          q(hipMemcpyAsync(c->d_pk + j * c->NMAX, rec.data() + at[j - j0], sizeof(float4) * n_in[j],
                           hipMemcpyHostToDevice, c->stream));
      q(fbr_sync(c->stream));  // rec is refilled next round
    }
  } else {
    for (int j = 0; j < n_jobs && !rc; ++j)
      if (n_in[j])
        q(hipMemcpyAsync(c->d_pts + j * c->NMAX, scans[j], sizeof(fbr_point_xyzirt) * n_in[j],
                         hipMemcpyHostToDevice, c->stream));
  }
  if (!rc) q(hipMemcpyAsync(c->d_nin, n_in, sizeof(int64_t) * n_jobs, hipMemcpyHostToDevice, c->stream));
  if (!rc) q(hipMemcpyAsync(c->d_guess, poses_in, sizeof(float) * 6 * n_jobs, hipMemcpyHostToDevice, c->stream));
  if (!rc && c->has_map && c->map_nocrop) rc = crop_stats(c, Sub{0, n_jobs, 0, c->stream});
  if (!rc) q(hipEventRecord(c->ev_staged, c->stream));  // every launch's streams start after it
  // the caller's host buffers may be reused once this returns: drain the queued copies on every path
  q(fbr_sync(c->stream));
  if (rc) return rc;
  c->crop_cached = c->has_map && c->map_nocrop;
  c->staged_B = n_jobs;
  c->staged_pk = pk ? c->d_pk : nullptr;
  c->staged_24 = !pk;
  c->staged_nin.assign(n_in, n_in + n_jobs);
  return FBR_OK;
}

int fbr_set_deskew(fbr_ctx* c, const fbr_deskew_table* tables, int n_tables) {
  if (!c || n_tables < 0 || (n_tables > 0 && !tables)) return FBR_ERR_INVALID_ARG;
  if (n_tables > c->Bcap) return FBR_ERR_CAPACITY;
  CK(enter(c));
  std::vector<int32_t> mode(c->Bcap, 0);
  bool any = false;
  for (int j = 0; j < n_tables; ++j) {
    if (tables[j].imu_available && (tables[j].imu_pointer_cur < 1 || tables[j].imu_pointer_cur >= FBR_IMU_QUEUE))
      return FBR_ERR_INVALID_ARG;
    // deskewPoint and transformUpdate both key on cloudInfo.imuAvailable (:548, mapOptmization.h:1447)
    mode[j] = tables[j].imu_available ? (kDeskPoints | kDeskImu) : 0;
    any = any || mode[j] != 0;
  }
  if (any && !c->d_desk) CK(hipMalloc((void**)&c->d_desk, sizeof(fbr_deskew_table) * c->Bcap));
  CK(fbr_sync(c->stream));
  if (any) CK(fbr_memcpy_sync(c->d_desk, tables, sizeof(fbr_deskew_table) * n_tables, hipMemcpyHostToDevice));
  CK(fbr_memcpy_sync(c->d_desk_mode, mode.data(), sizeof(int32_t) * c->Bcap, hipMemcpyHostToDevice));
  c->desk_any = any;
  return FBR_OK;
}

int fbr_batch_launch(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  if (c->staged_B <= 0) return FBR_ERR_STATE;
  if (!c->has_map) return FBR_ERR_NO_MAP;
  // deskew tables set after the batch was staged as 16-B records (no time field): stage it again
  if (c->desk_any && !c->no_time_call && !c->staged_24) return FBR_ERR_STATE;
  CK(enter(c));
  const auto t0 = std::chrono::steady_clock::now();
  // Sub-batches on separate streams: one sub-batch's low-occupancy phases (the features' ring-0
  // waves, the last Gauss-Newton iterations) overlap the others' work.  Consecutive launches take
  // alternate work slots with their own streams, and this call returns once the previous launch is
  // fully enqueued: this launch's projection and features run beside the previous one's GN tail.
  const int B = c->staged_B;
  const int slot = (int)(c->launch_seq % c->nslot);
  int rc = advance_runs(c, slot);  // (already enqueued by the previous call: launches n-2 < n-1)
  if (rc) return rc;
  const int nsub = std::max(1, std::min({c->nsub_pref, kMaxSub / c->nslot, B / 8}));
  Sub subs[kMaxSub];
  for (int k = 0; k < nsub; ++k) {
    const int j0 = (int)((int64_t)B * k / nsub), j1 = (int)((int64_t)B * (k + 1) / nsub);
    const int idx = slot * nsub + k;
    subs[k] = Sub{(int)((int64_t)slot * c->Bcap + j0), j1 - j0, idx, idx == 0 ? c->stream : c->xstream[idx], false, j0};
    CK(hipStreamWaitEvent(subs[k].st, c->ev_staged, 0));  // the staged inputs
  }
  for (int k = 0; k < nsub && !rc; ++k) {
    rc = stage_project(c, subs[k]);
    if (!rc && c->batch_full_masks)  // cloudLabel of a fresh FeatureExtraction: zeros outside the picks
      rc = hipMemsetAsync(c->d_label + (int64_t)subs[k].j0 * c->HW, 0, (size_t)subs[k].B * c->HW, subs[k].st) ? FBR_ERR_HIP
                                                                                                            : FBR_OK;
    if (!rc) rc = stage_features(c, subs[k], false, true, c->batch_full_masks);
    if (!rc) rc = register_prepare(c, subs[k], false);
  }
  if (rc) return rc;
  gn_run_start(c, c->run[slot], subs, nsub, false);
  c->last_slot = slot;
  c->slot_full_masks[slot] = c->batch_full_masks;
  c->slot_launch[slot] = c->launch_seq++;
  bool p = false;
  rc = gn_run_pass(c, c->run[slot], false, &p);  // the iterations that need no flag yet
  // return once launch n - (nslot - 1) is fully enqueued (its slot is launch_seq mod nslot now that
  // launch_seq = n + 1; nslot = 1: this launch itself)
  if (!rc) rc = advance_runs(c, (int)(c->launch_seq % c->nslot));
  debug_counters().batch_ns[0].fetch_add(
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
      std::memory_order_relaxed);
  return rc;
}

int fbr_batch_flush(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  return advance_runs(c, -1);
}

int fbr_batch_wait(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  const int rc = batch_quiesce(c);
  if (rc) return rc;
  CK(fbr_sync(c->stream));
  return FBR_OK;
}

int fbr_batch_results(fbr_ctx* c, float* poses_out, fbr_reg_stats* stats) {
  if (!c) return FBR_ERR_INVALID_ARG;
  if (c->staged_B <= 0 || c->last_slot < 0) return FBR_ERR_STATE;
  CK(enter(c));
  const int rc = batch_quiesce(c);
  if (rc) return rc;
  return copy_results(c, c->staged_B, stats, poses_out, true, (int64_t)c->last_slot * c->Bcap, true);
}

int fbr_batch_set_full_masks(fbr_ctx* c, int on) {
  if (!c) return FBR_ERR_INVALID_ARG;
  c->batch_full_masks = on != 0;
  return FBR_OK;
}

int fbr_batch_labels(fbr_ctx* c, int job, int8_t* label, int64_t cap, int64_t* n_out) {
  if (!c || !n_out || cap < 0 || (cap > 0 && !label)) return FBR_ERR_INVALID_ARG;
  *n_out = 0;
  if (c->staged_B <= 0 || c->last_slot < 0) return FBR_ERR_STATE;
  if (job < 0 || job >= c->staged_B) return FBR_ERR_INVALID_ARG;
  if (!c->slot_full_masks[c->last_slot]) return FBR_ERR_STATE;  // window masks are incomplete
  CK(enter(c));
  const int rc = batch_quiesce(c);
  if (rc) return rc;
  const int64_t w = (int64_t)c->last_slot * c->Bcap + job;
  CK(fbr_sync(c->stream));
  for (const GnRun& r : c->run)
    for (int k = 0; k < r.nsub; ++k) CK(fbr_sync(r.subs[k].st));
  int32_t nv = 0;
  CK(hipMemcpy(&nv, c->d_nvalid + w, sizeof(int32_t), hipMemcpyDeviceToHost));
  *n_out = nv;
  if (nv > cap) return FBR_ERR_CAPACITY;
  if (nv > 0) CK(hipMemcpy(label, c->d_label + w * c->HW, (size_t)nv, hipMemcpyDeviceToHost));
  return FBR_OK;
}

int fbr_batch_export(fbr_ctx* c, void* device_dst) {
  if (!c || !device_dst) return FBR_ERR_INVALID_ARG;
  if (c->staged_B <= 0 || c->last_slot < 0) return FBR_ERR_STATE;
  CK(enter(c));
  const int rc = batch_quiesce(c);
  if (rc) return rc;
  const int64_t w0 = (int64_t)c->last_slot * c->Bcap;
  launch_export_records(c->stream, c->staged_B, c->d_pose_out + w0 * 6, c->d_stats + w0, c->d_err + w0, c->d_guess,
                        (float*)device_dst);
  CK(hipGetLastError());
  c->exported = c->slot_launch[c->last_slot];
  return FBR_OK;
}

int fbr_batch_export_ready(fbr_ctx* c, void* device_dst, void* wait_stream, void** export_stream, int64_t* launch_id) {
  if (!c || !device_dst || !export_stream || !launch_id) return FBR_ERR_INVALID_ARG;
  *export_stream = nullptr;
  *launch_id = -1;
  if (c->staged_B <= 0) return FBR_ERR_STATE;
  CK(enter(c));
  // the oldest launch not yet exported, if it is fully enqueued: launches are exported in order
  // (one call per fbr_batch_launch never falls behind: launch n returns with n-1 enqueued)
  int s = -1;
  for (int q = 0; q < c->nslot; ++q)
    if (c->slot_launch[q] > c->exported && c->run[q].nsub > 0 && (s < 0 || c->slot_launch[q] < c->slot_launch[s]))
      s = q;
  if (s < 0 || c->run[s].pending) return FBR_OK;
  const GnRun& r = c->run[s];
  hipStream_t st = r.subs[0].st;
  for (int k = 1; k < r.nsub; ++k) CK(hipStreamWaitEvent(st, c->xev[r.subs[k].k], 0));
  if (wait_stream) {  // the caller's previous reader of device_dst
    CK(hipEventRecord(c->ev_ext, (hipStream_t)wait_stream));
    CK(hipStreamWaitEvent(st, c->ev_ext, 0));
  }
  const int64_t w0 = (int64_t)s * c->Bcap;
  launch_export_records(st, c->staged_B, c->d_pose_out + w0 * 6, c->d_stats + w0, c->d_err + w0, c->d_guess,
                        (float*)device_dst);
  CK(hipGetLastError());
  c->exported = c->slot_launch[s];
  *export_stream = (void*)st;
  *launch_id = c->slot_launch[s];
  return FBR_OK;
}

// ---------------------------------------------------------------------------------------------
// RCCL pose gather.  librccl is opened on first use (dlopen, RTLD_LOCAL): a host
// that never builds a communicator does not need it, and a process that already holds RCCL (torch)
// shares the loaded copy through its soname.  Only the types come from the header.
// ---------------------------------------------------------------------------------------------
}  // extern "C" (reopened below)
#include <rccl/rccl.h>
namespace {
struct RcclApi {
  bool ok = false;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
};
const RcclApi& rccl() {
  static const RcclApi api = [] {
    RcclApi a;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
    if (!h) return a;
    a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
    a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
    a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
    a.comm_abort = (decltype(a.comm_abort))dlsym(h, "ncclCommAbort");
    a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
    a.group_start = (decltype(a.group_start))dlsym(h, "ncclGroupStart");
    a.group_end = (decltype(a.group_end))dlsym(h, "ncclGroupEnd");
    a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.comm_abort && a.all_gather && a.group_start &&
           a.group_end;
    return a;
  }();
  return api;
}
}  // namespace

struct fbr_comm {
  ncclComm_t nc = nullptr;
  int dev = 0, nranks = 0, rank = 0, max_jobs = 0;
  float* send = nullptr;  // [max_jobs][8] this rank's padded records
  hipEvent_t done = nullptr;  // after the latest all-gather: the next one (on another launch's
  bool used = false;          // stream) reuses `send` and the caller's recv buffer
  hipEvent_t ev_wait = nullptr;  // the caller's reader of recv (fbr_batch_allgather's wait_stream)
  bool failed = false;        // a call returned an error: peers may be blocked, destroy aborts
};

extern "C" {

int fbr_comm_unique_id(uint8_t id_out[FBR_COMM_ID_BYTES]) {
  static_assert(FBR_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  if (!id_out) return FBR_ERR_INVALID_ARG;
  if (!rccl().ok) return FBR_ERR_UNSUPPORTED;
  ncclUniqueId id;
  if (rccl().get_unique_id(&id) != ncclSuccess) return FBR_ERR_HIP;
  std::memcpy(id_out, id.internal, FBR_COMM_ID_BYTES);
  return FBR_OK;
}

int fbr_comm_create(fbr_comm** out, fbr_ctx* c, const uint8_t id[FBR_COMM_ID_BYTES], int nranks, int rank,
                    int max_jobs_per_rank) {
  if (!out || !c || !id || nranks < 1 || rank < 0 || rank >= nranks || max_jobs_per_rank < 1) return FBR_ERR_INVALID_ARG;
  *out = nullptr;
  // every batch this ctx can stage fits the rank's block: the collective never fails on capacity
  if (max_jobs_per_rank < c->Bcap) return FBR_ERR_CAPACITY;
  if (!rccl().ok) return FBR_ERR_UNSUPPORTED;
  CK(enter(c));
  fbr_comm* m = new fbr_comm();
  m->dev = c->dev;
  m->nranks = nranks;
  m->rank = rank;
  m->max_jobs = max_jobs_per_rank;
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, FBR_COMM_ID_BYTES);
  if (hipMalloc((void**)&m->send, sizeof(float) * 8 * (size_t)max_jobs_per_rank) != hipSuccess ||
      hipEventCreateWithFlags(&m->done, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&m->ev_wait, hipEventDisableTiming) != hipSuccess) {
    (void)hipFree(m->send);
    if (m->done) (void)hipEventDestroy(m->done);
    delete m;
    return FBR_ERR_HIP;
  }
  // blocks until every rank has joined (bootstrap over the id's socket)
  if (rccl().comm_init_rank(&m->nc, nranks, uid, rank) != ncclSuccess) {
    (void)hipFree(m->send);
    (void)hipEventDestroy(m->done);
    (void)hipEventDestroy(m->ev_wait);
    delete m;
    return FBR_ERR_HIP;
  }
  *out = m;
  return FBR_OK;
}

int fbr_comm_create_local(fbr_comm** out, fbr_ctx* const* ctxs, int n, int max_jobs_per_rank) {
  if (!out || !ctxs || n < 1 || max_jobs_per_rank < 1) return FBR_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i) out[i] = nullptr;
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i]) return FBR_ERR_INVALID_ARG;
    for (int j = 0; j < i; ++j)
      if (ctxs[j]->dev == ctxs[i]->dev) return FBR_ERR_INVALID_ARG;  // one rank per device
    if (max_jobs_per_rank < ctxs[i]->Bcap) return FBR_ERR_CAPACITY;
  }
  if (!rccl().ok) return FBR_ERR_UNSUPPORTED;
  ncclUniqueId uid;
  if (rccl().get_unique_id(&uid) != ncclSuccess) return FBR_ERR_HIP;
  std::vector<fbr_comm*> m(n, nullptr);
  auto cleanup = [&] {
    for (fbr_comm* q : m) {
      if (!q) continue;
      (void)hipSetDevice(q->dev);
      if (q->nc) (void)rccl().comm_abort(q->nc);
      (void)hipFree(q->send);
      if (q->done) (void)hipEventDestroy(q->done);
      if (q->ev_wait) (void)hipEventDestroy(q->ev_wait);
      delete q;
    }
  };
  for (int i = 0; i < n; ++i) {
    if (enter(ctxs[i]) != hipSuccess) {
      cleanup();
      return FBR_ERR_HIP;
    }
    m[i] = new fbr_comm();
    m[i]->dev = ctxs[i]->dev;
    m[i]->nranks = n;
    m[i]->rank = i;
    m[i]->max_jobs = max_jobs_per_rank;
    if (hipMalloc((void**)&m[i]->send, sizeof(float) * 8 * (size_t)max_jobs_per_rank) != hipSuccess ||
        hipEventCreateWithFlags(&m[i]->done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m[i]->ev_wait, hipEventDisableTiming) != hipSuccess) {
      cleanup();
      return FBR_ERR_HIP;
    }
  }
  // every device's rank from this thread: the inits form one group (RCCL would otherwise wait in
  // the first init for ranks this thread has not started yet)
  bool ok = rccl().group_start() == ncclSuccess;
  for (int i = 0; ok && i < n; ++i) {
    ok = hipSetDevice(m[i]->dev) == hipSuccess && rccl().comm_init_rank(&m[i]->nc, n, uid, i) == ncclSuccess;
  }
  ok = (rccl().group_end() == ncclSuccess) && ok;
  if (!ok) {
    cleanup();
    return FBR_ERR_HIP;
  }
  for (int i = 0; i < n; ++i) out[i] = m[i];
  return FBR_OK;
}

int fbr_comm_destroy(fbr_comm* m) {
  if (!m) return FBR_ERR_INVALID_ARG;
  (void)hipSetDevice(m->dev);
  int rc = FBR_OK;
  // after a failed collective the peers may be inside an all-gather this rank never joined:
  // abort (tear down without the collective handshake) instead of destroying
  if (m->nc && (m->failed ? rccl().comm_abort(m->nc) : rccl().comm_destroy(m->nc)) != ncclSuccess) rc = FBR_ERR_HIP;
  (void)hipFree(m->send);
  if (m->done) (void)hipEventDestroy(m->done);
  if (m->ev_wait) (void)hipEventDestroy(m->ev_wait);
  delete m;
  return rc;
}

namespace {
int batch_allgather(fbr_ctx* c, fbr_comm* m, int64_t launch_id, void* recv, void* wait_stream, void** done_stream) {
  if (m->dev != c->dev) return FBR_ERR_INVALID_ARG;
  if (c->staged_B <= 0 || c->launch_seq == 0) return FBR_ERR_STATE;
  if (c->staged_B > m->max_jobs) return FBR_ERR_CAPACITY;  // unreachable: fbr_comm_create checks max_batch
  if (launch_id < 0) launch_id = c->launch_seq - 1;
  if (launch_id < c->first_valid || launch_id >= c->launch_seq) return FBR_ERR_STATE;
  int s = -1;
  for (int q = 0; q < c->nslot; ++q)
    if (c->slot_launch[q] == launch_id) s = q;
  if (s < 0) return FBR_ERR_STATE;  // its slot has been reused by a later launch
  CK(enter(c));
  int rc = advance_runs(c, s);  // the launch fully enqueued (the host follows its GN flags)
  if (rc) return rc;
  const GnRun& r = c->run[s];
  hipStream_t st = r.subs[0].st;
  for (int k = 1; k < r.nsub; ++k) CK(hipStreamWaitEvent(st, c->xev[r.subs[k].k], 0));
  if (m->used) CK(hipStreamWaitEvent(st, m->done, 0));  // the previous gather (maybe another stream)
  if (wait_stream) {  // the caller's reads of the previous result out of recv
    CK(hipEventRecord(m->ev_wait, (hipStream_t)wait_stream));
    CK(hipStreamWaitEvent(st, m->ev_wait, 0));
  }
  const int64_t w0 = (int64_t)s * c->Bcap;
  if (c->staged_B < m->max_jobs)  // padding records: zeros
    CK(hipMemsetAsync(m->send + 8 * (int64_t)c->staged_B, 0, sizeof(float) * 8 * (m->max_jobs - c->staged_B), st));
  launch_export_records(st, c->staged_B, c->d_pose_out + w0 * 6, c->d_stats + w0, c->d_err + w0, c->d_guess, m->send);
  CK(hipGetLastError());
  if (rccl().all_gather(m->send, recv, (size_t)8 * m->max_jobs, ncclFloat32, m->nc, st) != ncclSuccess) return FBR_ERR_HIP;
  CK(hipEventRecord(m->done, st));
  m->used = true;
  if (done_stream) *done_stream = (void*)st;
  else {
    CK(hipEventRecord(c->ev_ext, st));
    CK(hipStreamWaitEvent(c->stream, c->ev_ext, 0));
  }
  return FBR_OK;
}
}  // namespace

int fbr_batch_allgather(fbr_ctx* c, fbr_comm* m, int64_t launch_id, void* recv, void* wait_stream, void** done_stream) {
  if (!c || !m || !recv) return FBR_ERR_INVALID_ARG;
  if (done_stream) *done_stream = nullptr;
  const int rc = batch_allgather(c, m, launch_id, recv, wait_stream, done_stream);
  if (rc) m->failed = true;
  return rc;
}

int fbr_batch_bytes(fbr_ctx* c, double* bytes_total, double* bytes_gn) {
  if (!c) return FBR_ERR_INVALID_ARG;
  if (c->last_iters.empty()) return FBR_ERR_STATE;
  double tot = 0.0, gn = 0.0;
  for (size_t j = 0; j < c->last_iters.size(); ++j) {
    const double nin = j < c->staged_nin.size() ? (double)c->staged_nin[j] : 0.0;
    const double n = c->last_n[j], M = c->last_m[j], Q = c->last_q[j], I = c->last_iters[j];
    const double g = I * 96.0 * Q;  // query 16 B + 5 neighbours x 16 B per iteration
    tot += 22.0 * nin + 80.0 * n + 16.0 * M + 16.0 * Q + g;
    gn += g;
  }
  if (bytes_total) *bytes_total = tot;
  if (bytes_gn) *bytes_gn = gn;
  return FBR_OK;
}

namespace {

// FBR_INGEST_XSTREAM=0: k_expand_scans on the copy stream, one device stage (A/B).
bool ingest_expand_stream() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_INGEST_XSTREAM");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

int ingest_init(fbr_ctx* c) {
  Ingest& g = c->ing;
  if (g.cstream) return FBR_OK;
  int64_t mb = 64;
  if (const char* e = std::getenv("FBR_STAGE_MB")) mb = std::max<int64_t>(1, std::atoll(e));
  g.chunk_bytes = std::max<int64_t>(mb << 20, c->NMAX * (int64_t)sizeof(fbr_point_xyzirt));
  g.chunk_bytes = (g.chunk_bytes + 63) & ~(int64_t)63;  // 16-B aligned records for the streaming stores
  // 16 packing threads (the CPU share of a one-GPU box; 8 -> 16: ingest line +10-20 %, r06m/r06n)
  g.nthreads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (const char* e = std::getenv("FBR_STAGE_THREADS")) g.nthreads = std::max(1, std::atoi(e));
  CK(hipStreamCreateWithFlags(&g.cstream, hipStreamNonBlocking));
  if (ingest_expand_stream()) {
    CK(hipStreamCreateWithFlags(&g.xstream, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&g.copied_ev, hipEventDisableTiming));
  }
  for (auto& e : g.up_ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : g.chunk_ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  CK(hipHostMalloc((void**)&g.h_stage, (size_t)g.chunk_bytes * Ingest::kChunks, hipHostMallocDefault));
  g.d_pts_slot[0] = c->d_pts;
  if (dalloc(&g.d_pts_slot[1], (int64_t)c->Bcap * c->NMAX)) return FBR_ERR_HIP;
  for (int k = 0; k < (g.xstream ? 2 : 1); ++k)
    if (dalloc(&g.d_stage[k], (int64_t)c->Bcap * ingest_region_bytes(c->NMAX))) return FBR_ERR_HIP;
  if (dalloc(&g.d_nin, 4 * (int64_t)c->Bcap)) return FBR_ERR_HIP;
  CK(hipHostMalloc((void**)&g.h_nin, sizeof(int64_t) * 4 * c->Bcap, hipHostMallocDefault));
  return FBR_OK;
}

// FBR_INGEST_NT=0: the packers use plain stores instead of streaming ones.
bool ingest_nt_stores() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_INGEST_NT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// One scan's compact record (fbr_kernels.h: ingest_plane / ingest_region_bytes) at the 16-B aligned
// `out`, in one pass over the caller's 24-B points.  Groups of 16 points go out as streaming stores
// (no read-for-ownership of the pinned chunk, and the caller's points are read once); a ring at or
// beyond H (projectPointCloud drops it, imageProjection.cpp:599) is stored as 255 when rb = 1.
void pack_compact(const fbr_point_xyzirt* src, int64_t n, int H, int rb, uint8_t* out) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const int64_t m = ingest_plane(n);
  float* px = reinterpret_cast<float*>(out);
  float* py = px + m;
  float* pz = py + m;
  uint8_t* rr = out + 12 * m;
  auto ring8 = [&](const fbr_point_xyzirt& p) { return p.ring < H ? (uint8_t)p.ring : (uint8_t)255; };
  int64_t i = 0;
  if (ingest_nt_stores())
    for (; i + 16 <= n; i += 16) {
      const fbr_point_xyzirt* s = src + i;
      for (int g = 0; g < 4; ++g) {
        const fbr_point_xyzirt* q = s + 4 * g;
        __builtin_nontemporal_store(f4{q[0].x, q[1].x, q[2].x, q[3].x}, reinterpret_cast<f4*>(px + i + 4 * g));
        __builtin_nontemporal_store(f4{q[0].y, q[1].y, q[2].y, q[3].y}, reinterpret_cast<f4*>(py + i + 4 * g));
        __builtin_nontemporal_store(f4{q[0].z, q[1].z, q[2].z, q[3].z}, reinterpret_cast<f4*>(pz + i + 4 * g));
      }
      if (rb == 1) {
        u4 w;
        for (int g = 0; g < 4; ++g)
          w[g] = (unsigned)ring8(s[4 * g]) | (unsigned)ring8(s[4 * g + 1]) << 8 |
                 (unsigned)ring8(s[4 * g + 2]) << 16 | (unsigned)ring8(s[4 * g + 3]) << 24;
        __builtin_nontemporal_store(w, reinterpret_cast<u4*>(rr + i));  // 12 m and i are multiples of 16
      } else {
        for (int k = 0; k < 16; ++k) reinterpret_cast<uint16_t*>(rr)[i + k] = s[k].ring;
      }
    }
  for (; i < n; ++i) {
    px[i] = src[i].x;
    py[i] = src[i].y;
    pz[i] = src[i].z;
    if (rb == 1)
      rr[i] = ring8(src[i]);
    else
      reinterpret_cast<uint16_t*>(rr)[i] = src[i].ring;
  }
}

// FBR_INGEST_COMPACT=0: always ship the 24-B records.
bool ingest_compact_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("FBR_INGEST_COMPACT");
    return e ? std::atoi(e) != 0 : true;
  }();
  return v;
}

// Upload B scans into input slot `slot`: pack them into free pinned chunks (host threads), queue
// one H2D copy per chunk (compact records) or per scan (24-B records) on the copy stream, expand the
// compact records into the slot's scan buffer, then record up_ev[slot].  Runs on a worker thread
// while the previous device batch computes.
int ingest_upload(fbr_ctx* c, int slot, const fbr_point_xyzirt* const* scans, const int64_t* n_in, int B) {
  CK(enter(c));
  Ingest& g = c->ing;
  fbr_point_xyzirt* dst = g.d_pts_slot[slot];
  // compact records unless a deskew table may read the per-point time (deskewPoint, :545-580)
  const bool compact = ingest_compact_enabled() && !c->desk_any;
  g.compact_used = compact;
  // compact records expand into 16-B device records (k_project / k_compact read those)
  const bool pk = compact && packed_scans_enabled();
  g.pk_slot[slot] = pk;
  // ring bytes per point: u8 for sensors of < 256 rings, where every out-of-range ring (>= H, which
  // projectPointCloud drops, imageProjection.cpp:599) is stored as 255, still out of range
  const int rb = c->H < 256 ? 1 : 2;
  auto host_bytes = [&](int64_t n) {
    return compact ? 12 * ingest_plane(n) + rb * n : n * (int64_t)sizeof(fbr_point_xyzirt);
  };
  // k_expand_scans' counts and record offsets (the slot's half of the pinned array)
  int64_t* h_nin = g.h_nin + 2 * (int64_t)slot * c->Bcap;
  int64_t* h_off = h_nin + c->Bcap;
  uint8_t* dstage = g.d_stage[g.xstream ? slot : 0];
  int64_t dpos = 0;  // dstage offset of the next chunk: the chunks land back to back
  std::vector<int64_t> off;
  for (int j = 0; j < B;) {
    const int k = g.next_chunk;
    g.next_chunk = (k + 1) % Ingest::kChunks;
    if (g.chunk_used[k]) CK(hipEventSynchronize(g.chunk_ev[k]));  // its previous copies are done
    uint8_t* base = g.h_stage + (int64_t)k * g.chunk_bytes;
    int j1 = j;
    int64_t used = 0;
    off.clear();
    while (j1 < B && used + host_bytes(n_in[j1]) <= g.chunk_bytes) {
      off.push_back(used);
      used += (host_bytes(n_in[j1]) + 15) & ~(int64_t)15;
      ++j1;
    }
    if (j1 == j) return FBR_ERR_CAPACITY;  // (chunk_bytes >= NMAX * 24: not reached)
    const int64_t end = off.back() + host_bytes(n_in[j1 - 1]);  // the chunk's bytes
    for (int jj = j; jj < j1; ++jj) {
      h_nin[jj] = n_in[jj];
      h_off[jj] = dpos + off[jj - j];
    }
    const int nt = std::max(1, std::min(g.nthreads, j1 - j));
    auto pack = [&](int t) {
      for (int jj = j + t; jj < j1; jj += nt) {
        const int64_t n = n_in[jj];
        if (!n) continue;
        if (!compact) {
          std::memcpy(base + off[jj - j], scans[jj], n * sizeof(fbr_point_xyzirt));
          continue;
        }
        pack_compact(scans[jj], n, c->H, rb, base + off[jj - j]);
      }
      if (ingest_nt_stores()) __builtin_ia32_sfence();  // the streaming stores before the DMA reads them
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(pack, t);
    pack(0);
    for (auto& x : th) x.join();
    // compact records: the whole chunk in one copy (1.4 MB copies ran at 41 GB/s on the box, 64 MB
    // ones at 57: tools/h2d_probe.py); 24-B records straight into their scan slots
    if (compact)
      CK(hipMemcpyAsync(dstage + dpos, base, end, hipMemcpyHostToDevice, g.cstream));
    else
      for (int jj = j; jj < j1; ++jj)
        if (n_in[jj])
          CK(hipMemcpyAsync(dst + (int64_t)jj * c->NMAX, base + off[jj - j], n_in[jj] * sizeof(fbr_point_xyzirt),
                            hipMemcpyHostToDevice, g.cstream));
    CK(hipEventRecord(g.chunk_ev[k], g.cstream));
    dpos += (end + 15) & ~(int64_t)15;
    g.chunk_used[k] = true;
    for (int jj = j; jj < j1; ++jj) g.h2d_bytes += (double)(n_in[jj] ? host_bytes(n_in[jj]) : 0);
    j = j1;
  }
  if (compact) {  // stream order: after the copies
    int64_t* d_nin = g.d_nin + 2 * (int64_t)slot * c->Bcap;
    CK(hipMemcpyAsync(d_nin, h_nin, sizeof(int64_t) * 2 * c->Bcap, hipMemcpyHostToDevice, g.cstream));
    hipStream_t es = g.cstream;
    if (g.xstream) {  // the expand off the copy stream: the next upload's copies start at once
      CK(hipEventRecord(g.copied_ev, g.cstream));
      CK(hipStreamWaitEvent(g.xstream, g.copied_ev, 0));
      es = g.xstream;
    }
    launch_expand_scans(es, dstage, c->NMAX, B, d_nin, d_nin + c->Bcap, rb, dst, pk);
    CK(hipEventRecord(g.up_ev[slot], es));
    return FBR_OK;
  }
  CK(hipEventRecord(g.up_ev[slot], g.cstream));
  return FBR_OK;
}

// Stage device batch `slot` whose scans ingest_upload queued: job metadata on the primary stream,
// which then waits for the slot's upload.
int ingest_stage(fbr_ctx* c, int slot, const int64_t* n_in, int B, const float* poses_in) {
  const int rc0 = drop_staged_batch(c);
  if (rc0) return rc0;
  c->no_time_call = false;
  c->d_pts = c->ing.d_pts_slot[slot];
  // 16-B records live in the slot's scan buffer (16 <= 24 B per point at the same NMAX stride)
  c->staged_pk = c->ing.pk_slot[slot] ? reinterpret_cast<const float4*>(c->d_pts) : nullptr;
  CK(hipMemcpyAsync(c->d_nin, n_in, sizeof(int64_t) * B, hipMemcpyHostToDevice, c->stream));
  CK(hipMemcpyAsync(c->d_guess, poses_in, sizeof(float) * 6 * B, hipMemcpyHostToDevice, c->stream));
  CK(hipStreamWaitEvent(c->stream, c->ing.up_ev[slot], 0));
  if (c->has_map && c->map_nocrop) {
    const int rc = crop_stats(c, Sub{0, B, 0, c->stream});
    if (rc) return rc;
  }
  CK(hipEventRecord(c->ev_staged, c->stream));
  CK(fbr_sync(c->stream));  // n_in / poses_in are the caller's
  c->crop_cached = c->has_map && c->map_nocrop;
  c->staged_B = B;
  c->staged_24 = !c->staged_pk;
  c->staged_nin.assign(n_in, n_in + B);
  return FBR_OK;
}

}  // namespace

// Independent jobs in device batches of max_batch.  The scans go through pinned staging on a copy
// stream, double-buffered: batch k+1 is packed and copied while batch k computes.
int fbr_process_batch(fbr_ctx* c, const fbr_point_xyzirt* const* scans, const int64_t* n_in, int n_jobs,
                      float* poses_inout, fbr_reg_stats* stats) {
  if (!c || !scans || !n_in || !poses_inout || n_jobs < 0) return FBR_ERR_INVALID_ARG;
  for (int j = 0; j < n_jobs; ++j) {  // validated before anything is copied
    if (n_in[j] < 0 || n_in[j] > c->NMAX) return FBR_ERR_CAPACITY;
    if (n_in[j] && !scans[j]) return FBR_ERR_INVALID_ARG;
  }
  if (n_jobs == 0) return FBR_OK;
  if (!c->has_map) return FBR_ERR_NO_MAP;
  CK(enter(c));
  int rc = ingest_init(c);
  if (rc) return rc;
  c->ing.h2d_bytes = 0.0;
  const int nb = (n_jobs + c->Bcap - 1) / c->Bcap;
  auto first = [&](int b) { return b * c->Bcap; };
  auto count = [&](int b) { return std::min(c->Bcap, n_jobs - b * c->Bcap); };
  rc = ingest_upload(c, 0, scans, n_in, count(0));
  for (int b = 0; b < nb && !rc; ++b) {
    const int slot = b & 1, j0 = first(b), B = count(b);
    int up_rc = FBR_OK;
    std::thread up;
    if (b + 1 < nb)  // the other slot is free: batch b - 1 finished before its results were read
      up = std::thread([&, b] { up_rc = ingest_upload(c, slot ^ 1, scans + first(b + 1), n_in + first(b + 1), count(b + 1)); });
    rc = ingest_stage(c, slot, n_in + j0, B, poses_inout + 6 * j0);
    if (!rc) rc = fbr_batch_launch(c);
    if (!rc) rc = fbr_batch_wait(c);
    if (!rc) rc = fbr_batch_results(c, poses_inout + 6 * j0, stats ? stats + j0 : nullptr);
    if (up.joinable()) up.join();
    if (!rc) rc = up_rc;
  }
  (void)fbr_sync(c->ing.cstream);
  if (c->ing.xstream) (void)fbr_sync(c->ing.xstream);
  c->d_pts = c->ing.d_pts_slot[0];
  if (rc) (void)drop_staged_batch(c);
  return rc;
}

int fbr_debug_counters(long long* launches, long long* host_syncs, long long* flag_polls, int reset) {
  DebugCounters& d = debug_counters();
  if (launches) *launches = d.launches.load();
  if (host_syncs) *host_syncs = d.host_syncs.load();
  if (flag_polls) *flag_polls = d.flag_polls.load();
  if (reset) {
    d.launches = 0;
    d.host_syncs = 0;
    d.flag_polls = 0;
  }
  return FBR_OK;
}

// Diagnostic: host wall time (ns) of the single-scan calls since the last reset (DebugCounters).
extern "C" int fbr_diag_host_times(long long* out4, int reset) {
  DebugCounters& d = debug_counters();
  for (int k = 0; k < 4; ++k) {
    if (out4) out4[k] = d.host_ns[k].load();
    if (reset) d.host_ns[k] = 0;
  }
  return FBR_OK;
}

// Diagnostic: host waits on device results since the last reset: [0] fallbacks (a flag or a direct
// result not visible although its stream drained: the value is then read from device memory / the
// enqueued copy), [1] completed waits longer than 1 ms, [2] the longest wait (ns), [3] stream
// queries made by the waits.
extern "C" int fbr_diag_wait_stats(long long* out4, int reset) {
  DebugCounters& d = debug_counters();
  std::atomic<long long>* v[4] = {&d.flag_fallbacks, &d.waits_over_1ms, &d.wait_max_ns, &d.stream_queries};
  for (int k = 0; k < 4; ++k) {
    if (out4) out4[k] = v[k]->load();
    if (reset) *v[k] = 0;
  }
  return FBR_OK;
}

// Diagnostic: host wall time (ns) of fbr_batch_launch calls and the part of it spent waiting for
// the Gauss-Newton iteration flags, since the last reset.
extern "C" int fbr_diag_batch_times(long long* out2, int reset) {
  DebugCounters& d = debug_counters();
  for (int k = 0; k < 2; ++k) {
    if (out2) out2[k] = d.batch_ns[k].load();
    if (reset) d.batch_ns[k] = 0;
  }
  return FBR_OK;
}

// Diagnostic: the per-ring surf filter kernel of this context's default-order launches: -1 by
// launch size (four waves per ring above 256 rings, else the 512-thread kernel), 0 the 512-thread
// kernel, 2 four waves per ring -- so a test can compare the two on the same scans.
extern "C" int fbr_diag_ring_filter(fbr_ctx* c, int kernel) {
  if (!c || (kernel != -1 && kernel != 0 && kernel != 2)) return FBR_ERR_INVALID_ARG;
  c->diag_ring_filter = kernel;
  return FBR_OK;
}

// Diagnostic: batch job `job` of the following launches is treated as over the feature capacity
// (as if k_features had flagged it), so the tests can check how fbr_batch_results and the exported
// records report such a job (no valid scan reaches the capacity: a ring holds at most W points);
// job < 0 clears it.
extern "C" int fbr_diag_force_capacity_error(fbr_ctx* c, int job) {
  if (!c) return FBR_ERR_INVALID_ARG;
  c->diag_err_job = job < 0 ? -1 : job;
  return FBR_OK;
}

int fbr_ingest_bytes(fbr_ctx* c, double* h2d_bytes) {
  if (!c || !h2d_bytes) return FBR_ERR_INVALID_ARG;
  *h2d_bytes = c->ing.h2d_bytes;
  return FBR_OK;
}

int fbr_voxel_grid(fbr_ctx* c, const fbr_point_xyzi* in, int64_t n, float leaf, fbr_point_xyzi* out, int64_t* n_out) {
  if (!c || n < 0 || (n && !in) || !(leaf > 0)) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  std::vector<fbr_point_xyzi> o;
  int rc = voxel_grid_once(c, in, n, leaf, o);
  if (rc) return rc;
  if (out) std::memcpy(out, o.data(), sizeof(fbr_point_xyzi) * o.size());
  if (n_out) *n_out = (int64_t)o.size();
  return FBR_OK;
}

// Diagnostic: per-ring phase cycle sums of k_features (only filled by a -DFBR_FEAT_STAMPS build).
extern "C" int fbr_diag_feature_stamps(fbr_ctx* c, unsigned long long* out /* [max_batch*n_scan][12] */) {
  if (!c) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  const size_t n = (size_t)c->Bwork * c->H * 12;  // both launch slots (the first launch uses slot 0)
  if (!c->d_feat_stamps) {
    CK(hipMalloc(&c->d_feat_stamps, sizeof(unsigned long long) * n));
    CK(hipMemset(c->d_feat_stamps, 0, sizeof(unsigned long long) * n));
    return FBR_OK;
  }
  if (out) CK(fbr_memcpy_sync(out, c->d_feat_stamps, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
  return FBR_OK;
}

int fbr_set_profiling(fbr_ctx* c, int enable) {
  if (!c) return FBR_ERR_INVALID_ARG;
  c->profiling = enable != 0;
  return FBR_OK;
}

int fbr_set_profiling_kernels(fbr_ctx* c, const char* names) {
  if (!c) return FBR_ERR_INVALID_ARG;
  c->profile_only.clear();
  if (!names) return FBR_OK;
  std::string cur;
  for (const char* q = names;; ++q) {
    if (*q == ',' || *q == '\0') {
      if (!cur.empty()) c->profile_only.insert(cur);
      cur.clear();
      if (*q == '\0') break;
    } else {
      cur.push_back(*q);
    }
  }
  return FBR_OK;
}

int fbr_kernel_time(fbr_ctx* c, const char* kernel, double* total_ms, int64_t* launches) {
  if (!c || !kernel) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  auto itr = c->timers.find(kernel);
  if (itr == c->timers.end()) {
    if (total_ms) *total_ms = 0.0;
    if (launches) *launches = 0;
    return FBR_OK;
  }
  KernelTimer& t = itr->second;
  for (auto& pr : t.pending) {
    CK(hipEventSynchronize(pr.second));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, pr.first, pr.second));
    t.total_ms += ms;
    t.launches += 1;
    t.pool.push_back(pr);
  }
  t.pending.clear();
  if (total_ms) *total_ms = t.total_ms;
  if (launches) *launches = t.launches;
  return FBR_OK;
}

void* fbr_stream(fbr_ctx* c) { return c ? (void*)c->stream : nullptr; }

// pcl::getTransformation(x, y, z, roll, pitch, yaw) (pcl/common/impl/eigen.hpp), float, with
// glibc's sinf / cosf (fbr_sincosf.h).
void fbr_affine_from_pose(const float pose[6], float m[16]) {
  const float roll = pose[0], pitch = pose[1], yaw = pose[2];
  const float A = fbr::gl_cosf(yaw), B = fbr::gl_sinf(yaw), C = fbr::gl_cosf(pitch), D = fbr::gl_sinf(pitch),
              E = fbr::gl_cosf(roll), F = fbr::gl_sinf(roll), DE = D * E, DF = D * F;
  m[0] = A * C; m[1] = A * DF - B * E; m[2] = B * F + A * DE; m[3] = pose[3];
  m[4] = B * C; m[5] = A * E + B * DF; m[6] = B * DE - A * F; m[7] = pose[4];
  m[8] = -D;    m[9] = C * F;          m[10] = C * E;         m[11] = pose[5];
  m[12] = 0.0f; m[13] = 0.0f; m[14] = 0.0f; m[15] = 1.0f;
}

// pcl::getTranslationAndEulerAngles (pcl/common/impl/eigen.hpp), float.
void fbr_pose_from_affine(const float m[16], float pose[6]) {
  pose[3] = m[3];
  pose[4] = m[7];
  pose[5] = m[11];
  pose[0] = std::atan2(m[9], m[10]);
  pose[1] = std::asin(-m[8]);
  pose[2] = std::atan2(m[4], m[0]);
}


void fbr_keyframe_params_default(fbr_keyframe_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->search_radius = 50.0f;  // params.yaml:66-71
  p->pose_density = 2.0f;
  p->loop_closure = 0;
  p->submap_size = 25;
  p->recent_window = 10.0;   // mapOptmization.h:900
}

int fbr_keyframes_add(fbr_ctx* c, const fbr_keypose* pose, const fbr_point_xyzi* corner, int64_t n_corner,
                      const fbr_point_xyzi* surf, int64_t n_surf) {
  if (!c || !pose || n_corner < 0 || n_surf < 0 || (n_corner && !corner) || (n_surf && !surf)) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  int rc = grow(&c->d_kf_c, &c->kf_c_cap, c->kf_c_used + n_corner, c->kf_c_used, c->stream);
  if (!rc) rc = grow(&c->d_kf_s, &c->kf_s_cap, c->kf_s_used + n_surf, c->kf_s_used, c->stream);
  if (rc) return rc;
  if (n_corner)
    CK(hipMemcpyAsync(c->d_kf_c + c->kf_c_used, corner, sizeof(float4) * n_corner, hipMemcpyHostToDevice, c->stream));
  if (n_surf) CK(hipMemcpyAsync(c->d_kf_s + c->kf_s_used, surf, sizeof(float4) * n_surf, hipMemcpyHostToDevice, c->stream));
  CK(fbr_sync(c->stream));
  fbr_keypose p = *pose;
  p.intensity = (float)c->kf_poses.size();  // "this can be used as index" (:1687, :1694)
  c->kf_poses.push_back(p);
  c->kf_c_off.push_back(c->kf_c_used);
  c->kf_c_cnt.push_back(n_corner);
  c->kf_s_off.push_back(c->kf_s_used);
  c->kf_s_cnt.push_back(n_surf);
  c->kf_c_used += n_corner;
  c->kf_s_used += n_surf;
  return FBR_OK;
}

int fbr_keyframes_set_pose(fbr_ctx* c, int64_t index, const fbr_keypose* pose) {
  if (!c || !pose || index < 0 || index >= (int64_t)c->kf_poses.size()) return FBR_ERR_INVALID_ARG;
  fbr_keypose& k = c->kf_poses[index];  // correctPoses (:1746-1757): x, y, z, roll, pitch, yaw
  k.x = pose->x;
  k.y = pose->y;
  k.z = pose->z;
  k.roll = pose->roll;
  k.pitch = pose->pitch;
  k.yaw = pose->yaw;
  return FBR_OK;
}

int fbr_keyframes_count(fbr_ctx* c, int64_t* n) {
  if (!c || !n) return FBR_ERR_INVALID_ARG;
  *n = (int64_t)c->kf_poses.size();
  return FBR_OK;
}

int fbr_keyframes_reset(fbr_ctx* c) {
  if (!c) return FBR_ERR_INVALID_ARG;
  c->kf_poses.clear();
  c->kf_c_off.clear();
  c->kf_c_cnt.clear();
  c->kf_s_off.clear();
  c->kf_s_cnt.clear();
  c->kf_c_used = c->kf_s_used = 0;
  return FBR_OK;
}

int fbr_extract_surrounding_keyframes(fbr_ctx* c, double stamp, const fbr_keyframe_params* kp, int64_t* n_corner_map,
                                      int64_t* n_surf_map, int32_t* n_frames) {
  if (!c || !kp || !(kp->search_radius >= 0) || !(kp->pose_density > 0)) return FBR_ERR_INVALID_ARG;
  CK(enter(c));
  if (n_frames) *n_frames = 0;
  const int64_t N = (int64_t)c->kf_poses.size();
  if (N == 0) {  // extractSurroundingKeyFrames (:967-968): nothing to extract, map unchanged
    if (n_corner_map) *n_corner_map = c->map_nocrop ? c->kds_c_n : 0;
    if (n_surf_map) *n_surf_map = c->map_nocrop ? c->kds_s_n : 0;
    return FBR_OK;
  }
  const fbr_keypose& back = c->kf_poses.back();
  std::vector<fbr_keypose> toExtract;  // cloudToExtract (x, y, z, intensity = key index)
  if (kp->loop_closure) {  // extractForLoopClosure (:857-870)
    for (int64_t i = N - 1; i >= 0; --i) {
      if ((int)toExtract.size() <= kp->submap_size) toExtract.push_back(c->kf_poses[i]);
      else break;
    }
  } else {  // extractNearby (:872-907)
    // kdtreeSurroundingKeyPoses->radiusSearch(back, radius): d2 = ((dx dx + dy dy) + dz dz) < r^2,
    // sorted by distance (ties by index)
    const float r2 = (float)((double)kp->search_radius * (double)kp->search_radius);
    std::vector<std::pair<float, int64_t>> hits;
    for (int64_t i = 0; i < N; ++i) {
      const fbr_keypose& q = c->kf_poses[i];
      float d = 0.0f, diff;
      diff = back.x - q.x; d += diff * diff;
      diff = back.y - q.y; d += diff * diff;
      diff = back.z - q.z; d += diff * diff;
      if (d < r2) hits.emplace_back(d, i);
    }
    std::stable_sort(hits.begin(), hits.end(),
                     [](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) { return a.first < b.first; });
    std::vector<fbr_point_xyzi> sur(hits.size());
    for (size_t k = 0; k < hits.size(); ++k) {
      const fbr_keypose& q = c->kf_poses[hits[k].second];
      sur[k] = fbr_point_xyzi{q.x, q.y, q.z, q.intensity};
    }
    std::vector<fbr_point_xyzi> ds;  // downSizeFilterSurroundingKeyPoses (leaf surroundingKeyframeDensity)
    const int rc = voxel_grid_once(c, sur.data(), (int64_t)sur.size(), kp->pose_density, ds);
    if (rc) return rc;
    for (const fbr_point_xyzi& p : ds) {
      fbr_keypose k{};
      k.x = p.x;
      k.y = p.y;
      k.z = p.z;
      k.intensity = p.intensity;
      toExtract.push_back(k);
    }
    for (int64_t i = N - 1; i >= 0; --i) {  // the last recent_window seconds of keyframes (:896-904)
      if (stamp - c->kf_poses[i].time < kp->recent_window) toExtract.push_back(c->kf_poses[i]);
      else break;
    }
  }
  // extractCloud (:909-955): transform + concatenate the selected keyframes' clouds, then DS
  std::vector<KfSeg> segs;
  int64_t tot_c = 0, tot_s = 0, max_cnt = 0;
  for (int pass = 0; pass < 2; ++pass) {
    for (const fbr_keypose& e : toExtract) {
      if (key_distance(e, back) > kp->search_radius) continue;  // :924-925
      const int k = (int)e.intensity;                              // :927
      if (k < 0 || k >= N) return FBR_ERR_STATE;
      const fbr_keypose& pose = c->kf_poses[k];
      KfSeg g;
      const float tr[6] = {pose.roll, pose.pitch, pose.yaw, pose.x, pose.y, pose.z};
      float m[16];
      fbr_affine_from_pose(tr, m);  // pcl::getTransformation(x, y, z, roll, pitch, yaw), host libm
      for (int q = 0; q < 12; ++q) g.T[q] = m[q];
      if (pass == 0) {
        g.src = c->kf_c_off[k];
        g.count = c->kf_c_cnt[k];
        g.dst = tot_c;
        tot_c += g.count;
      } else {
        g.src = c->kf_s_off[k];
        g.count = c->kf_s_cnt[k];
        g.dst = tot_s;
        tot_s += g.count;
      }
      max_cnt = std::max(max_cnt, g.count);
      segs.push_back(g);
    }
  }
  const int nseg_c = (int)(segs.size() / 2);
  if (n_frames) *n_frames = (int32_t)toExtract.size();
  int rc = grow(&c->d_kraw_c, &c->kraw_c_cap, std::max<int64_t>(tot_c, 1), 0, c->stream);
  if (!rc) rc = grow(&c->d_kraw_s, &c->kraw_s_cap, std::max<int64_t>(tot_s, 1), 0, c->stream);
  if (!rc) rc = grow(&c->d_kf_segs, &c->kf_segs_cap, std::max<int64_t>((int64_t)segs.size(), 1), 0, c->stream);
  if (rc) return rc;
  if (!segs.empty())
    CK(hipMemcpyAsync(c->d_kf_segs, segs.data(), sizeof(KfSeg) * segs.size(), hipMemcpyHostToDevice, c->stream));
  launch_kf_transform(c->stream, c->d_kf_c, c->d_kf_segs, nseg_c, max_cnt, c->d_kraw_c);
  launch_kf_transform(c->stream, c->d_kf_s, c->d_kf_segs + nseg_c, (int)segs.size() - nseg_c, max_cnt, c->d_kraw_s);
  CK(hipGetLastError());
  if (c->d_kds_c) CK(hipFree(c->d_kds_c));
  if (c->d_kds_s) CK(hipFree(c->d_kds_s));
  c->d_kds_c = c->d_kds_s = nullptr;
  if (dalloc(&c->d_kds_c, std::max<int64_t>(tot_c, 1)) || dalloc(&c->d_kds_s, std::max<int64_t>(tot_s, 1))) {
    (void)fbr_sync(c->stream);  // the pageable copy of `segs` must finish before it goes out of scope
    return FBR_ERR_HIP;
  }
  // downSizeFilterCorner / downSizeFilterSurf (:946-954)
  rc = voxel_grid_dev(c, c->d_kraw_c, tot_c, c->P.mapping_corner_leaf_size, c->d_kds_c, &c->kds_c_n);
  if (!rc) rc = voxel_grid_dev(c, c->d_kraw_s, tot_s, c->P.mapping_surf_leaf_size, c->d_kds_s, &c->kds_s_n);
  // the kNN grids (both maps share one cell size, as in fbr_set_map)
  if (!rc) rc = build_map_grids(c, c->d_kds_c, c->kds_c_n, c->d_kds_s, c->kds_s_n);
  c->has_map = rc == FBR_OK;
  c->map_nocrop = rc == FBR_OK;
  c->crop_cached = false;
  c->map_c_host.clear();
  c->map_s_host.clear();
  if (rc) return rc;
  if (n_corner_map) *n_corner_map = c->kds_c_n;
  if (n_surf_map) *n_surf_map = c->kds_s_n;
  return FBR_OK;
}

}  // extern "C"

