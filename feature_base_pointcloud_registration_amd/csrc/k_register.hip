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
#include "fbr_gn.h"
#include "fbr_imu.h"

namespace fbr {



__global__ void k_gn_init(GnArgs a) {
  __shared__ int32_t scan[1024];
  const int tid = threadIdx.x;
  for (int i = tid; i < 4 * max(1, a.max_iter); i += 1024) a.iter_cnt[i] = 0;  // k_gn_solve's + block-tile counters
  if (a.direct_done && tid == 0) *a.direct_done = 0;
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
    // exclusive prefix of the jobs' item counts: wave scans, then the 16 wave totals (two barriers
    // per 1024 jobs; the Hillis-Steele form took 20, ~5 us of a single scan's critical path)
    const int v = nc_items + ns_items, lane = tid & 63, w = tid >> 6;
    int inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(inc, off);
      if (lane >= off) inc += y;
    }
    if (lane == 63) scan[w] = inc;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int k = 0; k < 16; ++k) {
      pre += k < w ? scan[k] : 0;
      tot += scan[k];
    }
    const int excl = base + pre + inc - v;
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
    base += tot;
    __syncthreads();  // every wave read scan[] before the next chunk's totals overwrite it
  }
  if (tid == 0) a.nitems[0] = min(base, a.max_items);
}

// As k_gn_knn / k_gn_loop_knn: one item per workgroup from base, or a grid-stride loop from base.
__global__ void __launch_bounds__(kResThreads)
k_gn_residual(GnArgs a, int base) {
  __shared__ double red[kResThreads / 64][28];
  const int it = base + (int)blockIdx.x;
  if (it < a.nitems[0]) gn_residual_item(a, it, red);
}
__global__ void __launch_bounds__(kResThreads)
k_gn_loop_residual(GnArgs a, int base) {
  __shared__ double red[kResThreads / 64][28];
  const int nitems = a.nitems[0];
  for (int it = base + blockIdx.x; it < nitems; it += gridDim.x) gn_residual_item(a, it, red);
}


// transformUpdate of one job (:1444-1479) into pose_out / stats.
__device__ void gn_finalize_job(const GnArgs& a, int job) {
  const GnState& g = a.gn[job];
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

// One job's packed result (k_pack_results; the solve's direct path with pad = the run's generation).
__device__ JobResult pack_job(int j, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                              const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf,
                              const int32_t* cropcnt, const int32_t* err, const float* guess, int32_t pad) {
  JobResult r;
  if (with_reg && guess && err[j]) {  // batch job over the feature capacity: the guess, flagged
    for (int k = 0; k < 6; ++k) r.pose[k] = guess[6 * j + k];
    r.st = fbr_reg_stats{};
    r.st.status = FBR_REG_FEATURE_CAPACITY;
    r.st.n_corner_map = cropcnt[2 * j];
    r.st.n_surf_map = cropcnt[2 * j + 1];
  } else if (with_reg) {
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
  r.pad = pad;
  return r;
}

// Two waves per job: wave 0's lanes 0..27 sum the job's item partials (each entry in item order,
// as before); then wave 0's lane 0 solves the normal equations while, at iteration 0, wave 1's
// lane 0 computes the degeneracy projection (the two are independent; on one wave they would run
// back to back); lane 0 then runs the rest of the LMOptimization step.  The number of jobs still
// iterating is accumulated with agent-scope atomics; the last workgroup to finish publishes it to
// host-mapped memory as (generation << 32 | count) so the host stops enqueueing iterations once
// the batch converged.
__global__ void __launch_bounds__(kSolveThreads) k_gn_solve(GnArgs a, int iter_idx, unsigned long long gen) {
  __shared__ SolveLds sl;
  const int job = blockIdx.x, tid = threadIdx.x;
  gn_solve_block(a, job, sl);
  const GnState& g = a.gn[job];
  if (tid == 0) {
    atomicAdd(&a.iter_cnt[2 * iter_idx], g.active);
    __threadfence();
    const int done = atomicAdd(&a.iter_cnt[2 * iter_idx + 1], 1);
    if (done == a.B - 1) {
      __threadfence();
      const int cnt = atomicAdd(&a.iter_cnt[2 * iter_idx], 0);
      // the run ends here (the host enqueues nothing after a zero count, and no iteration after the
      // last): transformUpdate and the packed results straight into host memory, once per run
      // (the host enables it for one-job runs, where this thread's own solve wrote the job's state)
      if (a.direct && (cnt == 0 || iter_idx == a.max_iter - 1) && atomicExch(a.direct_done, 1) == 0) {
        constexpr int NW = (int)(sizeof(JobResult) / 4);  // the last word is pad: the generation
        for (int j = 0; j < a.B; ++j) {
          gn_finalize_job(a, j);
          const JobResult r = pack_job(j, 1, a.pose_out, a.stats, a.nvalid, a.ncorner, a.nsurf, a.cropcnt, a.ferr,
                                       nullptr, a.direct_gen);
          const uint32_t* w = reinterpret_cast<const uint32_t*>(&r);
          uint32_t* d = reinterpret_cast<uint32_t*>(a.direct + j);
          for (int q = 0; q < NW - 1; ++q) __hip_atomic_store(d + q, w[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          __threadfence_system();  // the record before its generation word
          __hip_atomic_store(d + NW - 1, w[NW - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __threadfence_system();
      }
      if (a.items_flag && iter_idx == 0)  // the run's item count, for the host's launch grids
        __hip_atomic_store(a.items_flag, (gen << 32) | (unsigned long long)(uint32_t)a.nitems[0], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      if (a.iter_flags)
        __hip_atomic_store(&a.iter_flags[iter_idx], (gen << 32) | (unsigned long long)cnt, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void k_gn_finalize(GnArgs a) {
  const int job = blockIdx.x * blockDim.x + threadIdx.x;
  if (job < a.B) gn_finalize_job(a, job);
}

// CropBox counts of the global map for every job's box (laserCloud{Corner,Surf}FromMapDSNum,
// statistics only: the registration applies the box per kNN candidate).  The box is the guess's
// translation +- crop_half (registration :289-304), identical to the one k_gn_init stores.
// One wave per (tile of 512 map points, 64 jobs): the tile is staged in LDS and every lane tests
// all of it against its job's box (LDS broadcast reads), then adds its count once.  The counts of a
// launch accumulate in a per-work-slot buffer (zeroed first) and are then copied to the inputs'
// statistics slots, so a launch recomputing them never exposes a partial count to an earlier
// launch of the same staged batch that reads them.  Integer counts: exact in any order.
constexpr int kCropTile = 512;
__global__ void __launch_bounds__(64) k_crop_count(GnArgs a, const float4* __restrict__ pc, int64_t nc,
                                                   const float4* __restrict__ ps, int64_t ns, int64_t tiles_c,
                                                   int32_t* counts) {
  __shared__ float4 tile[kCropTile];
  const int lane = threadIdx.x;
  const int64_t t = blockIdx.x;
  const int which = t < tiles_c ? 0 : 1;
  const float4* pts = which ? ps : pc;
  const int64_t n = which ? ns : nc;
  const int64_t i0 = (which ? t - tiles_c : t) * kCropTile;
  const int m = (int)min<int64_t>(kCropTile, n - i0);
  for (int i = lane; i < m; i += 64) tile[i] = pts[i0 + i];
  __syncthreads();
  const int j = blockIdx.y * 64 + lane;
  if (j >= a.B) return;
  const float* gp = a.guess + 6 * j;  // registration :289-292 (k_gn_init's box)
  const float mn0 = -a.crop_half[0] + gp[3], mn1 = -a.crop_half[1] + gp[4], mn2 = -a.crop_half[2] + gp[5];
  const float mx0 = a.crop_half[0] + gp[3], mx1 = a.crop_half[1] + gp[4], mx2 = a.crop_half[2] + gp[5];
  int cnt = 0;
  for (int i = 0; i < m; ++i) {
    const float4 p = tile[i];
    cnt += (int)(!(p.x < mn0 || p.y < mn1 || p.z < mn2) && !(p.x > mx0 || p.y > mx1 || p.z > mx2));
  }
  if (cnt) atomicAdd(&counts[2 * j + which], cnt);
}

// 32-byte pose record per job {pose[6], iterations, status} for the cross-GPU gather.  A job over the
// feature capacity gets the same record fbr_batch_results reports for it (k_pack_results): its guess,
// 0 iterations, FBR_REG_FEATURE_CAPACITY.
__global__ void k_export_records(int B, const float* pose_out, const fbr_reg_stats* stats, const int32_t* err,
                                 const float* guess, float* dst) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B) return;
  const bool cap = err[j] != 0;
  for (int k = 0; k < 6; ++k) dst[8 * j + k] = cap ? guess[6 * j + k] : pose_out[6 * j + k];
  dst[8 * j + 6] = __int_as_float(cap ? 0 : stats[j].iterations);
  dst[8 * j + 7] = __int_as_float(cap ? FBR_REG_FEATURE_CAPACITY : stats[j].status);
}

__global__ void k_pack_results(int B, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                               const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf,
                               const int32_t* cropcnt, const int32_t* err, const float* guess, JobResult* out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < B) out[j] = pack_job(j, with_reg, pose_out, stats, nvalid, ncorner, nsurf, cropcnt, err, guess, 0);
}

void launch_pack_results(hipStream_t s, int B, int with_reg, const float* pose_out, const fbr_reg_stats* stats,
                         const int32_t* nvalid, const int32_t* ncorner, const int32_t* nsurf, const int32_t* cropcnt,
                         const int32_t* err, const float* guess, JobResult* out) {
  fbr_launch(k_pack_results, dim3((B + 63) / 64), dim3(64), 0, s, B, with_reg, pose_out, stats, nvalid, ncorner, nsurf,
             cropcnt, err, guess, out);
}

void launch_export_records(hipStream_t s, int B, const float* pose_out, const fbr_reg_stats* stats, const int32_t* err,
                           const float* guess, float* dst) {
  fbr_launch(k_export_records, dim3((B + 63) / 64), dim3(64), 0, s, B, pose_out, stats, err, guess, dst);
}

void launch_gn_init(hipStream_t s, const GnArgs& a) { fbr_launch(k_gn_init, dim3(1), dim3(1024), 0, s, a); }
// kNN launchers per y/z cell size (instantiated in k_knn_r{1,2,4}{,f}.hip)
extern template void launch_gn_knn_r<1, false>(hipStream_t, const GnArgs&, int, int);
extern template void launch_gn_knn_r<2, false>(hipStream_t, const GnArgs&, int, int);
extern template void launch_gn_knn_r<4, false>(hipStream_t, const GnArgs&, int, int);
extern template void launch_gn_knn_r<1, true>(hipStream_t, const GnArgs&, int, int);
extern template void launch_gn_knn_r<2, true>(hipStream_t, const GnArgs&, int, int);
extern template void launch_gn_knn_r<4, true>(hipStream_t, const GnArgs&, int, int);

template <bool F>
void launch_gn_knn_f(hipStream_t s, const GnArgs& a, int grid, int use_prev) {
  const float inv = a.mc.g.inv_cell;  // == a.ms.g.inv_cell (fbr_set_map): y / z cells
  if (inv > 2.0f) launch_gn_knn_r<4, F>(s, a, grid, use_prev);  // 0.25 m
  else if (inv > 1.0f) launch_gn_knn_r<2, F>(s, a, grid, use_prev);  // 0.5 m
  else launch_gn_knn_r<1, F>(s, a, grid, use_prev);                  // >= 1 m
}

void launch_gn_knn(hipStream_t s, const GnArgs& a, int grid, int iter, bool fused) {
  const int use_prev = iter > 0;  // nbr holds this launch's previous iteration
  // no loop launch after this one (or the LDS-tile path, which covers every item itself)
  if (a.one_part == 2 && (a.one_item != 1 || (!fused && gn_knn_tile_applies(a, iter)))) return;
  if (!fused && launch_gn_knn_tile(s, a, grid, iter)) return;  // dense maps: LDS tiles (k_knn_tile.hip)
  if (fused) launch_gn_knn_f<true>(s, a, grid, use_prev);
  else launch_gn_knn_f<false>(s, a, grid, use_prev);
}
void launch_gn_residual(hipStream_t s, const GnArgs& a, int grid) {
  launch_one_item(s, a, grid, a.max_items, 0, k_gn_residual, k_gn_loop_residual, a);
}
void launch_gn_solve(hipStream_t s, const GnArgs& a, int iter_idx, unsigned long long gen) {
  fbr_launch(k_gn_solve, dim3(a.B), dim3(kSolveThreads), 0, s, a, iter_idx, gen);
}
void launch_gn_finalize(hipStream_t s, const GnArgs& a) {
  fbr_launch(k_gn_finalize, dim3((a.B + 63) / 64), dim3(64), 0, s, a);
}
void launch_crop_count(hipStream_t s, const GnArgs& a, const float4* pc, int64_t nc, const float4* ps, int64_t ns,
                       int32_t* work, int32_t* counts) {
  if (a.B <= 0) return;
  (void)hipMemsetAsync(work, 0, sizeof(int32_t) * 2 * a.B, s);
  const int64_t tc = (nc + kCropTile - 1) / kCropTile, ts = (ns + kCropTile - 1) / kCropTile;
  if (tc + ts > 0)
    fbr_launch(k_crop_count, dim3((unsigned)(tc + ts), (unsigned)((a.B + 63) / 64)), dim3(64), 0, s, a, pc, nc, ps, ns, tc,
               work);
  (void)hipMemcpyAsync(counts, work, sizeof(int32_t) * 2 * a.B, hipMemcpyDeviceToDevice, s);
}
}  // namespace fbr

#ifdef FBR_KNN_STATS
// Diagnostic builds only: read (and optionally reset) the kNN counters of k_gn_knn
// (GnArgs::knn_stats, allocated on first use).
namespace fbr {
unsigned long long* knn_stats_buffer() {
  static unsigned long long* p = [] {
    unsigned long long* q = nullptr;
    if (hipMalloc(&q, sizeof(unsigned long long) * 48) != hipSuccess) return (unsigned long long*)nullptr;
    hipMemset(q, 0, sizeof(unsigned long long) * 48);
    return q;
  }();
  return p;
}
}  // namespace fbr
extern "C" int fbr_diag_knn_stats(unsigned long long* out, int reset) {
  unsigned long long* p = fbr::knn_stats_buffer();
  if (!p) return FBR_ERR_HIP;
  if (out && hipMemcpy(out, p, sizeof(unsigned long long) * 48, hipMemcpyDeviceToHost) != hipSuccess) return FBR_ERR_HIP;
  if (reset && hipMemset(p, 0, sizeof(unsigned long long) * 48) != hipSuccess) return FBR_ERR_HIP;
  return FBR_OK;
}
#endif
