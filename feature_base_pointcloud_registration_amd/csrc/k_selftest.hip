// k_selftest.hip — device numerics probe behind fbr_selftest_math (diagnostic entry point).
//
// The path's bit-exactness rests on a few device primitives matching the reference's host libm:
// correctly rounded f32 sqrt and division (SSE sqrtss / divss), glibc atan2f
// (imageProjection.cpp:605,618) and glibc sinf / cosf (pcl::getTransformation, LMOptimization
// mapOptmization.h:1259-1264).  tests/test_gpu_parity.py feeds random operands through this
// kernel and compares every output bit with the host.
#include <algorithm>

#include "fbr_common.h"
#include "fbr_fdlibm.h"
#include "fbr_sincosf.h"
#include "fbr_introsort.h"
#include "fbr_solvers.h"

namespace fbr {

constexpr int kSelftestMathOut = 6;

__global__ void k_selftest_math(int n, const float* a, const float* b, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i], y = b[i];
  float* o = out + (int64_t)kSelftestMathOut * i;
  o[0] = sqrt_rn(x < 0.0f ? -x : x);
  o[1] = x / y;
  o[2] = fd_atan2f(x, y);
  o[3] = x * y + y * x - x;  // plain mul/add with contraction disabled
  o[4] = gl_sinf(x);
  o[5] = gl_cosf(x);
}

// One 64-lane workgroup per symmetric 6x6 matrix: the single-lane jacobi_eigen<6> (lane 0) and the
// wave-parallel jacobi_eigen_wave<6>; out = 2 x (6 eigenvalues + 36 eigenvector entries).
__global__ void __launch_bounds__(64) k_selftest_eigen6(const float* a, float* out) {
  __shared__ float A[36], V[36], W[6];
  __shared__ int R[6], C[6];
  const int m = blockIdx.x, lane = threadIdx.x;
  float* o = out + (int64_t)m * 84;
  if (lane == 0) {
    float Ar[36], Wr[6], Vr[36];
    for (int k = 0; k < 36; ++k) Ar[k] = a[(int64_t)m * 36 + k];
    jacobi_eigen<6>(Ar, Wr, Vr);
    for (int k = 0; k < 6; ++k) o[k] = Wr[k];
    for (int k = 0; k < 36; ++k) o[6 + k] = Vr[k];
  }
  if (lane < 36) A[lane] = a[(int64_t)m * 36 + lane];
  __syncthreads();
  jacobi_eigen_wave<6>(A, W, V, R, C);
  if (lane < 6) o[42 + lane] = W[lane];
  if (lane < 36) o[48 + lane] = V[lane];
}

// out[i] = 1 when eig_above_certified<6> certifies every eigenvalue of matrix i above `thr`.
__global__ void k_selftest_eig_cert(int n, const float* a, float thr, int32_t* out) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < n) out[m] = eig_above_certified<6>(a + (int64_t)m * 36, thr) ? 1 : 0;
}

// std::sort's partition phase (fbr_introsort.h) on one array: lds = 0 keeps everything in global
// memory (the device-wide VoxelGrid's variant), lds = 1 the keys / values / positions in LDS
// (n <= kIsortLdsCap, the per-segment kernels' variant), lds = 2 keys / values in LDS and the
// positions in global memory (the mapping-DS kernel's variant).  v[] ends as the permuted indices.
constexpr int kIsortLdsCap = 8192;
__global__ void __launch_bounds__(1024) k_selftest_isort(uint32_t* k, uint32_t* v, int32_t* posL, int32_t* posR,
                                                         int* fa, int* fb, int n, int lds) {
  __shared__ int sh[64];
  if (!lds) {
    is_partition_phase<1024>(k, v, posL, posR, n, fa, fb, sh);
    return;
  }
  __shared__ uint32_t lk[kIsortLdsCap];
  __shared__ uint16_t lv[kIsortLdsCap], lpl[kIsortLdsCap], lpr[kIsortLdsCap];
  __shared__ int lfa[3 * (kIsortLdsCap / 17 + 2)], lfb[3 * (kIsortLdsCap / 17 + 2)];
  for (int i = threadIdx.x; i < n; i += 1024) {
    lk[i] = k[i];
    lv[i] = (uint16_t)i;
  }
  is_partition_phase<1024>((FBR_IS_LDS uint32_t*)lk, (FBR_IS_LDS uint16_t*)lv, (FBR_IS_LDS uint16_t*)lpl,
                           (FBR_IS_LDS uint16_t*)lpr, n, (FBR_IS_LDS int*)lfa, (FBR_IS_LDS int*)lfb, sh);
  for (int i = threadIdx.x; i < n; i += 1024) {
    k[i] = lk[i];
    v[i] = lv[i];
  }
}

// lds = 2: keys / values in LDS up to the mapping-DS kernel's 1024 * 18 points, positions in
// global memory (k_voxel_grid_ip's variant).
constexpr int kIsortLdsCap2 = 1024 * 18;
__global__ void __launch_bounds__(1024) k_selftest_isort2(uint32_t* k, uint32_t* v, int32_t* posL, int32_t* posR,
                                                          int n) {
  __shared__ int sh[64];
  __shared__ uint32_t lk[kIsortLdsCap2];
  __shared__ uint16_t lv[kIsortLdsCap2];
  __shared__ int lfa[3 * (kIsortLdsCap2 / 17 + 2)], lfb[3 * (kIsortLdsCap2 / 17 + 2)];
  for (int i = threadIdx.x; i < n; i += 1024) {
    lk[i] = k[i];
    lv[i] = (uint16_t)i;
  }
  is_partition_phase<1024>((FBR_IS_LDS uint32_t*)lk, (FBR_IS_LDS uint16_t*)lv, posL, posR, n, (FBR_IS_LDS int*)lfa,
                           (FBR_IS_LDS int*)lfb, sh);
  for (int i = threadIdx.x; i < n; i += 1024) {
    k[i] = lk[i];
    v[i] = lv[i];
  }
}

// lds = 3: the per-ring filter's shape -- 512 threads, everything in LDS (n <= 4096, u16
// positions) -- with the whole-workgroup partition from 128 elements up (the ring kernel uses 512)
// so that the block partition and its parallel K count see many frames.
constexpr int kIsortLdsCap3 = 4096;
__global__ void __launch_bounds__(512) k_selftest_isort3(uint32_t* k, uint32_t* v, int n) {
  __shared__ int sh[64];
  __shared__ uint32_t lk[kIsortLdsCap3];
  __shared__ uint16_t lv[kIsortLdsCap3], lpl[kIsortLdsCap3], lpr[kIsortLdsCap3];
  __shared__ int lfa[3 * (kIsortLdsCap3 / 17 + 2)], lfb[3 * (kIsortLdsCap3 / 17 + 2)];
  for (int i = threadIdx.x; i < n; i += 512) {
    lk[i] = k[i];
    lv[i] = (uint16_t)i;
  }
  is_partition_phase<512, FBR_IS_LDS uint32_t*, FBR_IS_LDS uint16_t*, FBR_IS_LDS uint16_t*, FBR_IS_LDS int*, 128>(
      (FBR_IS_LDS uint32_t*)lk, (FBR_IS_LDS uint16_t*)lv, (FBR_IS_LDS uint16_t*)lpl, (FBR_IS_LDS uint16_t*)lpr, n,
      (FBR_IS_LDS int*)lfa, (FBR_IS_LDS int*)lfb, sh);
  for (int i = threadIdx.x; i < n; i += 512) {
    k[i] = lk[i];
    v[i] = lv[i];
  }
}

}  // namespace fbr

extern "C" int fbr_selftest_voxel_order(int64_t n, const uint32_t* keys, int lds, uint32_t* perm) {
  if (n < 0 || n > (int64_t)INT32_MAX / 4 || (n && (!keys || !perm)) || (lds == 1 && n > fbr::kIsortLdsCap) ||
      (lds == 2 && n > fbr::kIsortLdsCap2) || (lds == 3 && n > fbr::kIsortLdsCap3) || lds < 0 || lds > 3)
    return FBR_ERR_INVALID_ARG;
  if (n == 0) return FBR_OK;
  std::vector<uint32_t> iv(n);
  for (int64_t i = 0; i < n; ++i) iv[i] = (uint32_t)i;
  uint32_t *dk = nullptr, *dv = nullptr;
  int32_t *pl = nullptr, *pr = nullptr;
  int *fa = nullptr, *fb = nullptr;
  const int64_t nf = n / 17 + 2;
  int rc = FBR_OK;
  if (hipMalloc(&dk, 4 * n) != hipSuccess || hipMalloc(&dv, 4 * n) != hipSuccess || hipMalloc(&pl, 4 * n) != hipSuccess ||
      hipMalloc(&pr, 4 * n) != hipSuccess || hipMalloc(&fa, 3 * sizeof(int) * nf) != hipSuccess ||
      hipMalloc(&fb, 3 * sizeof(int) * nf) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else if (hipMemcpy(dk, keys, 4 * n, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(dv, iv.data(), 4 * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    if (lds == 3) hipLaunchKernelGGL(fbr::k_selftest_isort3, dim3(1), dim3(512), 0, 0, dk, dv, (int)n);
    else if (lds == 2) hipLaunchKernelGGL(fbr::k_selftest_isort2, dim3(1), dim3(1024), 0, 0, dk, dv, pl, pr, (int)n);
    else hipLaunchKernelGGL(fbr::k_selftest_isort, dim3(1), dim3(1024), 0, 0, dk, dv, pl, pr, fa, fb, (int)n, lds);
    if (hipMemcpy(perm, dv, 4 * n, hipMemcpyDeviceToHost) != hipSuccess) rc = FBR_ERR_HIP;
  }
  for (void* q : {(void*)dk, (void*)dv, (void*)pl, (void*)pr, (void*)fa, (void*)fb}) (void)hipFree(q);
  return rc;
}

extern "C" int fbr_selftest_eig_certified(int n, const float* a, float thr, int32_t* out) {
  if (n <= 0 || !a || !out) return FBR_ERR_INVALID_ARG;
  float* da = nullptr;
  int32_t* dout = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&da, sizeof(float) * 36 * n) != hipSuccess || hipMalloc(&dout, sizeof(int32_t) * n) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else if (hipMemcpy(da, a, sizeof(float) * 36 * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    hipLaunchKernelGGL(fbr::k_selftest_eig_cert, dim3((n + 63) / 64), dim3(64), 0, 0, n, da, thr, dout);
    if (hipMemcpy(out, dout, sizeof(int32_t) * n, hipMemcpyDeviceToHost) != hipSuccess) rc = FBR_ERR_HIP;
  }
  (void)hipFree(da);
  (void)hipFree(dout);
  return rc;
}

extern "C" int fbr_selftest_math(int n, const float* a, const float* b, float* out) {
  if (n <= 0 || !a || !b || !out) return FBR_ERR_INVALID_ARG;
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&da, sizeof(float) * n) != hipSuccess || hipMalloc(&db, sizeof(float) * n) != hipSuccess ||
      hipMalloc(&dout, sizeof(float) * fbr::kSelftestMathOut * n) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else if (hipMemcpy(da, a, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(db, b, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    hipLaunchKernelGGL(fbr::k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, 0, n, da, db, dout);
    if (hipMemcpy(out, dout, sizeof(float) * fbr::kSelftestMathOut * n, hipMemcpyDeviceToHost) != hipSuccess) rc = FBR_ERR_HIP;
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}

extern "C" int fbr_selftest_eigen6(int n, const float* a, float* out) {
  if (n <= 0 || !a || !out) return FBR_ERR_INVALID_ARG;
  float *da = nullptr, *dout = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&da, sizeof(float) * 36 * n) != hipSuccess || hipMalloc(&dout, sizeof(float) * 84 * n) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else if (hipMemcpy(da, a, sizeof(float) * 36 * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    hipLaunchKernelGGL(fbr::k_selftest_eigen6, dim3(n), dim3(64), 0, 0, da, dout);
    if (hipMemcpy(out, dout, sizeof(float) * 84 * n, hipMemcpyDeviceToHost) != hipSuccess) rc = FBR_ERR_HIP;
  }
  (void)hipFree(da);
  (void)hipFree(dout);
  return rc;
}

// STREAM-copy probe (measurement helper, BASELINE.md "report vs measured STREAM-copy bandwidth"):
// float4 copies of `bytes` per direction, timed with HIP events over `iters` launches.  Three
// shapes are timed and the best is reported: a grid-stride loop, one float4 per thread with one
// workgroup per 4 KiB, and U float4 per thread (all loads issued before the stores, non-temporal
// stores) with one workgroup per U * 4 KiB.
namespace fbr {
__global__ void __launch_bounds__(256) k_stream_copy(const float4* __restrict__ a, float4* __restrict__ b, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) b[i] = a[i];
}
template <int U>
__global__ void __launch_bounds__(256) k_stream_copy_u(const float4* __restrict__ a, float4* __restrict__ b, int64_t n) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  float4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * 256;
    v[u] = i < n ? a[i] : make_float4(0, 0, 0, 0);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + (int64_t)u * 256;
    if (i < n) {
      __builtin_nontemporal_store(v[u].x, &b[i].x);
      __builtin_nontemporal_store(v[u].y, &b[i].y);
      __builtin_nontemporal_store(v[u].z, &b[i].z);
      __builtin_nontemporal_store(v[u].w, &b[i].w);
    }
  }
}
}  // namespace fbr

extern "C" int fbr_stream_copy_bandwidth(int hip_device, int64_t bytes, int iters, double* gbps) {
  if (bytes < 16 || iters <= 0 || !gbps) return FBR_ERR_INVALID_ARG;
  if (hipSetDevice(hip_device) != hipSuccess) return FBR_ERR_NO_DEVICE;
  const int64_t n = bytes / 16;
  float4 *a = nullptr, *b = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&a, sizeof(float4) * n) != hipSuccess || hipMalloc(&b, sizeof(float4) * n) != hipSuccess ||
      hipMemset(a, 0, sizeof(float4) * n) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    *gbps = 0.0;
    for (int variant = 0; variant < 3 && !rc; ++variant) {
      auto launch = [&]() {
        if (variant == 0)  // grid stride: 8 XCDs x 32 CUs, several workgroups per CU
          hipLaunchKernelGGL(fbr::k_stream_copy, dim3(256 * 8 * 4), dim3(256), 0, 0, a, b, n);
        else if (variant == 1)
          hipLaunchKernelGGL(fbr::k_stream_copy_u<1>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, b, n);
        else
          hipLaunchKernelGGL(fbr::k_stream_copy_u<4>, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, 0, a, b, n);
      };
      launch();  // warm-up
      (void)hipEventRecord(e0, 0);
      for (int k = 0; k < iters; ++k) launch();
      (void)hipEventRecord(e1, 0);
      float ms = 0.0f;
      if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.0f)
        rc = FBR_ERR_HIP;
      else
        *gbps = std::max(*gbps, 2.0 * 16.0 * (double)n * iters / (ms * 1e-3) / 1e9);  // read + write
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(a);
  (void)hipFree(b);
  return rc;
}

// VALU issue-rate probe (measurement helper for the VALU roofline, bench.py / tools/valu_calib.py):
// every lane runs 8 independent dependency chains of one VALU instruction for `iters` rounds, written
// as inline asm so the compiler can neither pack (SLP) nor drop them.  kind 0: v_fma_f32, 1:
// v_add_u32, 2: v_pk_fma_f32 (2 lanes of f32 per slot), 3: v_cmp_lt_u64, 4: v_cmp_lt_u32 (both
// into SGPR pairs: the compares of the kNN list insertion).  The grid is n_cu * waves_per_simd
// workgroups of 256 threads (4 waves: one per SIMD), so every SIMD holds waves_per_simd waves.
namespace fbr {
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int KIND>
__global__ void __launch_bounds__(256) k_valu_peak(float* out, int iters, float a, float b) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if constexpr (KIND == 0) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = (float)(t + u);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x[u]) : "v"(a), "v"(b));
    }
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
    out[t] = s;
  } else if constexpr (KIND == 1) {
    uint32_t x[8];
    const uint32_t ia = __float_as_uint(a);
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = (uint32_t)(t + u);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[u]) : "v"(ia));
    }
    uint32_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
    out[t] = (float)s;
  } else if constexpr (KIND == 3 || KIND == 4) {  // 64-bit / 32-bit unsigned compares into SGPR pairs
    uint64_t x[8], m[8];
    const uint64_t y = (uint64_t)__float_as_uint(a) << 20;
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = (uint64_t)(t + u) << 16;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if constexpr (KIND == 3) asm volatile("v_cmp_lt_u64_e64 %0, %1, %2" : "=s"(m[u]) : "v"(x[u]), "v"(y));
          else asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(m[u]) : "v"((uint32_t)x[u]), "v"((uint32_t)y));
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) s ^= m[u];
    out[t] = (float)(s & 0xffff);
  } else {
    f32x2 x[8];
    f32x2 va = {a, a}, vb = {b, b};
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = f32x2{(float)(t + u), (float)(t - u)};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x[u]) : "v"(va), "v"(vb));
    }
    float s = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u].x + x[u].y;
    out[t] = s;
  }
}
}  // namespace fbr

// Wave-level VALU instructions per second of the probe above (32 per lane per round, timed with HIP
// events over `reps` launches after one warm-up launch).
extern "C" int fbr_valu_peak(int hip_device, int waves_per_simd, int kind, int iters, int reps, double* ginst_per_s,
                             double* ms_per_launch) {
  if (waves_per_simd < 1 || waves_per_simd > 8 || kind < 0 || kind > 4 || iters <= 0 || reps <= 0 || !ginst_per_s)
    return FBR_ERR_INVALID_ARG;
  if (hipSetDevice(hip_device) != hipSuccess) return FBR_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) return FBR_ERR_HIP;
  const int blocks = prop.multiProcessorCount * waves_per_simd;
  float* out = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&out, sizeof(float) * 256 * blocks) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
      hipEventCreate(&e1) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    auto launch = [&]() {
      if (kind == 0) hipLaunchKernelGGL(fbr::k_valu_peak<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001f, 0.5f);
      else if (kind == 1) hipLaunchKernelGGL(fbr::k_valu_peak<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001f, 0.5f);
      else if (kind == 2) hipLaunchKernelGGL(fbr::k_valu_peak<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001f, 0.5f);
      else if (kind == 3) hipLaunchKernelGGL(fbr::k_valu_peak<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001f, 0.5f);
      else hipLaunchKernelGGL(fbr::k_valu_peak<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0000001f, 0.5f);
    };
    launch();
    (void)hipEventRecord(e0, 0);
    for (int k = 0; k < reps; ++k) launch();
    (void)hipEventRecord(e1, 0);
    float ms = 0.0f;
    if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&ms, e0, e1) != hipSuccess || ms <= 0.0f) {
      rc = FBR_ERR_HIP;
    } else {
      const double waves = 4.0 * blocks;
      *ginst_per_s = waves * 32.0 * iters * reps / (ms * 1e-3) / 1e9;
      if (ms_per_launch) *ms_per_launch = ms / reps;
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(out);
  return rc;
}
