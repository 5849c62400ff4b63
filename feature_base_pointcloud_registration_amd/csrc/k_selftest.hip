// k_selftest.hip — device numerics probe behind fbr_selftest_math (diagnostic entry point).
//
// The path's bit-exactness rests on a few device primitives matching the reference's host libm:
// correctly rounded f32 sqrt and division (SSE sqrtss / divss) and glibc atan2f
// (imageProjection.cpp:605,618).  tests/test_gpu_parity.py feeds random operands through this
// kernel and compares every output bit with the host.
#include "fbr_common.h"
#include "fbr_fdlibm.h"

namespace fbr {

__global__ void k_selftest_math(int n, const float* a, const float* b, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i], y = b[i];
  out[4 * i + 0] = sqrt_rn(x < 0.0f ? -x : x);
  out[4 * i + 1] = x / y;
  out[4 * i + 2] = fd_atan2f(x, y);
  out[4 * i + 3] = x * y + y * x - x;  // plain mul/add with contraction disabled
}

}  // namespace fbr

extern "C" int fbr_selftest_math(int n, const float* a, const float* b, float* out) {
  if (n <= 0 || !a || !b || !out) return FBR_ERR_INVALID_ARG;
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  int rc = FBR_OK;
  if (hipMalloc(&da, sizeof(float) * n) != hipSuccess || hipMalloc(&db, sizeof(float) * n) != hipSuccess ||
      hipMalloc(&dout, sizeof(float) * 4 * n) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else if (hipMemcpy(da, a, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess ||
             hipMemcpy(db, b, sizeof(float) * n, hipMemcpyHostToDevice) != hipSuccess) {
    rc = FBR_ERR_HIP;
  } else {
    hipLaunchKernelGGL(fbr::k_selftest_math, dim3((n + 255) / 256), dim3(256), 0, 0, n, da, db, dout);
    if (hipMemcpy(out, dout, sizeof(float) * 4 * n, hipMemcpyDeviceToHost) != hipSuccess) rc = FBR_ERR_HIP;
  }
  (void)hipFree(da);
  (void)hipFree(db);
  (void)hipFree(dout);
  return rc;
}
