// fbr_fdlibm.h — bit-exact single-precision atan2 for the range-image column index.
//
// The reference computes the column of every point as
//     horizonAngle = atan2(thisPoint.x, thisPoint.y) * 180 / M_PI;
// (/root/reference/src/imageProjection.cpp:605) with float arguments, i.e. it calls
// glibc's atan2f.  glibc 2.35's atan2f/atanf (sysdeps/ieee754/flt-32/e_atan2f.c,
// s_atanf.c) are the classic fdlibm single-precision algorithm; a 1-ulp difference in
// the angle moves ~6 column indices per million points, so the device path carries
// its own restatement of that algorithm instead of ocml's atan2f.  The restatement is
// checked bit-for-bit against the host glibc atan2f by tests/test_atan2f_port.py.
//
// Must be compiled with -ffp-contract=off (fused a*b+c would change the bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fbr {

__host__ __device__ inline int32_t f2bits(float x) { return __builtin_bit_cast(int32_t, x); }
__host__ __device__ inline float bits2f(int32_t i) { return __builtin_bit_cast(float, i); }

// fdlibm s_atanf.c argument reduction + odd/even polynomial split.
__host__ __device__ inline float fd_atanf(float x) {
  const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
              atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
  const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
              atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
  const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
              aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
              aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
              aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
  const float one = 1.0f;
  int32_t hx = f2bits(x);
  int32_t ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x4c000000) {          // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;  // NaN
    return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  if (ix < 0x3ee00000) {           // |x| < 0.4375
    if (ix < 0x31000000) return x; // |x| < 2^-29
    id = -1;
  } else {
    x = __builtin_fabsf(x);
    if (ix < 0x3f980000) {         // |x| < 1.1875
      if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }
      else                 { id = 1; x = (x - one) / (x + one); }
    } else {
      if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }
      else                 { id = 3; x = -1.0f / x; }
    }
  }
  float z = x * x;
  float w = z * z;
  float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  if (id < 0) return x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  return hx < 0 ? -z : z;
}

// fdlibm e_atan2f.c: atan2(y, x) in single precision.
__host__ __device__ inline float fd_atan2f(float y, float x) {
  const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
              pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
  int32_t hx = f2bits(x), hy = f2bits(y);
  int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
  if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
  if (hx == 0x3f800000) return fd_atanf(y);
  int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
  if (iy == 0) {
    switch (m) {
      case 0: case 1: return y;
      case 2: return pi + tiny;
      default: return -pi - tiny;
    }
  }
  if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  if (ix == 0x7f800000) {
    if (iy == 0x7f800000) {
      switch (m) {
        case 0: return pi_o_4 + tiny;
        case 1: return -pi_o_4 - tiny;
        case 2: return 3.0f * pi_o_4 + tiny;
        default: return -3.0f * pi_o_4 - tiny;
      }
    } else {
      switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
      }
    }
  }
  if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
  int32_t k = (iy - ix) >> 23;
  float z;
  if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
  else if (hx < 0 && k < -60) z = 0.0f;
  else z = fd_atanf(__builtin_fabsf(y / x));
  switch (m) {
    case 0: return z;
    case 1: return bits2f(f2bits(z) ^ (int32_t)0x80000000);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
  }
}

}  // namespace fbr
