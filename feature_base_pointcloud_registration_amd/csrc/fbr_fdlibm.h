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

// fdlibm s_atanf.c argument reduction + odd/even polynomial split.  The four reduction branches
// (id 0..3) and the small-argument one (id -1) are computed as selects feeding ONE division
// (num / den: each branch's own operands, so the same IEEE operation; x / 1 = x exactly for id -1):
// across a wave the lanes fall into all five ranges, and the branchy form ran up to four division
// sequences per wave.
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
  if (ix >= 0x4c000000) {          // |x| >= 2^25
    if (ix > 0x7f800000) return x + x;  // NaN
    return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
  }
  const float ax = __builtin_fabsf(x);
  // id: -1 |x| < 0.4375; 0 < 0.6875; 1 < 1.1875; 2 < 2.4375; 3 above
  const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
  const float n0 = 2.0f * ax - one, d0 = 2.0f + ax;     // id 0: (2x - 1) / (2 + x)
  const float n1 = ax - one, d1 = ax + one;             // id 1: (x - 1) / (x + 1)
  const float n2 = ax - 1.5f, d2 = one + 1.5f * ax;     // id 2: (x - 1.5) / (1 + 1.5x)
  const float num = id < 0 ? x : id == 0 ? n0 : id == 1 ? n1 : id == 2 ? n2 : -1.0f;  // id 3: -1 / x
  const float den = id < 0 ? one : id == 0 ? d0 : id == 1 ? d1 : id == 2 ? d2 : ax;
  x = num / den;
  float z = x * x;
  float w = z * z;
  float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
  float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
  const float small = x - x * (s1 + s2);
  float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
  float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
  z = hi - ((x * (s1 + s2) - lo) - x);
  const float big = hx < 0 ? -z : z;
  return ix < 0x31000000 ? bits2f(hx) : (id < 0 ? small : big);  // |x| < 2^-29: x itself
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
