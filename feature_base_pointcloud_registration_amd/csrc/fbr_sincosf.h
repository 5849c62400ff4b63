// fbr_sincosf.h — bit-exact single-precision sin / cos for the pose transforms.
//
// The reference builds every rotation from float Euler angles with glibc's sinf / cosf:
//   pcl::getTransformation (pcl/common/impl/eigen.hpp, called by trans2Affine3f,
//     /root/reference/src/mapOptmization.h:444-448, and deskewPoint, imageProjection.cpp:574)
//   LMOptimization's srx/crx/sry/cry/srz/crz (mapOptmization.h:1259-1264).
// glibc 2.35's sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c, s_cosf.c, sincosf.h,
// s_sincosf_data.c) evaluate a double-precision polynomial after a double range reduction and
// round once to float.  On x86-64 the symbols are IFUNCs; every CPU with FMA + AVX2 (the GPU
// box's EPYC and this container's Xeon) runs the `-mfma -mavx2` build of the same C source
// (sysdeps/x86_64/fpu/multiarch/s_sinf-fma.c), in which GCC contracts each `a + b * c` into one
// fused multiply-add.  This header restates that variant with explicit fma() calls so the device
// reproduces the host bits; tests/test_oracle_pinning.py checks it against the host glibc
// exhaustively over the float range the pose angles take, and on random samples of the rest.
//
// Must be compiled with -ffp-contract=off (only the fma() calls below may fuse).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define FBR_SC_HD __host__ __device__
#else
#define FBR_SC_HD
#endif

namespace fbr {
namespace glibc_sincosf {

// __sincosf_table (s_sincosf_data.c): sign[4], hpi_inv (2/pi * 2^24: x86-64 has no
// TOINT_INTRINSICS), hpi, cosine c0..c4, sine s1..s3; entry 1 negates the cosine polynomial.
struct Table {
  double sign[4];
  double hpi_inv, hpi;
  double c0, c1, c2, c3, c4;
  double s1, s2, s3;
};

constexpr Table kTable[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, 0x1p0, -0x1.ffffffd0c621cp-2,
     0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45F306DC9C883p+23, 0x1.921FB54442D18p0, -0x1p0, 0x1.ffffffd0c621cp-2,
     -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16, -0x1.555545995a603p-3,
     0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
FBR_SC_HD inline const Table& table(int k) { return kTable[k]; }

// __inv_pio4: 4/pi in 192 bits, read at a 32-bit window chosen by the exponent.
constexpr uint32_t kInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};
FBR_SC_HD inline uint32_t inv_pio4(int i) { return kInvPio4[i]; }

FBR_SC_HD inline uint32_t asuint(float x) { return __builtin_bit_cast(uint32_t, x); }
FBR_SC_HD inline uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

// sinf_poly (sincosf.h): n even -> sine polynomial of x, odd -> cosine polynomial.
FBR_SC_HD inline float poly(double x, double x2, const Table& p, int n) {
  if ((n & 1) == 0) {
    const double x3 = x * x2;
    const double s1 = fma(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = fma(x3, p.s1, x);
    return (float)fma(x7, s1, s);
  }
  const double x4 = x2 * x2;
  const double c2 = fma(x2, p.c4, p.c3);
  const double c1 = fma(x2, p.c1, p.c0);
  const double x6 = x4 * x2;
  const double c = fma(x4, p.c2, c1);
  return (float)fma(x6, c2, c);
}

// reduce_fast: |x| < 120, quadrant in bits 24..31 of the scaled product.
FBR_SC_HD inline double reduce_fast(double x, const Table& p, int* np) {
  const double r = x * p.hpi_inv;
  const int n = ((int32_t)r + 0x800000) >> 24;
  *np = n;
  return fma(-(double)n, p.hpi, x);
}

// reduce_large: 32x96-bit product with the 4/pi table, exact 2.62 fixed-point modulo.
FBR_SC_HD inline double reduce_large(uint32_t xi, int* np) {
  const int base = (xi >> 26) & 15;
  const int shift = (xi >> 23) & 7;
  xi = (xi & 0xffffff) | 0x800000;
  xi <<= shift;
  uint64_t res0 = (uint64_t)(uint32_t)(xi * inv_pio4(base));
  const uint64_t res1 = (uint64_t)xi * inv_pio4(base + 4);
  const uint64_t res2 = (uint64_t)xi * inv_pio4(base + 8);
  res0 = (res2 >> 32) | (res0 << 32);
  res0 += res1;
  const uint64_t n = (res0 + (1ULL << 61)) >> 62;
  res0 -= n << 62;
  const double x = (double)(int64_t)res0;
  *np = (int)n;
  return x * 0x1.921FB54442D18p-62;  // pi63 = 2pi * 2^-64
}

}  // namespace glibc_sincosf

// glibc 2.35 sinf (s_sinf.c, FMA variant).
FBR_SC_HD inline float gl_sinf(float y) {
  using namespace glibc_sincosf;
  double x = y;
  const Table* p = &table(0);
  int n;
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {  // |y| < pi/4
    const double s = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return y;
    return poly(x, s, *p, 0);
  }
  if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, *p, &n);
    const double s = p->sign[n & 3];
    if (n & 2) p = &table(1);
    return poly(x * s, x * x, *p, n);
  }
  if (abstop12(y) < abstop12(__builtin_inff())) {
    const uint32_t xi = asuint(y);
    const int sign = xi >> 31;
    x = reduce_large(xi, &n);
    const double s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) p = &table(1);
    return poly(x * s, x * x, *p, n);
  }
  return (y - y) / (y - y);  // __math_invalidf: NaN
}

// glibc 2.35 cosf (s_cosf.c, FMA variant).
FBR_SC_HD inline float gl_cosf(float y) {
  using namespace glibc_sincosf;
  double x = y;
  const Table* p = &table(0);
  int n;
  if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
    const double x2 = x * x;
    if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
    return poly(x, x2, *p, 1);
  }
  if (abstop12(y) < abstop12(120.0f)) {
    x = reduce_fast(x, *p, &n);
    const double s = p->sign[n & 3];
    if (n & 2) p = &table(1);
    return poly(x * s, x * x, *p, n ^ 1);
  }
  if (abstop12(y) < abstop12(__builtin_inff())) {
    const uint32_t xi = asuint(y);
    const int sign = xi >> 31;
    x = reduce_large(xi, &n);
    const double s = p->sign[(n + sign) & 3];
    if ((n + sign) & 2) p = &table(1);
    return poly(x * s, x * x, *p, n ^ 1);
  }
  return (y - y) / (y - y);
}

}  // namespace fbr
