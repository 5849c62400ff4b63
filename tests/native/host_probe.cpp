// Host-compiled probes of the device headers (test infrastructure): the same source the kernels
// use (fbr_fdlibm.h, fbr_sort.h), compiled for the CPU so the tests can compare it with the
// reference's real dependencies (glibc atan2f, libstdc++ std::sort) without a GPU.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <thread>
#include <vector>

#include "fbr_fdlibm.h"
#include "fbr_sincosf.h"
#include "fbr_sort.h"

extern "C" {

void probe_atan2f(const float* y, const float* x, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = fbr::fd_atan2f(y[i], x[i]);
}

// The host glibc sinf / cosf (the reference's libm) on an array.
void probe_glibc_sincosf(const float* x, float* s, float* c, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    s[i] = ::sinf(x[i]);
    c[i] = ::cosf(x[i]);
  }
}

// fbr_sincosf.h against the host glibc over every float whose bit pattern u satisfies
// lo <= u < hi with u % stride == 0 (threads split the range); returns the mismatch count.
uint64_t probe_sincosf_range(uint64_t lo, uint64_t hi, uint64_t stride, int threads) {
  std::atomic<uint64_t> bad{0};
  std::vector<std::thread> th;
  if (threads < 1) threads = 1;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      uint64_t b = 0;
      for (uint64_t u = lo + (uint64_t)t * stride; u < hi; u += (uint64_t)threads * stride) {
        const uint32_t ui = (uint32_t)u;
        float x;
        memcpy(&x, &ui, 4);
        const float r[4] = {::sinf(x), fbr::gl_sinf(x), ::cosf(x), fbr::gl_cosf(x)};
        uint32_t k[4];
        memcpy(k, r, sizeof(k));
        if (k[0] != k[1] && !(isnan(r[0]) && isnan(r[1]))) ++b;
        if (k[2] != k[3] && !(isnan(r[2]) && isnan(r[3]))) ++b;
      }
      bad += b;
    });
  for (auto& x : th) x.join();
  return bad;
}

// std::sort emulation on {value, index} pairs; writes the resulting index order.
void probe_sort(const float* values, int64_t n, int64_t* ind_out) {
  fbr::SmoothEntry* a = new fbr::SmoothEntry[n > 0 ? n : 1];
  for (int64_t i = 0; i < n; ++i) a[i] = fbr::SmoothEntry{values[i], (int)i};
  fbr::std_sort_emul(a, (int)n);
  for (int64_t i = 0; i < n; ++i) ind_out[i] = a[i].ind;
  delete[] a;
}

}
