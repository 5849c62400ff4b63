// Host-compiled probes of the device headers (test infrastructure): the same source the kernels
// use (fbr_fdlibm.h, fbr_sort.h), compiled for the CPU so the tests can compare it with the
// reference's real dependencies (glibc atan2f, libstdc++ std::sort) without a GPU.
#include <stdint.h>

#include "fbr_fdlibm.h"
#include "fbr_sort.h"

extern "C" {

void probe_atan2f(const float* y, const float* x, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = fbr::fd_atan2f(y[i], x[i]);
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
