// Runtime probe: are host-to-device hipMemcpyAsync copies from pageable memory on a non-blocking
// stream seen intact by the next kernel on that stream?  Each trial fills a pageable buffer with a
// fresh pattern, copies it asynchronously, and a kernel on the same stream counts the words that
// differ from the pattern; small copies from a stack variable are checked the same way.
// Variants: 0 = pageable hipMemcpyAsync, 1 = hipMemcpy (blocking), 2 = pinned hipMemcpyAsync.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/pageable_probe tools/pageable_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_check(const unsigned* d, size_t n, unsigned seed, unsigned* bad) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    if (d[i] != (unsigned)(i * 2654435761u) + seed) atomicAdd(bad, 1u);
}

__global__ void k_check_small(const unsigned* d, unsigned want, unsigned* bad) {
  if (threadIdx.x == 0 && d[0] != want) atomicAdd(bad + 1, 1u);
}

static int run(int variant, size_t n, int trials) {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
  unsigned *d = nullptr, *dsmall = nullptr, *bad = nullptr, *hp = nullptr;
  if (hipMalloc(&d, n * 4) != hipSuccess || hipMalloc(&dsmall, 4) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess ||
      hipHostMalloc(&hp, n * 4, hipHostMallocDefault) != hipSuccess)
    return 2;
  std::vector<unsigned> pg(n);
  unsigned long long bad_big = 0, bad_small = 0;
  for (int t = 0; t < trials; ++t) {
    const unsigned seed = 0x9E3779B9u * (unsigned)(t + 1);
    unsigned* src = variant == 2 ? hp : pg.data();
    for (size_t i = 0; i < n; ++i) src[i] = (unsigned)(i * 2654435761u) + seed;
    (void)hipMemsetAsync(bad, 0, 8, s);
    if (variant == 1) {
      (void)hipStreamSynchronize(s);
      (void)hipMemcpy(d, src, n * 4, hipMemcpyHostToDevice);
    } else {
      (void)hipMemcpyAsync(d, src, n * 4, hipMemcpyHostToDevice, s);
    }
    {
      const unsigned v = seed ^ 0x5A5A5A5Au;  // stack source, out of scope after the call
      (void)hipMemcpyAsync(dsmall, &v, 4, hipMemcpyHostToDevice, s);
    }
    k_check<<<1024, 256, 0, s>>>(d, n, seed, bad);
    k_check_small<<<1, 64, 0, s>>>(dsmall, seed ^ 0x5A5A5A5Au, bad);
    unsigned hb[2] = {0, 0};
    (void)hipMemcpyAsync(hb, bad, 8, hipMemcpyDeviceToHost, s);
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    bad_big += hb[0] != 0;
    bad_small += hb[1] != 0;
    // rewrite the pageable buffer right away (a copy still reading it would now see junk)
    for (size_t i = 0; i < n; i += 1024) src[i] = 0xDEADBEEFu;
  }
  std::printf("variant %d n=%zu words trials=%d: bad big copies %llu, bad small copies %llu\n", variant, n, trials,
              bad_big, bad_small);
  (void)hipFree(d);
  (void)hipFree(dsmall);
  (void)hipFree(bad);
  (void)hipHostFree(hp);
  (void)hipStreamDestroy(s);
  return 0;
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 200;
  for (size_t n : {(size_t)6, (size_t)1024, (size_t)489440, (size_t)4 << 20})
    for (int v = 0; v < 3; ++v)
      if (int rc = run(v, n, trials)) return rc;
  return 0;
}
