// Diagnostic micro-benchmark of the small dense solvers of k_gn_solve (fbr_solvers.h): clock
// cycles per call of each solver on one 6x6 normal-equation matrix, one wave, no other work on
// the device (the single-scan latency regime).  Build and run (GPU box):
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 \
//     -I feature_base_pointcloud_registration_amd/csrc -I include tools/solver_bench.hip -o /tmp/sb && /tmp/sb
#include <hip/hip_runtime.h>

#include <cstdio>

#include "fbr_solvers.h"

using namespace fbr;

constexpr int kReps = 64;

__global__ void k_bench(const float* A0, const float* b0, long long* cyc, float* sink) {
  __shared__ float A[36], V[36], W[6];
  __shared__ int R[6], C[6];
  const int lane = threadIdx.x;
  float acc = 0.0f;
  // 0: single-lane register Jacobi
  long long t0 = clock64();
  for (int r = 0; r < kReps; ++r) {
    if (lane == 0) {
      float Ar[36], Wr[6], Vr[36];
      for (int k = 0; k < 36; ++k) Ar[k] = A0[k] + (float)(r & 1) * 0.0f;
      jacobi_eigen<6>(Ar, Wr, Vr);
      acc += Wr[5] + Vr[7];
    }
    __builtin_amdgcn_wave_barrier();
  }
  long long t1 = clock64();
  // 1: wave Jacobi in LDS
  for (int r = 0; r < kReps; ++r) {
    if (lane < 36) A[lane] = A0[lane];
    wave_lds_sync();
    jacobi_eigen_wave<6>(A, W, V, R, C);
    acc += W[5];
  }
  long long t2 = clock64();
  // 2: QR solve
  for (int r = 0; r < kReps; ++r) {
    if (lane == 0) {
      float Ar[36], x[6];
      for (int k = 0; k < 36; ++k) Ar[k] = A0[k];
      for (int k = 0; k < 6; ++k) x[k] = b0[k];
      qr_solve6(Ar, x);
      acc += x[3];
    }
    __builtin_amdgcn_wave_barrier();
  }
  long long t3 = clock64();
  // 3: LU inverse + gemm
  for (int r = 0; r < kReps; ++r) {
    if (lane == 0) {
      float Vi[36], P[36];
      lu_inv6(A0, Vi);
      for (int k = 0; k < 36; ++k) P[k] = 0.0f;
      gemm_f32_acc64<6, 6, 6>(Vi, A0, P);
      acc += P[11];
    }
    __builtin_amdgcn_wave_barrier();
  }
  long long t4 = clock64();
  // 4: cvhypot chain
  float h = A0[1];
  for (int r = 0; r < kReps * 36; ++r) h = cvhypot(h, A0[r % 36]) * 1e-3f;
  long long t5 = clock64();
  if (lane == 0) {
    cyc[0] = (t1 - t0) / kReps;
    cyc[1] = (t2 - t1) / kReps;
    cyc[2] = (t3 - t2) / kReps;
    cyc[3] = (t4 - t3) / kReps;
    cyc[4] = (t5 - t4) / (kReps * 36);
    sink[0] = acc + h;
  }
}

int main() {
  // a C2-like iteration-0 AtA (symmetric, ||A||_F ~ 3e5, min eigenvalue ~ 1e3) and AtB
  float A[36], b[6];
  const float d[6] = {3.1e5f, 1.2e5f, 4.0e4f, 9.0e3f, 2.5e3f, 1.1e3f};
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) A[i * 6 + j] = (i == j) ? d[i] : 0.0f;
  // dense symmetric coupling: A = Q D Q^T with a fixed rotation sequence
  for (int rep = 0; rep < 3; ++rep)
    for (int p = 0; p < 6; ++p)
      for (int q = p + 1; q < 6; ++q) {
        const float c = 0.9f, s = 0.43588989f;
        for (int i = 0; i < 6; ++i) {
          const float x = A[i * 6 + p], y = A[i * 6 + q];
          A[i * 6 + p] = c * x - s * y;
          A[i * 6 + q] = s * x + c * y;
        }
        for (int j = 0; j < 6; ++j) {
          const float x = A[p * 6 + j], y = A[q * 6 + j];
          A[p * 6 + j] = c * x - s * y;
          A[q * 6 + j] = s * x + c * y;
        }
      }
  for (int i = 0; i < 6; ++i)
    for (int j = i + 1; j < 6; ++j) A[j * 6 + i] = A[i * 6 + j];
  for (int i = 0; i < 6; ++i) b[i] = 100.0f * (float)(i + 1);
  float *dA, *db, *sink;
  long long* dc;
  hipMalloc(&dA, sizeof(A));
  hipMalloc(&db, sizeof(b));
  hipMalloc(&dc, 8 * sizeof(long long));
  hipMalloc(&sink, sizeof(float));
  hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  hipMemcpy(db, b, sizeof(b), hipMemcpyHostToDevice);
  for (int warm = 0; warm < 2; ++warm) hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, dA, db, dc, sink);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, dA, db, dc, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  long long c[8];
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  printf("cycles per call: jacobi_eigen<6> (lane) %lld, jacobi_eigen_wave<6> %lld, qr_solve6 %lld, lu_inv6+gemm %lld, "
         "cvhypot %lld; kernel %.1f us\n",
         c[0], c[1], c[2], c[3], c[4], ms * 1e3);
  return 0;
}
