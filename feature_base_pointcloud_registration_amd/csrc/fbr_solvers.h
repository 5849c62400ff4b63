// fbr_solvers.h — single-lane float small dense solvers used inside the registration kernels.
//
// The reference calls third-party solvers inside its hot loop; each is restated here in float
// with the published algorithm's operation order (no FMA: the library is built with
// -ffp-contract=off) so the device residuals and normal-equation solves follow the reference:
//   cv::eigen on the 3x3 corner covariance   mapOptmization.h:1060  -> jacobi_eigen<3>
//   cv::eigen on the 6x6 AtA (degeneracy)    mapOptmization.h:1353  -> jacobi_eigen<6>
//   cv::solve(AtA, AtB, X, DECOMP_QR)        mapOptmization.h:1343  -> qr_solve6
//   matV.inv() (LU)                          mapOptmization.h:1370  -> lu_inv6
//   Eigen colPivHouseholderQr().solve        mapOptmization.h:1169  -> colpiv_solve53
//   OpenCV CV_32F gemm (double accumulate)   mapOptmization.h:1338-1340,1370,1376
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>

#include "fbr_common.h"

namespace fbr {

__device__ __forceinline__ float cvhypot(float a, float b) {
  a = fabsf(a);
  b = fabsf(b);
  if (a > b) {
    b /= a;
    return a * sqrt_rn(1.0f + b * b);
  }
  if (b > 0.0f) {
    a /= b;
    return b * sqrt_rn(1.0f + a * a);
  }
  return 0.0f;
}

// Register-resident access helpers: every array index below is a compile-time constant after
// unrolling (data-dependent indices are resolved by selects), so nothing spills to scratch.
// (The empty asm keeps the optimiser from folding the select chain back into an indexed load
// from a stack array, which would put the whole array in scratch.)
template <int N>
__device__ __forceinline__ float sel_get(const float* a, int i) {
  float r = a[0];
#pragma unroll
  for (int j = 1; j < N; ++j) {
    r = (i == j) ? a[j] : r;
    __asm__ volatile("" : "+v"(r));
  }
  return r;
}
template <int N>
__device__ __forceinline__ int sel_geti(const int* a, int i) {
  int r = a[0];
#pragma unroll
  for (int j = 1; j < N; ++j) {
    r = (i == j) ? a[j] : r;
    __asm__ volatile("" : "+v"(r));
  }
  return r;
}

// OpenCV JacobiImpl_<float>: A (N x N row-major, destroyed), W eigenvalues (descending),
// V rows = eigenvectors.
template <int N, int IDX>
__device__ __forceinline__ void jac_update_ind(const float* A, int* indR, int* indC) {
  float mv;
  if constexpr (IDX < N - 1) {
    int m = IDX + 1;
    mv = fabsf(A[N * IDX + m]);
#pragma unroll
    for (int i = IDX + 2; i < N; i++) {
      float val = fabsf(A[N * IDX + i]);
      if (mv < val) mv = val, m = i;
    }
    indR[IDX] = m;
  }
  if constexpr (IDX > 0) {
    int m = 0;
    mv = fabsf(A[IDX]);
#pragma unroll
    for (int i = 1; i < IDX; i++) {
      float val = fabsf(A[N * i + IDX]);
      if (mv < val) mv = val, m = i;
    }
    indC[IDX] = m;
  }
}

template <int N, int I>
__device__ __forceinline__ void jac_init_ind(const float* A, int* indR, int* indC) {
  jac_update_ind<N, I>(A, indR, indC);
  if constexpr (I + 1 < N) jac_init_ind<N, I + 1>(A, indR, indC);
}

// One rotation on the pivot (K, L), K < L.  Returns true when |p| <= eps (converged).
template <int N, int K, int L>
__device__ __forceinline__ bool jac_step(float* A, float* W, float* V, int* indR, int* indC) {
  const float eps = FLT_EPSILON;
  float p = A[N * K + L];
  if (fabsf(p) <= eps) return true;
  float y = (float)((double)(W[L] - W[K]) * 0.5);
  float t = fabsf(y) + cvhypot(p, y);
  float s = cvhypot(p, t);
  float c = t / s;
  s = p / s;
  t = (p / t) * p;
  if (y < 0.0f) s = -s, t = -t;
  A[N * K + L] = 0.0f;
  W[K] -= t;
  W[L] += t;
  float a0, b0;
#define FBR_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
#pragma unroll
  for (int i = 0; i < K; i++) FBR_ROT(A[N * i + K], A[N * i + L]);
#pragma unroll
  for (int i = K + 1; i < L; i++) FBR_ROT(A[N * K + i], A[N * i + L]);
#pragma unroll
  for (int i = L + 1; i < N; i++) FBR_ROT(A[N * K + i], A[N * L + i]);
#pragma unroll
  for (int i = 0; i < N; i++) FBR_ROT(V[N * K + i], V[N * L + i]);
#undef FBR_ROT
  jac_update_ind<N, K>(A, indR, indC);
  jac_update_ind<N, L>(A, indR, indC);
  return false;
}

template <int N, int K, int L>
__device__ __forceinline__ bool jac_dispatch(int k, int l, float* A, float* W, float* V, int* indR, int* indC) {
  if (k == K && l == L) return jac_step<N, K, L>(A, W, V, indR, indC);
  if constexpr (L + 1 < N) return jac_dispatch<N, K, L + 1>(k, l, A, W, V, indR, indC);
  else if constexpr (K + 2 < N) return jac_dispatch<N, K + 1, K + 2>(k, l, A, W, V, indR, indC);
  else return true;
}

template <int N>
__device__ void jacobi_eigen(float* A, float* W, float* V) {
  int indR[N], indC[N];
#pragma unroll
  for (int i = 0; i < N; i++)
#pragma unroll
    for (int j = 0; j < N; j++) V[i * N + j] = (i == j) ? 1.0f : 0.0f;
#pragma unroll
  for (int k = 0; k < N; k++) {
    W[k] = A[(N + 1) * k];
    indR[k] = 0;
    indC[k] = 0;
  }
  jac_init_ind<N, 0>(A, indR, indC);
  const int maxIters = N * N * 30;
  for (int iters = 0; iters < maxIters; iters++) {
    // pivot search: row maxima (indR) then column maxima (indC), strict '<' keeps the first
    int k = 0;
    float mv = fabsf(sel_get<N>(A, indR[0]));
#pragma unroll
    for (int i = 1; i < N - 1; i++) {
      float val = fabsf(sel_get<N>(A + N * i, indR[i]));
      if (mv < val) mv = val, k = i;
    }
    int l = sel_geti<N>(indR, k);
#pragma unroll
    for (int i = 1; i < N; i++) {
      float col[N];
#pragma unroll
      for (int r = 0; r < N; ++r) col[r] = A[N * r + i];
      float val = fabsf(sel_get<N>(col, indC[i]));
      if (mv < val) mv = val, k = indC[i], l = i;
    }
    if (jac_dispatch<N, 0, 1>(k, l, A, W, V, indR, indC)) break;
  }
  // selection sort, descending (first maximum), swapping eigenvector rows
#pragma unroll
  for (int k = 0; k < N - 1; k++) {
    int m = k;
    float wm = W[k];
#pragma unroll
    for (int i = k + 1; i < N; i++)
      if (wm < W[i]) m = i, wm = W[i];
#pragma unroll
    for (int j = k + 1; j < N; j++) {
      if (m == j) {
        float t = W[j];
        W[j] = W[k];
        W[k] = t;
#pragma unroll
        for (int i = 0; i < N; i++) {
          float u = V[N * j + i];
          V[N * j + i] = V[N * k + i];
          V[N * k + i] = u;
        }
      }
    }
  }
}

// Same algorithm on per-lane arrays in LDS, element e of a lane's array at base[e * S] (S = the
// workgroup size, so lanes of a wave always hit distinct banks).  Data-dependent pivots index
// LDS directly: no divergence across lanes whose pivots differ (used for the 6x6 degeneracy
// eigen-decomposition, one job per lane).
template <int N, int S>
__device__ void jacobi_eigen_lds(float* A, float* W, float* V, int* indR, int* indC) {
  const float eps = FLT_EPSILON;
#define A_(i) A[(i) * S]
#define V_(i) V[(i) * S]
#define W_(i) W[(i) * S]
#define R_(i) indR[(i) * S]
#define C_(i) indC[(i) * S]
  for (int i = 0; i < N; i++)
    for (int j = 0; j < N; j++) V_(i * N + j) = (i == j) ? 1.0f : 0.0f;
  float mv;
  for (int k = 0; k < N; k++) {
    W_(k) = A_((N + 1) * k);
    if (k < N - 1) {
      int m = k + 1;
      mv = fabsf(A_(N * k + m));
      for (int i = k + 2; i < N; i++) {
        float val = fabsf(A_(N * k + i));
        if (mv < val) mv = val, m = i;
      }
      R_(k) = m;
    }
    if (k > 0) {
      int m = 0;
      mv = fabsf(A_(k));
      for (int i = 1; i < k; i++) {
        float val = fabsf(A_(N * i + k));
        if (mv < val) mv = val, m = i;
      }
      C_(k) = m;
    }
  }
  const int maxIters = N * N * 30;
  for (int iters = 0; iters < maxIters; iters++) {
    int k = 0;
    mv = fabsf(A_(R_(0)));
    for (int i = 1; i < N - 1; i++) {
      float val = fabsf(A_(N * i + R_(i)));
      if (mv < val) mv = val, k = i;
    }
    int l = R_(k);
    for (int i = 1; i < N; i++) {
      float val = fabsf(A_(N * C_(i) + i));
      if (mv < val) mv = val, k = C_(i), l = i;
    }
    float p = A_(N * k + l);
    if (fabsf(p) <= eps) break;
    float y = (float)((double)(W_(l) - W_(k)) * 0.5);
    float t = fabsf(y) + cvhypot(p, y);
    float s = cvhypot(p, t);
    float c = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0.0f) s = -s, t = -t;
    A_(N * k + l) = 0.0f;
    W_(k) -= t;
    W_(l) += t;
    float a0, b0;
#define FBR_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
    for (int i = 0; i < k; i++) FBR_ROT(A_(N * i + k), A_(N * i + l));
    for (int i = k + 1; i < l; i++) FBR_ROT(A_(N * k + i), A_(N * i + l));
    for (int i = l + 1; i < N; i++) FBR_ROT(A_(N * k + i), A_(N * l + i));
    for (int i = 0; i < N; i++) FBR_ROT(V_(N * k + i), V_(N * l + i));
#undef FBR_ROT
    for (int j = 0; j < 2; j++) {
      int idx = j == 0 ? k : l;
      if (idx < N - 1) {
        int m = idx + 1;
        mv = fabsf(A_(N * idx + m));
        for (int i = idx + 2; i < N; i++) {
          float val = fabsf(A_(N * idx + i));
          if (mv < val) mv = val, m = i;
        }
        R_(idx) = m;
      }
      if (idx > 0) {
        int m = 0;
        mv = fabsf(A_(idx));
        for (int i = 1; i < idx; i++) {
          float val = fabsf(A_(N * i + idx));
          if (mv < val) mv = val, m = i;
        }
        C_(idx) = m;
      }
    }
  }
  for (int k = 0; k < N - 1; k++) {
    int m = k;
    for (int i = k + 1; i < N; i++)
      if (W_(m) < W_(i)) m = i;
    if (k != m) {
      float t = W_(m);
      W_(m) = W_(k);
      W_(k) = t;
      for (int i = 0; i < N; i++) {
        float u = V_(N * m + i);
        V_(N * m + i) = V_(N * k + i);
        V_(N * k + i) = u;
      }
    }
  }
#undef A_
#undef V_
#undef W_
#undef R_
#undef C_
}

// LDS writes of this wave visible to all its lanes (no workgroup barrier: the other waves of the
// workgroup do not take part).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// isDegenerate without the eigen-decomposition (mapOptmization.h:1353-1366 only needs to know
// whether some eigenvalue of the float matAtA is below thr = 100; matP is used only when one is).
// Every eigenvalue exceeds thr + m, m = 1e-3 ||A||_F, iff A - (thr + m) I is positive definite,
// which an LDL^T factorisation in double decides (its own rounding, ~1e-16 ||A||, is negligible
// next to m).  OpenCV's float Jacobi returns eigenvalues within a few hundred float roundings of
// the exact ones (~1e-5 ||A|| at most, against the 1e-3 ||A|| margin), so when this returns true
// none of them can fall below thr and the reference's isDegenerate is false.  false = not
// certified: run the Jacobi.  NaN / Inf inputs are never certified.
template <int N>
__device__ __forceinline__ bool eig_above_certified(const float* A, float thr) {
  double fro = 0.0;
#pragma unroll
  for (int k = 0; k < N * N; ++k) fro += (double)A[k] * (double)A[k];
  const double tau = (double)thr + 1e-3 * sqrt(fro);
  double L[N][N], D[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double d = (double)A[j * N + j] - tau;
#pragma unroll
    for (int k = 0; k < j; ++k) d -= L[j][k] * L[j][k] * D[k];
    if (!(d > 0.0) || !(d < 1e300)) return false;
    D[j] = d;
#pragma unroll
    for (int i = j + 1; i < N; ++i) {
      double v = (double)A[i * N + j];
#pragma unroll
      for (int k = 0; k < j; ++k) v -= L[i][k] * L[j][k] * D[k];
      L[i][j] = v / d;
    }
  }
  return true;
}

// The same algorithm by one whole wave on shared arrays (A, V: N*N; W, indR, indC: N).  Every lane
// finds the pivot (uniform LDS reads); the element pairs of one rotation are disjoint, so lane i
// rotates the A pair and lane N+i the V pair of index i with the per-element operations of
// jac_step; lanes 0 and 1 refresh the row / column maxima of k and l.  Same rotation sequence and
// float results as jacobi_eigen<N> in a fraction of its dependent-instruction chain.
template <int N>
__device__ void jacobi_eigen_wave(float* A, float* W, float* V, int* indR, int* indC) {
  static_assert(2 * N <= 64 && N * N <= 64, "one wave");
  const int lane = threadIdx.x & 63;
  const float eps = FLT_EPSILON;
  if (lane < N * N) V[lane] = (lane / N == lane % N) ? 1.0f : 0.0f;
  auto update_ind = [&](int idx) {
    float mv;
    if (idx < N - 1) {
      int m = idx + 1;
      mv = fabsf(A[N * idx + m]);
      for (int i = idx + 2; i < N; i++) {
        float val = fabsf(A[N * idx + i]);
        if (mv < val) mv = val, m = i;
      }
      indR[idx] = m;
    }
    if (idx > 0) {
      int m = 0;
      mv = fabsf(A[idx]);
      for (int i = 1; i < idx; i++) {
        float val = fabsf(A[N * i + idx]);
        if (mv < val) mv = val, m = i;
      }
      indC[idx] = m;
    }
  };
  if (lane < N) {
    W[lane] = A[(N + 1) * lane];
    update_ind(lane);
  }
  wave_lds_sync();
  const int maxIters = N * N * 30;
  for (int iters = 0; iters < maxIters; iters++) {
    int k = 0;
    float mv = fabsf(A[indR[0]]);
    for (int i = 1; i < N - 1; i++) {
      float val = fabsf(A[N * i + indR[i]]);
      if (mv < val) mv = val, k = i;
    }
    int l = indR[k];
    for (int i = 1; i < N; i++) {
      float val = fabsf(A[N * indC[i] + i]);
      if (mv < val) mv = val, k = indC[i], l = i;
    }
    k = __builtin_amdgcn_readfirstlane(k);
    l = __builtin_amdgcn_readfirstlane(l);
    const float p = A[N * k + l];
    if (fabsf(p) <= eps) break;
    const float wl = W[l], wk = W[k];
    float y = (float)((double)(wl - wk) * 0.5);
    float t = fabsf(y) + cvhypot(p, y);
    float s = cvhypot(p, t);
    float c = t / s;
    s = p / s;
    t = (p / t) * p;
    if (y < 0.0f) s = -s, t = -t;
    wave_lds_sync();  // every lane has read the pivot row / column state
    if (lane < N) {
      const int i = lane;
      int e0 = -1, e1 = -1;
      if (i < k) e0 = N * i + k, e1 = N * i + l;
      else if (i > k && i < l) e0 = N * k + i, e1 = N * i + l;
      else if (i > l) e0 = N * k + i, e1 = N * l + i;
      if (e0 >= 0) {
        const float a0 = A[e0], b0 = A[e1];
        A[e0] = a0 * c - b0 * s;
        A[e1] = a0 * s + b0 * c;
      }
      if (i == 0) {
        A[N * k + l] = 0.0f;
        W[k] = wk - t;
        W[l] = wl + t;
      }
    } else if (lane < 2 * N) {
      const int i = lane - N;
      const float a0 = V[N * k + i], b0 = V[N * l + i];
      V[N * k + i] = a0 * c - b0 * s;
      V[N * l + i] = a0 * s + b0 * c;
    }
    wave_lds_sync();
    if (lane < 2) update_ind(lane == 0 ? k : l);
    wave_lds_sync();
  }
  if (lane == 0) {
    for (int k = 0; k < N - 1; k++) {
      int m = k;
      for (int i = k + 1; i < N; i++)
        if (W[m] < W[i]) m = i;
      if (k != m) {
        float t = W[m];
        W[m] = W[k];
        W[k] = t;
        for (int i = 0; i < N; i++) {
          float u = V[N * m + i];
          V[N * m + i] = V[N * k + i];
          V[N * k + i] = u;
        }
      }
    }
  }
  wave_lds_sync();
}

// OpenCV QRImpl (Householder) for a 6x6 system, eps = FLT_EPSILON*10; returns 0 if singular.
__device__ int qr_solve6(float* A, float* b) {
  const int n = 6, m = 6;
  const float eps = FLT_EPSILON * 10.0f;
  float vl[6], hF[6];
#pragma unroll
  for (int l = 0; l < n; l++) {
    const int vlSize = m - l;
    float vlNorm = 0.0f;
  #pragma unroll
  for (int i = 0; i < vlSize; i++) {
      vl[i] = A[(l + i) * n + l];
      vlNorm += vl[i] * vl[i];
    }
    float tmpV = vl[0];
    vl[0] = vl[0] + (vl[0] >= 0.0f ? 1.0f : -1.0f) * sqrt_rn(vlNorm);
    vlNorm = sqrt_rn(vlNorm + vl[0] * vl[0] - tmpV * tmpV);
  #pragma unroll
  for (int i = 0; i < vlSize; i++) vl[i] /= vlNorm;
  #pragma unroll
  for (int j = l; j < n; j++) {
      float v_lA = 0.0f;
    #pragma unroll
  for (int i = l; i < m; i++) v_lA += vl[i - l] * A[i * n + j];
    #pragma unroll
  for (int i = l; i < m; i++) A[i * n + j] -= 2.0f * vl[i - l] * v_lA;
    }
    hF[l] = vl[0] * vl[0];
  #pragma unroll
  for (int i = 1; i < vlSize; i++) A[(l + i) * n + l] = vl[i] / vl[0];
  }
#pragma unroll
  for (int l = 0; l < n; l++) {
    vl[0] = 1.0f;
  #pragma unroll
  for (int j = 1; j < m - l; j++) vl[j] = A[(j + l) * n + l];
    float v_lB = 0.0f;
  #pragma unroll
  for (int i = l; i < m; i++) v_lB += vl[i - l] * b[i];
  #pragma unroll
  for (int i = l; i < m; i++) b[i] -= 2.0f * vl[i - l] * v_lB * hF[l];
  }
#pragma unroll
  for (int i = n - 1; i >= 0; i--) {
  #pragma unroll
  for (int j = n - 1; j > i; j--) b[i] -= b[j] * A[i * n + j];
    if (fabsf(A[i * n + i]) < eps) return 0;
    b[i] /= A[i * n + i];
  }
  return 1;
}

// OpenCV LUImpl with an identity right-hand side (Mat::inv, DECOMP_LU), 6x6, eps FLT_EPSILON*10.
__device__ int lu_inv6(const float* Ain, float* Bi) {
  constexpr int n = 6;
  const float eps = FLT_EPSILON * 10.0f;
  float A[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) A[i] = Ain[i];
#pragma unroll
  for (int i = 0; i < n; i++)
#pragma unroll
    for (int j = 0; j < n; j++) Bi[i * n + j] = (i == j) ? 1.0f : 0.0f;
#pragma unroll
  for (int i = 0; i < n; i++) {
    int k = i;
    float ak = fabsf(A[i * n + i]);
#pragma unroll
    for (int j = i + 1; j < n; j++)
      if (fabsf(A[j * n + i]) > ak) k = j, ak = fabsf(A[j * n + i]);
    if (ak < eps) return 0;
#pragma unroll
    for (int r = i + 1; r < n; r++) {
      if (k == r) {
#pragma unroll
        for (int j = i; j < n; j++) {
          float t = A[i * n + j];
          A[i * n + j] = A[r * n + j];
          A[r * n + j] = t;
        }
#pragma unroll
        for (int j = 0; j < n; j++) {
          float t = Bi[i * n + j];
          Bi[i * n + j] = Bi[r * n + j];
          Bi[r * n + j] = t;
        }
      }
    }
    float d = -1.0f / A[i * n + i];
#pragma unroll
    for (int j = i + 1; j < n; j++) {
      float alpha = A[j * n + i] * d;
#pragma unroll
      for (int c = i + 1; c < n; c++) A[j * n + c] += alpha * A[i * n + c];
#pragma unroll
      for (int c = 0; c < n; c++) Bi[j * n + c] += alpha * Bi[i * n + c];
    }
  }
#pragma unroll
  for (int i = n - 1; i >= 0; i--)
#pragma unroll
    for (int j = 0; j < n; j++) {
      float s = Bi[i * n + j];
#pragma unroll
      for (int c = i + 1; c < n; c++) s -= A[i * n + c] * Bi[c * n + j];
      Bi[i * n + j] = s / A[i * n + i];
    }
  return 1;
}

// OpenCV gemm for CV_32F: double accumulation, float store.  C[M][N] = A[M][K] B[K][N].
template <int M, int K, int N>
__device__ __forceinline__ void gemm_f32_acc64(const float* A, const float* B, float* C) {
#pragma unroll
  for (int i = 0; i < M; i++)
#pragma unroll
    for (int j = 0; j < N; j++) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < K; k++) s += (double)A[i * K + k] * (double)B[k * N + j];
      C[i * N + j] = (float)s;
    }
}

// Eigen 3.3 ColPivHouseholderQR<Matrix<float,5,3>>::compute(A).solve(b), sequential sums.
__device__ void colpiv_solve53(const float (&Ain)[5][3], const float (&bin)[5], float (&x)[3]) {
  constexpr int rows = 5, cols = 3, size = 3;
  float qr[5][3];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) qr[i][j] = Ain[i][j];
  float hc[3], nUpd[3], nDir[3];
  int transp[3];
#pragma unroll
  for (int k = 0; k < cols; ++k) {
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < rows; i++) s += qr[i][k] * qr[i][k];
    nDir[k] = sqrt_rn(s);
    nUpd[k] = nDir[k];
  }
  const float eps = FLT_EPSILON;
  float mxn = nUpd[0];
#pragma unroll
  for (int k = 1; k < cols; ++k)
    if (nUpd[k] > mxn) mxn = nUpd[k];
  const float th = (mxn * eps) * (mxn * eps) / (float)rows;
  const float ndt = sqrt_rn(eps);
  int nz = size;
#pragma unroll
  for (int k = 0; k < size; ++k) {
    int big = k;
    float bv = nUpd[k];
#pragma unroll
    for (int j = k + 1; j < cols; ++j)
      if (nUpd[j] > bv) bv = nUpd[j], big = j;
    const float bsq = bv * bv;
    if (nz == size && bsq < th * (float)(rows - k)) nz = k;
    transp[k] = big;
#pragma unroll
    for (int j = k + 1; j < cols; ++j) {
      if (big == j) {
#pragma unroll
        for (int i = 0; i < rows; ++i) {
          float t = qr[i][k];
          qr[i][k] = qr[i][j];
          qr[i][j] = t;
        }
        float t = nUpd[k];
        nUpd[k] = nUpd[j];
        nUpd[j] = t;
        t = nDir[k];
        nDir[k] = nDir[j];
        nDir[j] = t;
      }
    }
    float tailSq = 0.0f;
#pragma unroll
    for (int i = k + 1; i < rows; ++i) tailSq += qr[i][k] * qr[i][k];
    const float c0 = qr[k][k];
    float beta, tau;
    if (tailSq <= FLT_MIN) {
      tau = 0.0f;
      beta = c0;
#pragma unroll
      for (int i = k + 1; i < rows; ++i) qr[i][k] = 0.0f;
    } else {
      beta = sqrt_rn(c0 * c0 + tailSq);
      if (c0 >= 0.0f) beta = -beta;
      const float den = c0 - beta;
#pragma unroll
      for (int i = k + 1; i < rows; ++i) qr[i][k] = qr[i][k] / den;
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    qr[k][k] = beta;
    if (k + 1 < cols && tau != 0.0f) {
#pragma unroll
      for (int j = k + 1; j < cols; ++j) {
        float tmp = 0.0f;
#pragma unroll
        for (int i = k + 1; i < rows; ++i) tmp += qr[i][k] * qr[i][j];
        tmp += qr[k][j];
        qr[k][j] -= tau * tmp;
#pragma unroll
        for (int i = k + 1; i < rows; ++i) qr[i][j] -= tmp * (tau * qr[i][k]);
      }
    }
#pragma unroll
    for (int j = k + 1; j < cols; ++j) {
      if (nUpd[j] != 0.0f) {
        float temp = fabsf(qr[k][j]) / nUpd[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        const float q = nUpd[j] / nDir[j];
        const float temp2 = temp * (q * q);
        if (temp2 <= ndt) {
          float s = 0.0f;
#pragma unroll
          for (int i = k + 1; i < rows; i++) s += qr[i][j] * qr[i][j];
          nDir[j] = sqrt_rn(s);
          nUpd[j] = nDir[j];
        } else {
          nUpd[j] *= sqrt_rn(temp);
        }
      }
    }
  }
  // permutation from the transpositions
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < size; ++k) {
#pragma unroll
    for (int j = k + 1; j < size; ++j) {
      if (transp[k] == j) {
        int t = perm[k];
        perm[k] = perm[j];
        perm[j] = t;
      }
    }
  }
  if (nz == 0) {
    x[0] = x[1] = x[2] = 0.0f;
    return;
  }
  float c[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) c[i] = bin[i];
#pragma unroll
  for (int k = 0; k < size; ++k) {
    if (k >= nz) break;
    const float tau = hc[k];
    if (rows - k == 1) {
      c[k] *= 1.0f - tau;
    } else if (tau != 0.0f) {
      float tmp = 0.0f;
#pragma unroll
      for (int i = k + 1; i < rows; ++i) tmp += qr[i][k] * c[i];
      tmp += c[k];
      c[k] -= tau * tmp;
#pragma unroll
      for (int i = k + 1; i < rows; ++i) c[i] -= tmp * (tau * qr[i][k]);
    }
  }
#pragma unroll
  for (int i = size - 1; i >= 0; --i) {
    if (i < nz && c[i] != 0.0f) {
      c[i] /= qr[i][i];
#pragma unroll
      for (int t = 0; t < i; ++t) c[t] -= c[i] * qr[t][i];
    }
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) x[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < size; ++i) {
    if (i < nz) {
#pragma unroll
      for (int j = 0; j < 3; ++j)
        if (perm[i] == j) x[j] = c[i];
    }
  }
}

}  // namespace fbr
