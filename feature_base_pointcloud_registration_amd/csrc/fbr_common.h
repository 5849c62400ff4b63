// fbr_common.h — shared device-side definitions of the MI355X registration path.
//
// HBM layout (per device batch of B jobs, each job = one scan registered from its own guess):
//   raw points   fbr_point_xyzirt [B][NMAX]           (24 B AoS, the PointXYZIRT payload)
//   cell owner   int32            [B][H*W]            first-wins claim (atomicMin of input index)
//   cloud        float4           [B][H*W]            ring-major compacted xyzi (cloud_deskewed)
//   col / range  int32 / float    [B][H*W]            cloud_info.pointColInd / pointRange
//   ring index   int32            [B][H] x2           cloud_info.startRingIndex / endRingIndex
//   label        int8             [B][H*W]            cloudLabel (the feature mask)
//   corner slot  float4           [B][H][120]         per-ring corner picks in visit order
//   surf cand    float4           [B][H][W]           per-ring surf candidates (label <= 0)
//   surf ring DS float4           [B][H][W]           per-ring VoxelGrid output
//   corner/surf  float4           [B][CAPC] / [B][H*W] concatenated feature clouds
//   cornerDS/surfDS float4        [B][CAPC] / [B][H*W] registration down-sampled queries
// Map (shared by all jobs, read-only, built once by fbr_set_map):
//   pts          float4 [M] sorted by 1 m grid cell (w = bit pattern of the global map index)
//   cell start   int32 [ncells+1]
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <limits.h>
#include <stdint.h>

#include "../../include/fbr.h"

namespace fbr {

constexpr int kEmptyOwner = 0x7F7F7F7F;   // byte-memset sentinel: larger than any point index
constexpr int kCornerPerSeg = 20;         // featureExtraction.h:217
constexpr int kCornerPerRing = 20 * 6;
constexpr int kMaxSegment = 512;          // per-ring segment length capacity (W <= 3000)
constexpr int kMaxW = 4096;               // Horizon_SCAN capacity of the per-ring kernels
constexpr float kGridCell = 1.0f;         // kNN search grid cell (>= sqrt of the d2 < 1.0 gate)

// Correctly rounded f32 sqrt (glibc sqrtf / SSE sqrtss semantics).  gfx950's f32 sqrt lowering
// (including __fsqrt_rn) is off by one ulp on ~15 % of inputs; the double sqrt is correctly rounded
// and rounding it to float is innocuous for sqrt (53 >= 2*24+2 bits).
__host__ __device__ inline float sqrt_rn(float x) { return (float)sqrt((double)x); }

// 64-bit unsigned order through the f64 unit: a u64 below 0x7FF0000000000000 read as a double is a
// non-negative, non-NaN double (a subnormal below 2^52; the kernels keep f64 denormals), and the
// order of those doubles is the integers' order, so v_min_f64 / v_max_f64 pick the smaller / larger
// key in one instruction each, where a 64-bit compare and two selects take three.  Inline asm: the
// compiler's fmin / fmax would first canonicalise each operand (sNaN quieting in IEEE mode).
constexpr unsigned long long kF64KeyMax = 0x7FEFFFFFFFFFFFFFull;  // largest such key (finite double)
__device__ __forceinline__ unsigned long long key_min(unsigned long long a, unsigned long long b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(__longlong_as_double((long long)a)), "v"(__longlong_as_double((long long)b)));
  return (unsigned long long)__double_as_longlong(r);
}
__device__ __forceinline__ unsigned long long key_max(unsigned long long a, unsigned long long b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(__longlong_as_double((long long)a)), "v"(__longlong_as_double((long long)b)));
  return (unsigned long long)__double_as_longlong(r);
}

// x86-64 cvttsd2si: NaN / out-of-range -> INT_MIN (imageProjection.cpp:611 conversion).
__host__ __device__ inline int x86_cvt(double v) {
  if (!(v > -2147483649.0 && v < 2147483648.0)) return (int)0x80000000;
  return (int)v;
}

// Stream-mode FeatureExtraction state that survives between scans (featureExtraction.h:39-42):
// the never-recomputed smoothness slot 4 and cloudNeighborPicked[0..4].
struct StreamState {
  float smooth4_value;
  int32_t smooth4_ind;
  int8_t picked04[8];
};

// Per-job Gauss-Newton state (mapOptmization.h transformTobeMapped / isDegenerate / loop).
struct GnState {
  float pose[6];      // transformTobeMapped
  float T[12];        // trans2Affine3f(pose), row-major 3x4
  float trig[6];      // srx, crx, sry, cry, srz, crz for LMOptimization
  int32_t active;     // 1 while iterating
  int32_t iter;       // LMOptimization calls made
  int32_t converged;
  int32_t degenerate;
  int32_t n_sel;
  int32_t status;     // FBR_REG_*
  float matP[36];     // iteration-0 degeneracy projection (zero afterwards: local cv::Mat)
  float crop_min[3], crop_max[3];
  int32_t pad[2];
};

struct GridDesc {        // 3D grid over a map (cell indices, not metres, in origin)
  float origin[3];       // cell index of cell (0,0,0) per axis
  float inv_cell;        // 1 / cell size along y and z (a power of two)
  float inv_x;           // 1 / cell size along x (a power of two): cells may be shorter in x, the
                         // axis a grid row runs along, so rows scanned stay few and short
  int32_t dims[3];       // bounding box of the occupied cells
  int32_t n_cells;       // dense: dims product; sparse: occupied chunks
  int64_t n_points;
  int32_t sparse;        // 0: dense cell_start over the box; 1: hashed chunks of kChunkX cells in x
  uint32_t hmask;        // sparse: hash table size - 1
};

// Sparse grids: a row of cells (fixed y, z) is split into chunks of kChunkX cells along x; each
// occupied chunk stores kChunkX + 1 point offsets and is found through an open-addressing hash of
// its (z, y, x / kChunkX) key.  A kNN row range spans at most 2 chunks (<= 2 * 8 + 1 cells).
constexpr int kChunkX = 16;
// A map point that can be a kNN candidate (KdTreeFLANN drops non-finite points).
__host__ __device__ inline bool map_point_finite(const float4& p) {
  return fabsf(p.x) <= 3.402823466e38f && fabsf(p.y) <= 3.402823466e38f && fabsf(p.z) <= 3.402823466e38f;
}
constexpr unsigned long long kChunkEmpty = ~0ull;
__host__ __device__ inline unsigned long long chunk_key(int z, int y, int xc) {
  return ((unsigned long long)(unsigned)z << 48) | ((unsigned long long)(unsigned)y << 24) | (unsigned long long)(unsigned)xc;
}
__host__ __device__ inline uint32_t chunk_hash(unsigned long long k) {
  return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 32);
}

}  // namespace fbr
