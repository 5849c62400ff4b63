// fbr_oracle.cpp — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library, and only
// as the checker / the timed CPU baseline.  The product path (feature_base_pointcloud_registration_amd)
// never links or calls it.
//
// PARITY STATUS: "parity unpinned" against reference outputs.  The reference
// (/root/reference, ROS1 + PCL + OpenCV + Eigen + FLANN + GTSAM) cannot be built in this image and
// ships no tests, fixtures or golden vectors.  What IS pinned:
//   * glibc atan2f/sqrtf and libstdc++ 11 std::sort are the reference's real dependencies and are
//     called directly here (same glibc 2.35 / libstdc++ 11 as the reference's Ubuntu toolchains);
//   * everything else restates the reference source line by line (cited below) and the
//     third-party algorithms it calls (PCL VoxelGrid/CropBox/getTransformation/KdTreeFLANN,
//     OpenCV cv::eigen Jacobi / cv::solve QR / Mat::inv LU / gemm, Eigen ColPivHouseholderQR),
//     restated from their published algorithms with sequential (non-SIMD) summation order.
//
// Build: oracle/Makefile (g++ -O2 -fopenmp -ffp-contract=off).  No FMA contraction: the
// reference is plain x86-64 code with no FMA instructions.
#include "../include/fbr.h"

#include <omp.h>

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace orc {

using P4 = fbr_point_xyzi;

// x86-64 cvttsd2si semantics for the reference's double->int conversions (NaN / out of range give
// INT_MIN, which the reference's bounds checks then reject).
static inline int x86_cvt(double v) {
  if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
  return (int)v;
}

// =============================================================================================
// Pose conversions: pcl::getTransformation / pcl::getTranslationAndEulerAngles (PCL common/eigen)
// =============================================================================================
struct Affine {
  float m[3][4];
};

static Affine get_transformation(float x, float y, float z, float roll, float pitch, float yaw) {
  float A = std::cos(yaw), B = std::sin(yaw), C = std::cos(pitch), D = std::sin(pitch),
        E = std::cos(roll), F = std::sin(roll), DE = D * E, DF = D * F;
  Affine t;
  t.m[0][0] = A * C; t.m[0][1] = A * DF - B * E; t.m[0][2] = B * F + A * DE; t.m[0][3] = x;
  t.m[1][0] = B * C; t.m[1][1] = A * E + B * DF; t.m[1][2] = B * DE - A * F; t.m[1][3] = y;
  t.m[2][0] = -D;    t.m[2][1] = C * F;          t.m[2][2] = C * E;          t.m[2][3] = z;
  return t;
}

static void get_translation_euler(const Affine& t, float pose[6]) {
  pose[3] = t.m[0][3];
  pose[4] = t.m[1][3];
  pose[5] = t.m[2][3];
  pose[0] = std::atan2(t.m[2][1], t.m[2][2]);
  pose[1] = std::asin(-t.m[2][0]);
  pose[2] = std::atan2(t.m[1][0], t.m[0][0]);
}

// trans2Affine3f (mapOptmization.h:444-448)
static Affine trans2affine(const float tr[6]) { return get_transformation(tr[3], tr[4], tr[5], tr[0], tr[1], tr[2]); }

// pointAssociateToMap (mapOptmization.h:397-403)
static inline P4 associate(const Affine& T, const P4& p) {
  P4 o;
  o.x = T.m[0][0] * p.x + T.m[0][1] * p.y + T.m[0][2] * p.z + T.m[0][3];
  o.y = T.m[1][0] * p.x + T.m[1][1] * p.y + T.m[1][2] * p.z + T.m[1][3];
  o.z = T.m[2][0] * p.x + T.m[2][1] * p.y + T.m[2][2] * p.z + T.m[2][3];
  o.intensity = p.intensity;
  return o;
}


// =============================================================================================
// A3: deskewPoint / findRotation / findPosition (imageProjection.cpp:494-580) on the table that
// imuDeskewInfo (:323-393) builds.  The reference never runs this: deskewInfo() is commented out
// at :189-191, so imuAvailable == 0 and deskewPoint returns the point (:548-549).  It is restated
// for the path with that call enabled.  Third-party pieces: pcl::
// getTransformation (float, glibc sinf/cosf), Eigen 3.3 Affine3f::inverse (3x3 cofactor inverse,
// InverseImpl.h) and Affine3f * Affine3f (linear * linear, linear * t + t); Eigen's fixed-size
// 3-term sums reduce as x0 + (x1 + x2) (redux_novec_unroller).
// =============================================================================================
static void find_rotation(const fbr_deskew_table& T, double pointTime, float* rotXCur, float* rotYCur,
                          float* rotZCur) {  // :494-526
  *rotXCur = 0;
  *rotYCur = 0;
  *rotZCur = 0;
  int imuPointerFront = 0;
  while (imuPointerFront < T.imu_pointer_cur) {
    if (pointTime < T.imu_time[imuPointerFront]) break;
    ++imuPointerFront;
  }
  if (pointTime > T.imu_time[imuPointerFront] || imuPointerFront == 0) {
    *rotXCur = T.imu_rot_x[imuPointerFront];
    *rotYCur = T.imu_rot_y[imuPointerFront];
    *rotZCur = T.imu_rot_z[imuPointerFront];
  } else {
    int imuPointerBack = imuPointerFront - 1;
    double ratioFront = (pointTime - T.imu_time[imuPointerBack]) / (T.imu_time[imuPointerFront] - T.imu_time[imuPointerBack]);
    double ratioBack = (T.imu_time[imuPointerFront] - pointTime) / (T.imu_time[imuPointerFront] - T.imu_time[imuPointerBack]);
    *rotXCur = T.imu_rot_x[imuPointerFront] * ratioFront + T.imu_rot_x[imuPointerBack] * ratioBack;
    *rotYCur = T.imu_rot_y[imuPointerFront] * ratioFront + T.imu_rot_y[imuPointerBack] * ratioBack;
    *rotZCur = T.imu_rot_z[imuPointerFront] * ratioFront + T.imu_rot_z[imuPointerBack] * ratioBack;
  }
}

static inline float eig_sum3(float a, float b, float c) { return a + (b + c); }

static Affine eigen_affine_inverse(const Affine& a) {  // Transform<float,3,Affine>::inverse()
  auto cof = [&](int i, int j) {  // cofactor_3x3<i,j>
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return a.m[i1][j1] * a.m[i2][j2] - a.m[i1][j2] * a.m[i2][j1];
  };
  const float c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
  const float det = eig_sum3(c0 * a.m[0][0], c1 * a.m[1][0], c2 * a.m[2][0]);
  const float invdet = 1.0f / det;
  Affine r;
  r.m[0][0] = c0 * invdet;
  r.m[0][1] = c1 * invdet;
  r.m[0][2] = c2 * invdet;
  r.m[1][0] = cof(0, 1) * invdet;
  r.m[1][1] = cof(1, 1) * invdet;
  r.m[1][2] = cof(2, 1) * invdet;
  r.m[2][0] = cof(0, 2) * invdet;
  r.m[2][1] = cof(1, 2) * invdet;
  r.m[2][2] = cof(2, 2) * invdet;
  for (int i = 0; i < 3; ++i)  // (-L^-1) * t
    r.m[i][3] = eig_sum3(-r.m[i][0] * a.m[0][3], -r.m[i][1] * a.m[1][3], -r.m[i][2] * a.m[2][3]);
  return r;
}

static Affine eigen_affine_mul(const Affine& l, const Affine& r) {  // Affine3f * Affine3f
  Affine o;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) o.m[i][j] = eig_sum3(l.m[i][0] * r.m[0][j], l.m[i][1] * r.m[1][j], l.m[i][2] * r.m[2][j]);
    o.m[i][3] = eig_sum3(l.m[i][0] * r.m[0][3], l.m[i][1] * r.m[1][3], l.m[i][2] * r.m[2][3]) + l.m[i][3];
  }
  return o;
}

struct Deskewer {  // deskewPoint (:545-580) with its per-scan firstPointFlag / transStartInverse
  const fbr_deskew_table* T;
  bool firstPointFlag = true;
  Affine transStartInverse;
  P4 operator()(const P4& point, double relTime) {
    double pointTime = T->time_scan_cur + relTime;
    float rotXCur, rotYCur, rotZCur;
    find_rotation(*T, pointTime, &rotXCur, &rotYCur, &rotZCur);
    float posXCur = 0, posYCur = 0, posZCur = 0;  // findPosition (:528-542): positional deskew commented out
    if (firstPointFlag) {
      transStartInverse = eigen_affine_inverse(get_transformation(posXCur, posYCur, posZCur, rotXCur, rotYCur, rotZCur));
      firstPointFlag = false;
    }
    Affine transFinal = get_transformation(posXCur, posYCur, posZCur, rotXCur, rotYCur, rotZCur);
    Affine transBt = eigen_affine_mul(transStartInverse, transFinal);
    P4 newPoint;
    newPoint.x = transBt.m[0][0] * point.x + transBt.m[0][1] * point.y + transBt.m[0][2] * point.z + transBt.m[0][3];
    newPoint.y = transBt.m[1][0] * point.x + transBt.m[1][1] * point.y + transBt.m[1][2] * point.z + transBt.m[1][3];
    newPoint.z = transBt.m[2][0] * point.x + transBt.m[2][1] * point.y + transBt.m[2][2] * point.z + transBt.m[2][3];
    newPoint.intensity = point.intensity;
    return newPoint;
  }
};

// ---- tf LinearMath (tfScalar = double): Quaternion::setRPY / slerp, Matrix3x3::getRPY ----
struct TfQuaternion {
  double x, y, z, w;
};
static TfQuaternion tf_setRPY(double roll, double pitch, double yaw) {
  double halfYaw = yaw * 0.5, halfPitch = pitch * 0.5, halfRoll = roll * 0.5;
  double cosYaw = std::cos(halfYaw), sinYaw = std::sin(halfYaw);
  double cosPitch = std::cos(halfPitch), sinPitch = std::sin(halfPitch);
  double cosRoll = std::cos(halfRoll), sinRoll = std::sin(halfRoll);
  return TfQuaternion{sinRoll * cosPitch * cosYaw - cosRoll * sinPitch * sinYaw,
                      cosRoll * sinPitch * cosYaw + sinRoll * cosPitch * sinYaw,
                      cosRoll * cosPitch * sinYaw - sinRoll * sinPitch * cosYaw,
                      cosRoll * cosPitch * cosYaw + sinRoll * sinPitch * sinYaw};
}
static double tf_dot(const TfQuaternion& a, const TfQuaternion& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
static double tfAcos(double x) { return std::acos(x < -1 ? -1 : (x > 1 ? 1 : x)); }
static double tfAsin(double x) { return std::asin(x < -1 ? -1 : (x > 1 ? 1 : x)); }
static TfQuaternion tf_slerp(const TfQuaternion& a, const TfQuaternion& q, double t) {
  double s = std::sqrt(tf_dot(a, a) * tf_dot(q, q));  // angleShortestPath
  double angle = tf_dot(a, q) < 0 ? tfAcos(tf_dot(a, TfQuaternion{-q.x, -q.y, -q.z, -q.w}) / s) * 2.0
                                  : tfAcos(tf_dot(a, q) / s) * 2.0;
  double theta = angle / 2.0;
  if (theta == 0.0) return a;
  double d = 1.0 / std::sin(theta), s0 = std::sin((1.0 - t) * theta), s1 = std::sin(t * theta);
  if (tf_dot(a, q) < 0)
    return TfQuaternion{(a.x * s0 + -q.x * s1) * d, (a.y * s0 + -q.y * s1) * d, (a.z * s0 + -q.z * s1) * d,
                        (a.w * s0 + -q.w * s1) * d};
  return TfQuaternion{(a.x * s0 + q.x * s1) * d, (a.y * s0 + q.y * s1) * d, (a.z * s0 + q.z * s1) * d,
                      (a.w * s0 + q.w * s1) * d};
}
static void tf_getRPY(const TfQuaternion& q, double& roll, double& pitch, double& yaw) {
  double d = tf_dot(q, q), s = 2.0 / d;  // Matrix3x3::setRotation
  double xs = q.x * s, ys = q.y * s, zs = q.z * s;
  double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
  double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
  double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
  double el[3][3] = {{1.0 - (yy + zz), xy - wz, xz + wy}, {xy + wz, 1.0 - (xx + zz), yz - wx}, {xz - wy, yz + wx, 1.0 - (xx + yy)}};
  if (std::fabs(el[2][0]) >= 1) {  // getEulerYPR, solution 1
    yaw = 0;
    pitch = el[2][0] < 0 ? M_PI / 2.0 : -M_PI / 2.0;
    roll = std::atan2(el[2][1], el[2][2]);
  } else {
    pitch = -tfAsin(el[2][0]);
    roll = std::atan2(el[2][1] / std::cos(pitch), el[2][2] / std::cos(pitch));
    yaw = std::atan2(el[1][0] / std::cos(pitch), el[0][0] / std::cos(pitch));
  }
}

// =============================================================================================
// A2 + A4: ImageProjection::projectPointCloud + cloudExtraction (imageProjection.cpp:583-670)
// =============================================================================================
struct Projection {
  std::vector<int32_t> start, end, col;
  std::vector<float> range;
  std::vector<P4> cloud;
};

static void project(const fbr_params& P, const fbr_point_xyzirt* pts, int64_t n_in, Projection& out,
                    const fbr_deskew_table* T = nullptr) {
  const int H = P.n_scan, W = P.horizon_scan;
  const bool deskew = T && T->imu_available;  // deskewPoint (:548): deskewFlag != -1 is the caller's
  Deskewer deskewPoint{T};
  std::vector<float> rangeMat((size_t)H * W, FLT_MAX);  // :130
  std::vector<P4> full((size_t)H * W);                   // :114
  for (int64_t i = 0; i < n_in; ++i) {
    const fbr_point_xyzirt& q = pts[i];
    int rowIdn = q.ring;                                 // :598
    if (rowIdn < 0 || rowIdn >= H) continue;             // :599
    // :605  atan2(float,float) -> glibc atan2f; *180 in float; / M_PI in double; stored float
    float horizonAngle = (float)((double)(atan2f(q.x, q.y) * 180.0f) / M_PI);
    float ang_res_x = (float)(360.0 / (double)(float)W);                                // :608
    int columnIdn = x86_cvt(-std::round(((double)horizonAngle - 90.0) / (double)ang_res_x) +
                            (double)(W / 2));                                          // :611
    if (columnIdn >= W) columnIdn -= W;                                                // :612
    if (columnIdn < 0 || columnIdn >= W) continue;                                     // :615
    float range = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);                            // utility.h:308
    if (range < 1.0) continue;                                                         // :620
    size_t c = (size_t)rowIdn * W + columnIdn;
    if (rangeMat[c] != FLT_MAX) continue;                                              // :623
    rangeMat[c] = range;                                                               // :633
    P4 thisPoint{q.x, q.y, q.z, q.intensity};
    if (deskew) thisPoint = deskewPoint(thisPoint, q.time);                           // :635
    full[c] = thisPoint;  // without a table deskewPoint is the identity (imuAvailable == 0, :548)
  }
  out.start.assign(H, 0);
  out.end.assign(H, 0);
  out.col.clear();
  out.range.clear();
  out.cloud.clear();
  int count = 0;
  for (int i = 0; i < H; ++i) {
    out.start[i] = count - 1 + 5;                                                      // :650
    for (int j = 0; j < W; ++j) {
      float r = rangeMat[(size_t)i * W + j];
      if (r != FLT_MAX) {                                                              // :656
        out.col.push_back(j);
        out.range.push_back(r);
        out.cloud.push_back(full[(size_t)j + (size_t)i * W]);
        ++count;
      }
    }
    out.end[i] = count - 1 - 5;                                                        // :668
  }
}

// =============================================================================================
// A9: pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.8, downsample_all_data_ = true)
// =============================================================================================
struct cloud_point_index_idx {  // pcl/filters/voxel_grid.h
  unsigned int idx;
  unsigned int cloud_point_index;
  bool operator<(const cloud_point_index_idx& p) const { return idx < p.idx; }
};

static void voxel_grid(const P4* in, int64_t n, float leaf, std::vector<P4>& out) {
  out.clear();
  if (n <= 0) return;
  // a cloud with a non-finite point is not dense: applyFilter and getMinMax3D then skip those points
  // (voxel_grid.cpp, `if (!input_->is_dense) ... if (!pcl_isfinite(...)) continue;`), which is the
  // dense path over the finite points (cloud_point_index renumbered, the same key sequence)
  for (int64_t i = 0; i < n; ++i)
    if (!(std::isfinite(in[i].x) && std::isfinite(in[i].y) && std::isfinite(in[i].z))) {
      std::vector<P4> fin;
      fin.reserve(n);
      for (int64_t j = 0; j < n; ++j)
        if (std::isfinite(in[j].x) && std::isfinite(in[j].y) && std::isfinite(in[j].z)) fin.push_back(in[j]);
      voxel_grid(fin.data(), (int64_t)fin.size(), leaf, out);
      return;
    }
  const float inv = 1.0f / leaf;  // inverse_leaf_size_ = Ones / leaf_size_ (float)
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = 0; i < n; ++i) {  // getMinMax3D (dense cloud)
    const float v[3] = {in[i].x, in[i].y, in[i].z};
    for (int d = 0; d < 3; ++d) {
      mn[d] = std::min(mn[d], v[d]);
      mx[d] = std::max(mx[d], v[d]);
    }
  }
  int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
  int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
  int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)INT32_MAX) {  // "Leaf size is too small": output = input
    out.assign(in, in + n);
    return;
  }
  int min_b[3], max_b[3], div_b[3];
  for (int d = 0; d < 3; ++d) {
    min_b[d] = (int)std::floor(mn[d] * inv);
    max_b[d] = (int)std::floor(mx[d] * inv);
    div_b[d] = max_b[d] - min_b[d] + 1;
  }
  const int divb_mul[3] = {1, div_b[0], div_b[0] * div_b[1]};
  std::vector<cloud_point_index_idx> iv;
  iv.reserve(n);
  for (int64_t i = 0; i < n; ++i) {
    int ijk0 = (int)(std::floor(in[i].x * inv) - (float)min_b[0]);
    int ijk1 = (int)(std::floor(in[i].y * inv) - (float)min_b[1]);
    int ijk2 = (int)(std::floor(in[i].z * inv) - (float)min_b[2]);
    int idx = ijk0 * divb_mul[0] + ijk1 * divb_mul[1] + ijk2 * divb_mul[2];
    iv.push_back(cloud_point_index_idx{(unsigned)idx, (unsigned)i});
  }
  // unstable, libstdc++ (ORC_VG_STABLE=1, diagnostics only: std::stable_sort, the index order)
  static const bool stable_diag = std::getenv("ORC_VG_STABLE") && std::atoi(std::getenv("ORC_VG_STABLE")) != 0;
  if (stable_diag) std::stable_sort(iv.begin(), iv.end(), std::less<cloud_point_index_idx>());
  else std::sort(iv.begin(), iv.end(), std::less<cloud_point_index_idx>());
  size_t index = 0;
  while (index < iv.size()) {
    size_t i = index + 1;
    while (i < iv.size() && iv[i].idx == iv[index].idx) ++i;
    const P4& f = in[iv[index].cloud_point_index];
    float c[4] = {f.x, f.y, f.z, f.intensity};
    for (size_t li = index + 1; li < i; ++li) {
      const P4& p = in[iv[li].cloud_point_index];
      c[0] += p.x;
      c[1] += p.y;
      c[2] += p.z;
      c[3] += p.intensity;
    }
    const float cnt = (float)(i - index);
    out.push_back(P4{c[0] / cnt, c[1] / cnt, c[2] / cnt, c[3] / cnt});
    index = i;
  }
}

// =============================================================================================
// A6-A8: FeatureExtraction (featureExtraction.h:64-294) with its persistent scratch state
// =============================================================================================
struct smoothness_t {  // featureExtraction.h:8-11
  float value;
  size_t ind;
};
struct by_value {  // featureExtraction.h:13-17
  bool operator()(smoothness_t const& l, smoothness_t const& r) const { return l.value < r.value; }
};

// Persistent members of FeatureExtraction plus the cloud_info vectors it indexes.  Choices for
// state the reference leaves undefined:
//   - uninitialised new[] scratch (cloudCurvature/NeighborPicked/Label, :74-76) starts at 0;
//   - pointColInd[-1] = 0 and pointColInd[-2] = a large value (glibc chunk header on x86-64);
//   - the write to cloudNeighborPicked[-1] lands in a scratch slot.
struct FeatState {
  int H = 0, W = 0;
  size_t N = 0;
  std::vector<smoothness_t> smooth;  // resize(N): value-initialised {0, 0}   (:66)
  std::vector<float> curv;
  std::vector<int> picked_buf, label;
  std::vector<int32_t> col_buf;
  std::vector<float> range;
  int* picked = nullptr;
  int32_t* col = nullptr;
  static constexpr int kPad = 2;
  static constexpr int32_t kColM2 = 1 << 30;
  void init(int H_, int W_) {
    H = H_;
    W = W_;
    N = (size_t)H * W;
    smooth.assign(N, smoothness_t{0.0f, 0});
    curv.assign(N, 0.0f);
    picked_buf.assign(N + kPad, 0);
    label.assign(N, 0);
    col_buf.assign(N + kPad, 0);
    range.assign(N, 0.0f);
    picked = picked_buf.data() + kPad;
    col = col_buf.data() + kPad;
    col[-2] = kColM2;
    col[-1] = 0;
  }
};

struct Features {
  std::vector<P4> corner, surf;
};

static void extract_features(const fbr_params& P, FeatState& S, const Projection& pr, Features& F) {
  const int n = (int)pr.col.size();
  // cloudInfo = msgIn (:90): the pointColInd / pointRange vectors are sized N_SCAN*Horizon_SCAN
  // (imageProjection.cpp:119-120); entries past n keep earlier scans' values.
  for (int i = 0; i < n; ++i) {
    S.col[i] = pr.col[i];
    S.range[i] = pr.range[i];
  }
  const float* r = S.range.data();
  // ---- calculateSmoothness (:109-131) ----
  for (int i = 5; i < n - 5; i++) {
    float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 + r[i + 1] +
                      r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
    S.curv[i] = diffRange * diffRange;
    S.picked[i] = 0;
    S.label[i] = 0;
    S.smooth[i].value = S.curv[i];
    S.smooth[i].ind = i;
  }
  // ---- markOccludedPoints (:134-176) ----
  for (int i = 5; i < n - 6; ++i) {
    float depth1 = r[i];
    float depth2 = r[i + 1];
    int columnDiff = std::abs(int(S.col[i + 1] - S.col[i]));
    if (columnDiff < 10) {
      if (depth1 - depth2 > 0.3) {
        for (int l = 0; l <= 5; ++l) S.picked[i - l] = 1;
      } else if (depth2 - depth1 > 0.3) {
        for (int l = 1; l <= 6; ++l) S.picked[i + l] = 1;
      }
    }
    float diff1 = std::abs(float(r[i - 1] - r[i]));
    float diff2 = std::abs(float(r[i + 1] - r[i]));
    if (diff1 > 0.02 * r[i] && diff2 > 0.02 * r[i]) S.picked[i] = 1;
  }
  // ---- extractFeatures (:178-294) ----
  F.corner.clear();
  F.surf.clear();
  std::vector<P4> surfScan, surfScanDS;
  const std::vector<P4>& cloud = pr.cloud;
  auto suppress = [&](int ind) {
    for (int l = 1; l <= 5; l++) {
      int columnDiff = std::abs(int(S.col[ind + l] - S.col[ind + l - 1]));
      if (columnDiff > 10) break;
      S.picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      int columnDiff = std::abs(int(S.col[ind + l] - S.col[ind + l + 1]));
      if (columnDiff > 10) break;
      S.picked[ind + l] = 1;  // ind+l == -1 only for the stale entry: scratch slot
    }
  };
  for (int i = 0; i < P.n_scan; i++) {
    surfScan.clear();
    for (int j = 0; j < 6; j++) {
      int sp = (pr.start[i] * (6 - j) + pr.end[i] * j) / 6;
      int ep = (pr.start[i] * (5 - j) + pr.end[i] * (j + 1)) / 6 - 1;
      if (sp >= ep) continue;
      std::sort(S.smooth.begin() + sp, S.smooth.begin() + ep, by_value());  // ep excluded (:203)
      int largestPickedNum = 0;
      for (int k = ep; k >= sp; k--) {
        int ind = (int)S.smooth[k].ind;
        if (S.picked[ind] == 0 && S.curv[ind] > P.edge_threshold) {
          largestPickedNum++;
          if (largestPickedNum <= 20) {
            S.label[ind] = 1;
            F.corner.push_back(cloud[ind]);
          } else {
            break;
          }
          S.picked[ind] = 1;
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++) {
        int ind = (int)S.smooth[k].ind;
        if (S.picked[ind] == 0 && S.curv[ind] < P.surf_threshold) {
          S.label[ind] = -1;
          S.picked[ind] = 1;
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++) {
        if (S.label[k] <= 0) surfScan.push_back(cloud[k]);
      }
    }
    voxel_grid(surfScan.data(), (int64_t)surfScan.size(), P.odometry_surf_leaf_size, surfScanDS);
    F.surf.insert(F.surf.end(), surfScanDS.begin(), surfScanDS.end());
  }
}

// =============================================================================================
// KdTreeFLANN<PointXYZI>::nearestKSearch(k=5): exact kNN over xyz, L2_Simple float distance
// ((0 + dx*dx) + dy*dy) + dz*dz, results ascending.  Restated as a single-index KD-tree with
// leaf size 15 (PCL's KDTreeSingleIndexParams(15)); equal distances are ordered by point index
// (FLANN's own tie order is traversal dependent; the synthetic inputs avoid exact ties).
// =============================================================================================
struct KDTree {
  struct Node {
    int lo, hi;  // [lo,hi) into perm for leaves
    int left, right;
    int dim;
    float split;
  };
  const P4* pts = nullptr;
  int n = 0;
  std::vector<int> perm;
  std::vector<Node> nodes;

  static inline float coord(const P4& p, int d) { return d == 0 ? p.x : (d == 1 ? p.y : p.z); }

  int build_rec(int lo, int hi) {
    Node nd{lo, hi, -1, -1, -1, 0.0f};
    int id = (int)nodes.size();
    nodes.push_back(nd);
    if (hi - lo <= 15) return id;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = lo; i < hi; ++i)
      for (int d = 0; d < 3; ++d) {
        float c = coord(pts[perm[i]], d);
        mn[d] = std::min(mn[d], c);
        mx[d] = std::max(mx[d], c);
      }
    int dim = 0;
    for (int d = 1; d < 3; ++d)
      if (mx[d] - mn[d] > mx[dim] - mn[dim]) dim = d;
    int mid = (lo + hi) / 2;
    std::nth_element(perm.begin() + lo, perm.begin() + mid, perm.begin() + hi,
                     [&](int a, int b) { return coord(pts[a], dim) < coord(pts[b], dim); });
    float split = coord(pts[perm[mid]], dim);
    int l = build_rec(lo, mid);
    int r = build_rec(mid, hi);
    nodes[id].left = l;
    nodes[id].right = r;
    nodes[id].dim = dim;
    nodes[id].split = split;
    return id;
  }

  void build(const P4* p, int count) {
    pts = p;
    n = count;
    perm.resize(n);
    for (int i = 0; i < n; ++i) perm[i] = i;
    nodes.clear();
    nodes.reserve(2 * (n / 8 + 1));
    if (n > 0) build_rec(0, n);
  }

  struct Res {
    float d[5];
    int i[5];
    int cnt;
  };

  static inline bool better(float d, int i, float d2, int i2) { return d < d2 || (d == d2 && i < i2); }

  void insert(Res& r, float d, int idx) const {
    if (r.cnt == 5 && !better(d, idx, r.d[4], r.i[4])) return;
    int k = r.cnt < 5 ? r.cnt++ : 4;
    while (k > 0 && better(d, idx, r.d[k - 1], r.i[k - 1])) {
      r.d[k] = r.d[k - 1];
      r.i[k] = r.i[k - 1];
      --k;
    }
    r.d[k] = d;
    r.i[k] = idx;
  }

  void search_rec(int id, const float q[3], Res& r) const {
    const Node& nd = nodes[id];
    if (nd.left < 0) {
      for (int t = nd.lo; t < nd.hi; ++t) {
        const P4& p = pts[perm[t]];
        float dist = 0.0f;
        float diff = q[0] - p.x;
        dist += diff * diff;
        diff = q[1] - p.y;
        dist += diff * diff;
        diff = q[2] - p.z;
        dist += diff * diff;
        insert(r, dist, perm[t]);
      }
      return;
    }
    float diff = q[nd.dim] - nd.split;
    int first = diff < 0 ? nd.left : nd.right;
    int second = diff < 0 ? nd.right : nd.left;
    search_rec(first, q, r);
    if (r.cnt < 5 || diff * diff <= r.d[4]) search_rec(second, q, r);
  }

  Res knn5(const P4& q) const {
    Res r;
    r.cnt = 0;
    if (n == 0) return r;
    float qq[3] = {q.x, q.y, q.z};
    search_rec(0, qq, r);
    return r;
  }
};

// =============================================================================================
// OpenCV / Eigen small dense solvers (float), restated from the published algorithms.
// =============================================================================================
static inline float cv_hypot(float a, float b) {  // modules/core/src/lapack.cpp
  a = std::abs(a);
  b = std::abs(b);
  if (a > b) {
    b /= a;
    return a * std::sqrt(1 + b * b);
  }
  if (b > 0) {
    a /= b;
    return b * std::sqrt(1 + a * a);
  }
  return 0;
}

// cv::eigen(src, evals, evects) for a symmetric CV_32F matrix: JacobiImpl_ (lapack.cpp).
// A is n x n row-major (destroyed); W eigenvalues descending; V rows are eigenvectors.
static void cv_jacobi(float* A, int n, float* W, float* V) {
  const float eps = FLT_EPSILON;
  int indR[8], indC[8];
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) V[i * n + j] = 0.0f;
    V[i * n + i] = 1.0f;
  }
  int iters, maxIters = n * n * 30;
  float mv = 0.0f;
  for (int k = 0; k < n; k++) {
    W[k] = A[(n + 1) * k];
    if (k < n - 1) {
      int m = k + 1, i;
      for (mv = std::abs(A[n * k + m]), i = k + 2; i < n; i++) {
        float val = std::abs(A[n * k + i]);
        if (mv < val) mv = val, m = i;
      }
      indR[k] = m;
    }
    if (k > 0) {
      int m = 0, i;
      for (mv = std::abs(A[k]), i = 1; i < k; i++) {
        float val = std::abs(A[n * i + k]);
        if (mv < val) mv = val, m = i;
      }
      indC[k] = m;
    }
  }
  if (n > 1)
    for (iters = 0; iters < maxIters; iters++) {
      int k = 0, i;
      for (mv = std::abs(A[indR[0]]), i = 1; i < n - 1; i++) {
        float val = std::abs(A[n * i + indR[i]]);
        if (mv < val) mv = val, k = i;
      }
      int l = indR[k];
      for (i = 1; i < n; i++) {
        float val = std::abs(A[n * indC[i] + i]);
        if (mv < val) mv = val, k = indC[i], l = i;
      }
      float p = A[n * k + l];
      if (std::abs(p) <= eps) break;
      float y = (float)((W[l] - W[k]) * 0.5);
      float t = std::abs(y) + cv_hypot(p, y);
      float s = cv_hypot(p, t);
      float c = t / s;
      s = p / s;
      t = (p / t) * p;
      if (y < 0) s = -s, t = -t;
      A[n * k + l] = 0;
      W[k] -= t;
      W[l] += t;
      float a0, b0;
#define ORC_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
      for (i = 0; i < k; i++) ORC_ROT(A[n * i + k], A[n * i + l]);
      for (i = k + 1; i < l; i++) ORC_ROT(A[n * k + i], A[n * i + l]);
      for (i = l + 1; i < n; i++) ORC_ROT(A[n * k + i], A[n * l + i]);
      for (i = 0; i < n; i++) ORC_ROT(V[n * k + i], V[n * l + i]);
#undef ORC_ROT
      for (int j = 0; j < 2; j++) {
        int idx = j == 0 ? k : l;
        if (idx < n - 1) {
          int m = idx + 1;
          for (mv = std::abs(A[n * idx + m]), i = idx + 2; i < n; i++) {
            float val = std::abs(A[n * idx + i]);
            if (mv < val) mv = val, m = i;
          }
          indR[idx] = m;
        }
        if (idx > 0) {
          int m = 0;
          for (mv = std::abs(A[idx]), i = 1; i < idx; i++) {
            float val = std::abs(A[n * i + idx]);
            if (mv < val) mv = val, m = i;
          }
          indC[idx] = m;
        }
      }
    }
  for (int k = 0; k < n - 1; k++) {
    int m = k;
    for (int i = k + 1; i < n; i++)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      std::swap(W[m], W[k]);
      for (int i = 0; i < n; i++) std::swap(V[n * m + i], V[n * k + i]);
    }
  }
}

// cv::solve(A, b, x, DECOMP_QR) for square CV_32F: hal::QR32f -> QRImpl (Householder), eps =
// FLT_EPSILON*10.  A (n x n row-major) destroyed; b (n) overwritten with x.  Returns 0 if singular
// (cv::solve then sets x = 0).
static int cv_qr_solve(float* A, int n, float* b) {
  const float eps = FLT_EPSILON * 10;
  float vl[8], hFactors[8];
  const int m = n;
  for (int l = 0; l < n; l++) {
    int vlSize = m - l;
    float vlNorm = 0.0f;
    for (int i = 0; i < vlSize; i++) {
      vl[i] = A[(l + i) * n + l];
      vlNorm += vl[i] * vl[i];
    }
    float tmpV = vl[0];
    vl[0] = vl[0] + (vl[0] >= 0 ? 1.0f : -1.0f) * std::sqrt(vlNorm);
    vlNorm = std::sqrt(vlNorm + vl[0] * vl[0] - tmpV * tmpV);
    for (int i = 0; i < vlSize; i++) vl[i] /= vlNorm;
    for (int j = l; j < n; j++) {
      float v_lA = 0.0f;
      for (int i = l; i < m; i++) v_lA += vl[i - l] * A[i * n + j];
      for (int i = l; i < m; i++) A[i * n + j] -= 2 * vl[i - l] * v_lA;
    }
    hFactors[l] = vl[0] * vl[0];
    for (int i = 1; i < vlSize; i++) A[(l + i) * n + l] = vl[i] / vl[0];
  }
  for (int l = 0; l < n; l++) {
    vl[0] = 1.0f;
    for (int j = 1; j < m - l; j++) vl[j] = A[(j + l) * n + l];
    float v_lB = 0.0f;
    for (int i = l; i < m; i++) v_lB += vl[i - l] * b[i];
    for (int i = l; i < m; i++) b[i] -= 2 * vl[i - l] * v_lB * hFactors[l];
  }
  for (int i = n - 1; i >= 0; i--) {
    for (int j = n - 1; j > i; j--) b[i] -= b[j] * A[i * n + j];
    if (std::abs(A[i * n + i]) < eps) return 0;
    b[i] /= A[i * n + i];
  }
  return 1;
}

// Mat::inv() (DECOMP_LU) for CV_32F n > 3: LUImpl with partial pivoting, eps = FLT_EPSILON*10.
static int cv_lu_inv(const float* Ain, int n, float* Binv) {
  const float eps = FLT_EPSILON * 10;
  float A[64];
  std::memcpy(A, Ain, sizeof(float) * n * n);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) Binv[i * n + j] = (i == j) ? 1.0f : 0.0f;
  for (int i = 0; i < n; i++) {
    int k = i;
    for (int j = i + 1; j < n; j++)
      if (std::abs(A[j * n + i]) > std::abs(A[k * n + i])) k = j;
    if (std::abs(A[k * n + i]) < eps) return 0;
    if (k != i) {
      for (int j = i; j < n; j++) std::swap(A[i * n + j], A[k * n + j]);
      for (int j = 0; j < n; j++) std::swap(Binv[i * n + j], Binv[k * n + j]);
    }
    float d = -1 / A[i * n + i];
    for (int j = i + 1; j < n; j++) {
      float alpha = A[j * n + i] * d;
      for (int c = i + 1; c < n; c++) A[j * n + c] += alpha * A[i * n + c];
      for (int c = 0; c < n; c++) Binv[j * n + c] += alpha * Binv[i * n + c];
    }
  }
  for (int i = n - 1; i >= 0; i--)
    for (int j = 0; j < n; j++) {
      float s = Binv[i * n + j];
      for (int c = i + 1; c < n; c++) s -= A[i * n + c] * Binv[c * n + j];
      Binv[i * n + j] = s / A[i * n + i];
    }
  return 1;
}

// OpenCV gemm for CV_32F accumulates in double (GEMMSingleMul<float,double>), stores float.
static void cv_gemm(const float* A, const float* B, float* C, int M, int K, int N) {
  for (int i = 0; i < M; i++)
    for (int j = 0; j < N; j++) {
      double s = 0.0;
      for (int k = 0; k < K; k++) s += (double)A[i * K + k] * (double)B[k * N + j];
      C[i * N + j] = (float)s;
    }
}

// Eigen::ColPivHouseholderQR<Matrix<float,5,3>>::compute + solve (Eigen 3.3 algorithm,
// sequential summation).  A 5x3 row-major, b 5; x 3.
static void eigen_colpiv_solve(const float Ain[5][3], const float bin[5], float x[3]) {
  const int rows = 5, cols = 3, size = 3;
  float qr[5][3];
  std::memcpy(qr, Ain, sizeof(qr));
  float hc[3], nUpd[3], nDir[3];
  int transp[3];
  auto colnorm = [&](int j, int r0) {
    float s = 0.0f;
    for (int i = r0; i < rows; i++) s += qr[i][j] * qr[i][j];
    return std::sqrt(s);
  };
  for (int k = 0; k < cols; ++k) {
    nDir[k] = colnorm(k, 0);
    nUpd[k] = nDir[k];
  }
  const float eps = FLT_EPSILON;
  float mxn = nUpd[0];
  for (int k = 1; k < cols; ++k)
    if (nUpd[k] > mxn) mxn = nUpd[k];
  float th = (mxn * eps) * (mxn * eps) / (float)rows;
  float ndt = std::sqrt(eps);
  int nz = size;
  for (int k = 0; k < size; ++k) {
    int big = k;
    float bv = nUpd[k];
    for (int j = k + 1; j < cols; ++j)
      if (nUpd[j] > bv) bv = nUpd[j], big = j;
    float bsq = bv * bv;
    if (nz == size && bsq < th * (float)(rows - k)) nz = k;
    transp[k] = big;
    if (k != big) {
      for (int i = 0; i < rows; ++i) std::swap(qr[i][k], qr[i][big]);
      std::swap(nUpd[k], nUpd[big]);
      std::swap(nDir[k], nDir[big]);
    }
    // makeHouseholderInPlace on qr[k..4][k]
    float tailSq = 0.0f;
    for (int i = k + 1; i < rows; ++i) tailSq += qr[i][k] * qr[i][k];
    float c0 = qr[k][k], beta, tau;
    if (tailSq <= FLT_MIN) {
      tau = 0.0f;
      beta = c0;
      for (int i = k + 1; i < rows; ++i) qr[i][k] = 0.0f;
    } else {
      beta = std::sqrt(c0 * c0 + tailSq);
      if (c0 >= 0.0f) beta = -beta;
      const float den = c0 - beta;
      for (int i = k + 1; i < rows; ++i) qr[i][k] = qr[i][k] / den;
      tau = (beta - c0) / beta;
    }
    hc[k] = tau;
    qr[k][k] = beta;
    // applyHouseholderOnTheLeft on qr[k..4][k+1..2]
    if (k + 1 < cols && tau != 0.0f) {
      for (int j = k + 1; j < cols; ++j) {
        float tmp = 0.0f;
        for (int i = k + 1; i < rows; ++i) tmp += qr[i][k] * qr[i][j];
        tmp += qr[k][j];
        qr[k][j] -= tau * tmp;
        for (int i = k + 1; i < rows; ++i) qr[i][j] -= tmp * (tau * qr[i][k]);
      }
    }
    for (int j = k + 1; j < cols; ++j) {
      if (nUpd[j] != 0.0f) {
        float temp = std::abs(qr[k][j]) / nUpd[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        float q = nUpd[j] / nDir[j];
        float temp2 = temp * (q * q);
        if (temp2 <= ndt) {
          nDir[j] = colnorm(j, k + 1);
          nUpd[j] = nDir[j];
        } else {
          nUpd[j] *= std::sqrt(temp);
        }
      }
    }
  }
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < size; ++k) std::swap(perm[k], perm[transp[k]]);
  if (nz == 0) {
    x[0] = x[1] = x[2] = 0.0f;
    return;
  }
  float c[5];
  std::memcpy(c, bin, sizeof(c));
  for (int k = 0; k < nz; ++k) {  // apply H_0 .. H_{nz-1}
    const float tau = hc[k];
    if (rows - k == 1) {
      c[k] *= 1.0f - tau;
    } else if (tau != 0.0f) {
      float tmp = 0.0f;
      for (int i = k + 1; i < rows; ++i) tmp += qr[i][k] * c[i];
      tmp += c[k];
      c[k] -= tau * tmp;
      for (int i = k + 1; i < rows; ++i) c[i] -= tmp * (tau * qr[i][k]);
    }
  }
  for (int i = nz - 1; i >= 0; --i) {  // triangular_solve_vector, Upper, column-major
    if (c[i] != 0.0f) {
      c[i] /= qr[i][i];
      for (int t = 0; t < i; ++t) c[t] -= c[i] * qr[t][i];
    }
  }
  for (int i = 0; i < nz; ++i) x[perm[i]] = c[i];
  for (int i = nz; i < cols; ++i) x[perm[i]] = 0.0f;
}

// =============================================================================================
// A10-A18: mapOptimization::registration (mapOptmization.h:263-343) and scan2MapOptimization
// =============================================================================================
struct Map {
  std::vector<P4> corner, surf;  // global maps after the start-up VoxelGrid (:251-257)
};

struct RegResult {
  fbr_reg_stats st;
  std::vector<float> trace;  // pose after each LM iteration
};

static void crop(const std::vector<P4>& in, const float mn[3], const float mx[3], std::vector<P4>& out) {
  out.clear();
  for (const P4& p : in) {  // pcl::CropBox::applyFilter, inclusive bounds
    if (p.x < mn[0] || p.y < mn[1] || p.z < mn[2]) continue;
    if (p.x > mx[0] || p.y > mx[1] || p.z > mx[2]) continue;
    out.push_back(p);
  }
}

// Per-stage wall time accumulators for the CPU baseline report: A2/A4 projection,
// A6-A9 features, A11 CropBox, A12 downsampleCurrentScan, A13 KD-tree builds, A13-A18 GN
// iterations.  Relaxed atomics: the all-cores run calls process_scan from several threads.
static std::atomic<int64_t> g_stage_ns[6];
struct StageTimer {  // charges the time since the last lap to stage k; the destructor closes it
  int k;
  std::chrono::steady_clock::time_point t0;
  explicit StageTimer(int k_) : k(k_), t0(std::chrono::steady_clock::now()) {}
  void lap(int next) {
    const auto t1 = std::chrono::steady_clock::now();
    if (k >= 0)
      g_stage_ns[k].fetch_add(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                              std::memory_order_relaxed);
    k = next;
    t0 = t1;
  }
  ~StageTimer() { lap(-1); }
};

static void registration_core(const fbr_params& P, const Map& map, const P4* cornerLast, int64_t ncl,
                              const P4* surfLast, int64_t nsl, float tr[6], RegResult& R, int nthreads,
                              const fbr_deskew_table* T = nullptr, bool no_crop = false,
                              bool* deg_state = nullptr) {
  fbr_reg_stats& st = R.st;
  std::memset(&st, 0, sizeof(st));
  // mapOptimization::isDegenerate is a class member (:137): LMOptimization only rewrites it at
  // iteration 0 with >= 50 rows, so it carries across registration() calls (deg_state, when the
  // caller keeps one; independent jobs start from false)
  bool isDegenerate = deg_state ? *deg_state : false;
  st.degenerate = isDegenerate ? 1 : 0;
  R.trace.clear();
  // CropBox around the guess translation (:284-304); origin/edges in float
  const float origin[3] = {tr[3], tr[4], tr[5]};
  float mn[3], mx[3];
  for (int i = 0; i < 3; ++i) {
    mn[i] = -P.crop_half[i] + origin[i];
    mx[i] = P.crop_half[i] + origin[i];
  }
  StageTimer tm(2);
  std::vector<P4> cornerMap, surfMap;
  if (no_crop) {  // LIO-SAM path: scan2MapOptimization on laserCloud*FromMapDS as extracted
    cornerMap = map.corner;
    surfMap = map.surf;
  } else {
    crop(map.corner, mn, mx, cornerMap);
    crop(map.surf, mn, mx, surfMap);
  }
  st.n_corner_map = (int)cornerMap.size();
  st.n_surf_map = (int)surfMap.size();
  tm.lap(3);
  // downsampleCurrentScan (:981-993)
  std::vector<P4> cornerDS, surfDS;
  voxel_grid(cornerLast, ncl, P.mapping_corner_leaf_size, cornerDS);
  voxel_grid(surfLast, nsl, P.mapping_surf_leaf_size, surfDS);
  const int Nc = (int)cornerDS.size(), Ns = (int)surfDS.size();
  st.n_corner_ds = Nc;
  st.n_surf_ds = Ns;
  // scan2MapOptimization (:1403-1442)
  tm.lap(4);
  if (!(Nc > P.edge_feature_min_valid_num && Ns > P.surf_feature_min_valid_num)) {
    st.status = FBR_REG_NOT_ENOUGH_FEATURES;
    return;
  }
  struct DegSave {  // write the member back on every return below
    bool* state;
    const bool& v;
    ~DegSave() {
      if (state) *state = v;
    }
  } deg_save{deg_state, isDegenerate};
  KDTree kdc, kds;
  kdc.build(cornerMap.data(), (int)cornerMap.size());
  kds.build(surfMap.data(), (int)surfMap.size());
  tm.lap(5);
  std::vector<P4> oriC(Nc), coeffC(Nc), oriS(Ns), coeffS(Ns);
  std::vector<char> flagC(Nc), flagS(Ns);
  for (int iterCount = 0; iterCount < P.max_iterations; iterCount++) {
    const Affine T = trans2affine(tr);  // updatePointAssociateToMap (:995-1000)
    std::fill(flagC.begin(), flagC.end(), 0);
    std::fill(flagS.begin(), flagS.end(), 0);
    // ---- cornerOptimization (:1002-1124) ----
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int i = 0; i < Nc; i++) {
      P4 pointOri = cornerDS[i];
      P4 pointSel = associate(T, pointOri);
      KDTree::Res nn = kdc.knn5(pointSel);
      if (nn.cnt < 5) continue;  // < 5 map points: undefined in the reference; rejected here
      if (nn.d[4] < 1.0) {
        float cx = 0, cy = 0, cz = 0;
        for (int j = 0; j < 5; j++) {
          cx += cornerMap[nn.i[j]].x;
          cy += cornerMap[nn.i[j]].y;
          cz += cornerMap[nn.i[j]].z;
        }
        cx /= 5;
        cy /= 5;
        cz /= 5;
        float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
        for (int j = 0; j < 5; j++) {
          float ax = cornerMap[nn.i[j]].x - cx;
          float ay = cornerMap[nn.i[j]].y - cy;
          float az = cornerMap[nn.i[j]].z - cz;
          a11 += ax * ax; a12 += ax * ay; a13 += ax * az;
          a22 += ay * ay; a23 += ay * az;
          a33 += az * az;
        }
        a11 /= 5; a12 /= 5; a13 /= 5; a22 /= 5; a23 /= 5; a33 /= 5;
        float A1[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33};
        float D1[3], V1[9];
        cv_jacobi(A1, 3, D1, V1);
        if (D1[0] > 3 * D1[1]) {
          float x0 = pointSel.x, y0 = pointSel.y, z0 = pointSel.z;
          float x1 = cx + 0.1 * V1[0], y1 = cy + 0.1 * V1[1], z1 = cz + 0.1 * V1[2];
          float x2 = cx - 0.1 * V1[0], y2 = cy - 0.1 * V1[1], z2 = cz - 0.1 * V1[2];
          float a012 = std::sqrt(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                 ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                 ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
          float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
          float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                      (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) / a012 / l12;
          float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                       (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
          float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                       (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) / a012 / l12;
          float ld2 = a012 / l12;
          float s = 1 - 0.9 * std::fabs(ld2);
          P4 coeff{s * la, s * lb, s * lc, s * ld2};
          if (s > 0.1) {
            oriC[i] = pointOri;
            coeffC[i] = coeff;
            flagC[i] = 1;
          }
        }
      }
    }
    // ---- surfOptimization (:1126-1215) ----
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (int i = 0; i < Ns; i++) {
      P4 pointOri = surfDS[i];
      P4 pointSel = associate(T, pointOri);
      KDTree::Res nn = kds.knn5(pointSel);
      if (nn.cnt < 5) continue;
      if (nn.d[4] < 1.0) {
        float A0[5][3], B0[5], X0[3];
        for (int j = 0; j < 5; j++) {
          A0[j][0] = surfMap[nn.i[j]].x;
          A0[j][1] = surfMap[nn.i[j]].y;
          A0[j][2] = surfMap[nn.i[j]].z;
          B0[j] = -1.0f;
        }
        eigen_colpiv_solve(A0, B0, X0);
        float pa = X0[0], pb = X0[1], pc = X0[2], pd = 1;
        float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
        pa /= ps; pb /= ps; pc /= ps; pd /= ps;
        bool planeValid = true;
        for (int j = 0; j < 5; j++) {
          if (std::fabs(pa * surfMap[nn.i[j]].x + pb * surfMap[nn.i[j]].y + pc * surfMap[nn.i[j]].z + pd) > 0.2) {
            planeValid = false;
            break;
          }
        }
        if (planeValid) {
          float pd2 = pa * pointSel.x + pb * pointSel.y + pc * pointSel.z + pd;
          float s = 1 - 0.9 * std::fabs(pd2) /
                            std::sqrt(std::sqrt(pointSel.x * pointSel.x + pointSel.y * pointSel.y + pointSel.z * pointSel.z));
          P4 coeff{s * pa, s * pb, s * pc, s * pd2};
          if (s > 0.1) {
            oriS[i] = pointOri;
            coeffS[i] = coeff;
            flagS[i] = 1;
          }
        }
      }
    }
    // ---- combineOptimizationCoeffs (:1218-1243) ----
    std::vector<P4> laserCloudOri, coeffSel;
    for (int i = 0; i < Nc; ++i)
      if (flagC[i]) laserCloudOri.push_back(oriC[i]), coeffSel.push_back(coeffC[i]);
    for (int i = 0; i < Ns; ++i)
      if (flagS[i]) laserCloudOri.push_back(oriS[i]), coeffSel.push_back(coeffS[i]);
    // ---- LMOptimization (:1246-1401) ----
    st.iterations = iterCount + 1;
    float srx = std::sin(tr[1]), crx = std::cos(tr[1]);
    float sry = std::sin(tr[2]), cry = std::cos(tr[2]);
    float srz = std::sin(tr[0]), crz = std::cos(tr[0]);
    const int sel = (int)laserCloudOri.size();
    st.n_sel = sel;
    if (sel < 50) {  // :1268 return false: keep iterating with an unchanged pose
      R.trace.insert(R.trace.end(), tr, tr + 6);
      continue;
    }
    double AtA_d[36] = {0}, AtB_d[6] = {0};
    for (int i = 0; i < sel; i++) {
      P4 pointOri, coeff;
      pointOri.x = laserCloudOri[i].y;
      pointOri.y = laserCloudOri[i].z;
      pointOri.z = laserCloudOri[i].x;
      coeff.x = coeffSel[i].y;
      coeff.y = coeffSel[i].z;
      coeff.z = coeffSel[i].x;
      coeff.intensity = coeffSel[i].intensity;
      float arx = (crx * sry * srz * pointOri.x + crx * crz * sry * pointOri.y - srx * sry * pointOri.z) * coeff.x +
                  (-srx * srz * pointOri.x - crz * srx * pointOri.y - crx * pointOri.z) * coeff.y +
                  (crx * cry * srz * pointOri.x + crx * cry * crz * pointOri.y - cry * srx * pointOri.z) * coeff.z;
      float ary = ((cry * srx * srz - crz * sry) * pointOri.x + (sry * srz + cry * crz * srx) * pointOri.y + crx * cry * pointOri.z) * coeff.x +
                  ((-cry * crz - srx * sry * srz) * pointOri.x + (cry * srz - crz * srx * sry) * pointOri.y - crx * sry * pointOri.z) * coeff.z;
      float arz = ((crz * srx * sry - cry * srz) * pointOri.x + (-cry * crz - srx * sry * srz) * pointOri.y) * coeff.x +
                  (crx * crz * pointOri.x - crx * srz * pointOri.y) * coeff.y +
                  ((sry * srz + cry * crz * srx) * pointOri.x + (crz * sry - cry * srx * srz) * pointOri.y) * coeff.z;
      const float row[6] = {arz, arx, ary, coeff.z, coeff.x, coeff.y};
      const float b = -coeff.intensity;
      for (int r = 0; r < 6; ++r) {
        for (int c = 0; c < 6; ++c) AtA_d[r * 6 + c] += (double)row[r] * (double)row[c];
        AtB_d[r] += (double)row[r] * (double)b;
      }
    }
    float AtA[36], X[6], tmpA[36];
    for (int k = 0; k < 36; ++k) AtA[k] = (float)AtA_d[k];
    for (int k = 0; k < 6; ++k) X[k] = (float)AtB_d[k];
    std::memcpy(tmpA, AtA, sizeof(tmpA));
    if (!cv_qr_solve(tmpA, 6, X))
      for (int k = 0; k < 6; ++k) X[k] = 0.0f;
    float matP[36] = {0};  // local cv::Mat matP (:1278): zero unless filled at iterCount == 0
    if (iterCount == 0) {
      float E[6], V[36], V2[36];
      std::memcpy(tmpA, AtA, sizeof(tmpA));
      cv_jacobi(tmpA, 6, E, V);
      std::memcpy(V2, V, sizeof(V2));
      isDegenerate = false;
      const float eignThre[6] = {100, 100, 100, 100, 100, 100};
      for (int i = 5; i >= 0; i--) {
        if (E[i] < eignThre[i]) {
          for (int j = 0; j < 6; j++) V2[i * 6 + j] = 0;
          isDegenerate = true;
        } else {
          break;
        }
      }
      float Vinv[36];
      if (!cv_lu_inv(V, 6, Vinv)) std::memset(Vinv, 0, sizeof(Vinv));
      cv_gemm(Vinv, V2, matP, 6, 6, 6);
    }
    if (isDegenerate) {
      float X2[6];
      std::memcpy(X2, X, sizeof(X2));
      cv_gemm(matP, X2, X, 6, 6, 1);
    }
    st.degenerate = isDegenerate ? 1 : 0;
    for (int k = 0; k < 6; ++k) tr[k] += X[k];
    R.trace.insert(R.trace.end(), tr, tr + 6);
    const float r0 = X[0] * 57.29578f, r1 = X[1] * 57.29578f, r2 = X[2] * 57.29578f;  // pcl::rad2deg
    float deltaR = std::sqrt(std::pow(r0, 2) + std::pow(r1, 2) + std::pow(r2, 2));
    float deltaT = std::sqrt(std::pow(X[3] * 100, 2) + std::pow(X[4] * 100, 2) + std::pow(X[5] * 100, 2));
    if (deltaR < 0.05 && deltaT < 0.05) {
      st.converged = 1;
      break;
    }
  }
  // transformUpdate (:1444-1479)
  if (T && T->imu_available) {  // cloudInfo.imuAvailable (:1447)
    if (std::abs(T->imu_pitch_init) < 1.4) {
      double imuWeight = 0.05;
      double rollMid, pitchMid, yawMid;
      TfQuaternion transformQuaternion = tf_setRPY(tr[0], 0, 0);
      TfQuaternion imuQuaternion = tf_setRPY(T->imu_roll_init, 0, 0);
      tf_getRPY(tf_slerp(transformQuaternion, imuQuaternion, imuWeight), rollMid, pitchMid, yawMid);
      tr[0] = rollMid;
      transformQuaternion = tf_setRPY(0, tr[1], 0);
      imuQuaternion = tf_setRPY(0, T->imu_pitch_init, 0);
      tf_getRPY(tf_slerp(transformQuaternion, imuQuaternion, imuWeight), rollMid, pitchMid, yawMid);
      tr[1] = pitchMid;
    }
  }
  auto clampf = [](float v, float lim) {
    if (v < -lim) v = -lim;
    if (v > lim) v = lim;
    return v;
  };
  tr[0] = clampf(tr[0], P.rotation_tollerance);
  tr[1] = clampf(tr[1], P.rotation_tollerance);
  tr[5] = clampf(tr[5], P.z_tollerance);
}

}  // namespace orc

// =============================================================================================
// C-ABI used by the tests (ctypes) and by bench.py's cpu_baseline leg.
// =============================================================================================
using namespace orc;

struct orc_stream {
  fbr_params P;
  FeatState fs;
  double timeLastProcessing = -1;
  bool isDegenerate = false;  // mapOptimization::isDegenerate (carried between scans)
  bool has_desk = false;  // deskewInfo() enabled for the next scans (orc_stream_set_deskew)
  fbr_deskew_table desk;
  const fbr_deskew_table* table() const { return has_desk ? &desk : nullptr; }
};

extern "C" {

int64_t orc_project(const fbr_params* P, const fbr_point_xyzirt* pts, int64_t n_in, int32_t* start_ring,
                    int32_t* end_ring, int32_t* col_ind, float* range, fbr_point_xyzi* cloud,
                    const fbr_deskew_table* desk) {
  Projection pr;
  project(*P, pts, n_in, pr, desk);
  const int64_t n = (int64_t)pr.col.size();
  if (start_ring) std::memcpy(start_ring, pr.start.data(), sizeof(int32_t) * P->n_scan);
  if (end_ring) std::memcpy(end_ring, pr.end.data(), sizeof(int32_t) * P->n_scan);
  if (col_ind) std::memcpy(col_ind, pr.col.data(), sizeof(int32_t) * n);
  if (range) std::memcpy(range, pr.range.data(), sizeof(float) * n);
  if (cloud) std::memcpy(cloud, pr.cloud.data(), sizeof(fbr_point_xyzi) * n);
  return n;
}

int64_t orc_voxel_grid(const fbr_point_xyzi* in, int64_t n, float leaf, fbr_point_xyzi* out) {
  std::vector<P4> o;
  voxel_grid(in, n, leaf, o);
  if (out) std::memcpy(out, o.data(), sizeof(P4) * o.size());
  return (int64_t)o.size();
}

void* orc_stream_create(const fbr_params* P) {
  orc_stream* s = new orc_stream();
  s->P = *P;
  s->fs.init(P->n_scan, P->horizon_scan);
  return s;
}
void orc_stream_destroy(void* s) { delete (orc_stream*)s; }
void orc_stream_set_deskew(void* s, const fbr_deskew_table* t) {
  orc_stream* st = (orc_stream*)s;
  st->has_desk = t != nullptr;
  if (t) st->desk = *t;
}
void orc_stream_reset(void* s) {
  orc_stream* st = (orc_stream*)s;
  st->fs.init(st->P.n_scan, st->P.horizon_scan);
  st->timeLastProcessing = -1;
  st->isDegenerate = false;
}

// Projection + FeatureExtraction on one scan (stream state carried in `s`).
int orc_features(void* s, const fbr_point_xyzirt* pts, int64_t n_in, int8_t* label, fbr_point_xyzi* corner,
                 int64_t* n_corner, fbr_point_xyzi* surf, int64_t* n_surf, int64_t* n_points) {
  orc_stream* st = (orc_stream*)s;
  Projection pr;
  project(st->P, pts, n_in, pr, st->table());
  Features F;
  extract_features(st->P, st->fs, pr, F);
  const int64_t n = (int64_t)pr.col.size();
  if (n_points) *n_points = n;
  if (label)
    for (int64_t i = 0; i < n; ++i) label[i] = (int8_t)st->fs.label[i];
  if (corner) std::memcpy(corner, F.corner.data(), sizeof(P4) * F.corner.size());
  if (surf) std::memcpy(surf, F.surf.data(), sizeof(P4) * F.surf.size());
  if (n_corner) *n_corner = (int64_t)F.corner.size();
  if (n_surf) *n_surf = (int64_t)F.surf.size();
  return 0;
}

void* orc_map_create(const fbr_params* P, const fbr_point_xyzi* corner, int64_t nc, const fbr_point_xyzi* surf,
                     int64_t ns) {
  Map* m = new Map();
  voxel_grid(corner, nc, P->mapping_corner_leaf_size, m->corner);  // mapOptmization.h:251-252
  voxel_grid(surf, ns, P->mapping_surf_leaf_size, m->surf);        // :256-257
  return m;
}
void orc_map_destroy(void* m) { delete (Map*)m; }
// A map taken as it is (the keyframe local map is already down-sampled by extractCloud).
void* orc_map_create_raw(const fbr_point_xyzi* corner, int64_t nc, const fbr_point_xyzi* surf, int64_t ns) {
  Map* m = new Map();
  m->corner.assign(corner, corner + nc);
  m->surf.assign(surf, surf + ns);
  return m;
}

// extractSurroundingKeyFrames (mapOptmization.h:964-978): extractNearby (:872-907) or
// extractForLoopClosure (:857-870), then extractCloud (:909-955) with transformPointCloud
// (:405-425).  Key clouds are given as pools + per-keyframe offsets / counts; poses are
// PointXYZIRPYT with intensity = key index.  The radius search restates KdTreeFLANN::radiusSearch
// (d2 < r^2, results sorted by distance; equal distances by index).
int orc_kf_extract(const fbr_params* P, const fbr_keypose* poses, int64_t N, const fbr_point_xyzi* cpool,
                   const int64_t* c_off, const int64_t* c_cnt, const fbr_point_xyzi* spool, const int64_t* s_off,
                   const int64_t* s_cnt, const fbr_keyframe_params* kp, double timeLaserCloudInfoLast,
                   fbr_point_xyzi* corner_out, int64_t* n_corner, fbr_point_xyzi* surf_out, int64_t* n_surf,
                   int32_t* n_frames) {
  std::vector<P4> cloudToExtract;
  const fbr_keypose& back = poses[N - 1];
  auto pose3D = [&](int64_t i) { return P4{poses[i].x, poses[i].y, poses[i].z, poses[i].intensity}; };
  if (kp->loop_closure) {
    for (int64_t i = N - 1; i >= 0; --i) {
      if ((int)cloudToExtract.size() <= kp->submap_size) cloudToExtract.push_back(pose3D(i));
      else break;
    }
  } else {
    std::vector<std::pair<float, int64_t>> found;
    const float radius2 = (float)((double)kp->search_radius * (double)kp->search_radius);
    for (int64_t i = 0; i < N; ++i) {
      float dist = 0, diff;
      diff = back.x - poses[i].x; dist += diff * diff;
      diff = back.y - poses[i].y; dist += diff * diff;
      diff = back.z - poses[i].z; dist += diff * diff;
      if (dist < radius2) found.emplace_back(dist, i);
    }
    std::stable_sort(found.begin(), found.end(), [](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) {
      return a.first < b.first;
    });
    std::vector<P4> surroundingKeyPoses;
    for (auto& f : found) surroundingKeyPoses.push_back(pose3D(f.second));
    voxel_grid(surroundingKeyPoses.data(), (int64_t)surroundingKeyPoses.size(), kp->pose_density, cloudToExtract);
    for (int64_t i = N - 1; i >= 0; --i) {
      if (timeLaserCloudInfoLast - poses[i].time < kp->recent_window) cloudToExtract.push_back(pose3D(i));
      else break;
    }
  }
  *n_frames = (int32_t)cloudToExtract.size();
  std::vector<P4> cornerFromMap, surfFromMap;
  for (const P4& e : cloudToExtract) {
    const float dist = std::sqrt((e.x - back.x) * (e.x - back.x) + (e.y - back.y) * (e.y - back.y) +
                                 (e.z - back.z) * (e.z - back.z));  // pointDistance (utility.h:312-315)
    if (dist > kp->search_radius) continue;
    const int thisKeyInd = (int)e.intensity;
    if (thisKeyInd < 0 || thisKeyInd >= N) return -1;
    const fbr_keypose& t = poses[thisKeyInd];
    const Affine transCur = get_transformation(t.x, t.y, t.z, t.roll, t.pitch, t.yaw);
    for (int pass = 0; pass < 2; ++pass) {
      const P4* src = pass ? spool + s_off[thisKeyInd] : cpool + c_off[thisKeyInd];
      const int64_t cnt = pass ? s_cnt[thisKeyInd] : c_cnt[thisKeyInd];
      std::vector<P4>& dst = pass ? surfFromMap : cornerFromMap;
      for (int64_t i = 0; i < cnt; ++i) {
        const P4& pf = src[i];
        P4 o;
        o.x = transCur.m[0][0] * pf.x + transCur.m[0][1] * pf.y + transCur.m[0][2] * pf.z + transCur.m[0][3];
        o.y = transCur.m[1][0] * pf.x + transCur.m[1][1] * pf.y + transCur.m[1][2] * pf.z + transCur.m[1][3];
        o.z = transCur.m[2][0] * pf.x + transCur.m[2][1] * pf.y + transCur.m[2][2] * pf.z + transCur.m[2][3];
        o.intensity = pf.intensity;
        dst.push_back(o);
      }
    }
  }
  std::vector<P4> cds, sds;
  voxel_grid(cornerFromMap.data(), (int64_t)cornerFromMap.size(), P->mapping_corner_leaf_size, cds);
  voxel_grid(surfFromMap.data(), (int64_t)surfFromMap.size(), P->mapping_surf_leaf_size, sds);
  *n_corner = (int64_t)cds.size();
  *n_surf = (int64_t)sds.size();
  if (corner_out) std::memcpy(corner_out, cds.data(), sizeof(P4) * cds.size());
  if (surf_out) std::memcpy(surf_out, sds.data(), sizeof(P4) * sds.size());
  return 0;
}
int orc_map_get(void* mp, int64_t* nc, int64_t* ns, fbr_point_xyzi* corner, fbr_point_xyzi* surf) {
  Map* m = (Map*)mp;
  if (nc) *nc = (int64_t)m->corner.size();
  if (ns) *ns = (int64_t)m->surf.size();
  if (corner) std::memcpy(corner, m->corner.data(), sizeof(P4) * m->corner.size());
  if (surf) std::memcpy(surf, m->surf.data(), sizeof(P4) * m->surf.size());
  return 0;
}

// degenerate_inout: the isDegenerate member before / after the call (null: a fresh matcher, false)
int orc_register(const fbr_params* P, void* map, const fbr_point_xyzi* corner, int64_t nc, const fbr_point_xyzi* surf,
                 int64_t ns, float pose[6], fbr_reg_stats* st, float* trace, int nthreads,
                 const fbr_deskew_table* desk, int no_crop, int32_t* degenerate_inout) {
  RegResult R;
  bool deg = degenerate_inout ? *degenerate_inout != 0 : false;
  registration_core(*P, *(Map*)map, corner, nc, surf, ns, pose, R, nthreads, desk, no_crop != 0,
                    degenerate_inout ? &deg : nullptr);
  if (degenerate_inout) *degenerate_inout = deg ? 1 : 0;
  if (st) *st = R.st;
  if (trace) std::memcpy(trace, R.trace.data(), sizeof(float) * R.trace.size());
  return 0;
}

// cloudHandler minus the ROS queue: projection, features, registration with the time gate.
int orc_process_scan(void* s, void* map, const fbr_point_xyzirt* pts, int64_t n_in, double stamp, float pose[6],
                     fbr_reg_stats* st, int nthreads) {
  orc_stream* S = (orc_stream*)s;
  StageTimer tm(0);
  Projection pr;
  project(S->P, pts, n_in, pr, S->table());
  tm.lap(1);
  Features F;
  extract_features(S->P, S->fs, pr, F);
  tm.lap(-1);
  RegResult R;
  std::memset(&R.st, 0, sizeof(R.st));
  if (stamp - S->timeLastProcessing >= S->P.mapping_process_interval) {
    S->timeLastProcessing = stamp;
    registration_core(S->P, *(Map*)map, F.corner.data(), (int64_t)F.corner.size(), F.surf.data(),
                      (int64_t)F.surf.size(), pose, R, nthreads, S->table(), false, &S->isDegenerate);
  } else {
    R.st.status = FBR_REG_SKIPPED_INTERVAL;
  }
  R.st.n_points = (int)pr.col.size();
  R.st.n_corner = (int)F.corner.size();
  R.st.n_surf = (int)F.surf.size();
  if (st) *st = R.st;
  return 0;
}

void orc_affine_from_pose(const float pose[6], float m[16]) {
  Affine t = trans2affine(pose);
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) m[r * 4 + c] = t.m[r][c];
  m[12] = m[13] = m[14] = 0.0f;
  m[15] = 1.0f;
}
void orc_pose_from_affine(const float m[16], float pose[6]) {
  Affine t;
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) t.m[r][c] = m[r * 4 + c];
  get_translation_euler(t, pose);
}

// imuConverter (utility.h:219-253) for the CPU tests of fbr_imu_convert: Eigen Matrix3d * Vector3d
// (coefficient products summed x0 + (x1 + x2)), Quaterniond(Matrix3d), generic quaternion product.
int orc_imu_convert(const fbr_imu_extrinsics* ext, const fbr_imu_sample* in, fbr_imu_sample* out) {
  *out = *in;
  const double* R = ext->ext_rot;
  for (int r = 0; r < 3; ++r) {
    const double* a = in->linear_acceleration;
    const double* g = in->angular_velocity;
    out->linear_acceleration[r] = R[3 * r] * a[0] + (R[3 * r + 1] * a[1] + R[3 * r + 2] * a[2]);
    out->angular_velocity[r] = R[3 * r] * g[0] + (R[3 * r + 1] * g[1] + R[3 * r + 2] * g[2]);
  }
  const double* m = ext->ext_rpy;  // extQRPY = Eigen::Quaterniond(extRPY): x, y, z, w
  double e[4];
  double t = m[0] + (m[4] + m[8]);
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    e[3] = 0.5 * t;
    t = 0.5 / t;
    e[0] = (m[7] - m[5]) * t;
    e[1] = (m[2] - m[6]) * t;
    e[2] = (m[3] - m[1]) * t;
  } else {
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[4 * i]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(m[4 * i] - m[4 * j] - m[4 * k] + 1.0);
    e[i] = 0.5 * t;
    t = 0.5 / t;
    e[3] = (m[3 * k + j] - m[3 * j + k]) * t;
    e[j] = (m[3 * j + i] + m[3 * i + j]) * t;
    e[k] = (m[3 * k + i] + m[3 * i + k]) * t;
  }
  const double* b = in->orientation;  // q_final = extQRPY * q_from
  double w = e[3] * b[3] - e[0] * b[0] - e[1] * b[1] - e[2] * b[2];
  double x = e[3] * b[0] + e[0] * b[3] + e[1] * b[2] - e[2] * b[1];
  double y = e[3] * b[1] + e[1] * b[3] + e[2] * b[0] - e[0] * b[2];
  double z = e[3] * b[2] + e[2] * b[3] + e[0] * b[1] - e[1] * b[0];
  out->orientation[0] = x;
  out->orientation[1] = y;
  out->orientation[2] = z;
  out->orientation[3] = w;
  if (std::sqrt(x * x + y * y + z * z + w * w) < 0.1) return -1;  // "please use a 9-axis IMU!"
  return 0;
}

// deskewInfo + imuDeskewInfo (imageProjection.cpp:303-393) on a copy of the queue, run as written
// (pop_front, then the integration loop); *n_pop = samples popped.  imu*Init: imuRPY2rosRPY
// (tf::quaternionMsgToTF, normalised when |length2 - 1| > 0.1, then Matrix3x3::getRPY).
int orc_imu_deskew_info(const fbr_imu_sample* q, int64_t n, double timeScanCur, double timeScanNext,
                        fbr_deskew_table* out, int64_t* n_pop) {
  std::vector<fbr_imu_sample> imuQueue(q, q + n);
  size_t front = 0;
  const float ri = out->imu_roll_init, pi = out->imu_pitch_init, yi = out->imu_yaw_init;
  std::memset(out, 0, sizeof(*out));
  out->imu_roll_init = ri;
  out->imu_pitch_init = pi;
  out->imu_yaw_init = yi;
  out->time_scan_cur = timeScanCur;
  *n_pop = 0;
  if (imuQueue.empty() || imuQueue.front().stamp > timeScanCur || imuQueue.back().stamp < timeScanNext) {
    out->status = FBR_DESKEW_WAIT_IMU;  // "Waiting for IMU data ..." (:310-314)
    return 0;
  }
  out->status = FBR_DESKEW_READY;
  out->imu_available = 0;
  while (front < imuQueue.size()) {
    if (imuQueue[front].stamp < timeScanCur - 0.01) ++front;
    else break;
  }
  *n_pop = (int64_t)front;
  if (front == imuQueue.size()) return 0;
  int imuPointerCur = 0;
  for (size_t i = front; i < imuQueue.size(); ++i) {
    const fbr_imu_sample& thisImuMsg = imuQueue[i];
    double currentImuTime = thisImuMsg.stamp;
    if (currentImuTime <= timeScanCur) {
      TfQuaternion o{thisImuMsg.orientation[0], thisImuMsg.orientation[1], thisImuMsg.orientation[2],
                     thisImuMsg.orientation[3]};
      double l2 = tf_dot(o, o);
      if (std::fabs(l2 - 1) > 0.1f) {
        double f = 1.0 / std::sqrt(l2);
        o = TfQuaternion{o.x * f, o.y * f, o.z * f, o.w * f};
      }
      double imuRoll, imuPitch, imuYaw;
      tf_getRPY(o, imuRoll, imuPitch, imuYaw);
      out->imu_roll_init = imuRoll;
      out->imu_pitch_init = imuPitch;
      out->imu_yaw_init = imuYaw;
    }
    if (currentImuTime > timeScanNext + 0.01) break;
    if (imuPointerCur >= FBR_IMU_QUEUE) return -4;
    if (imuPointerCur == 0) {
      out->imu_rot_x[0] = 0;
      out->imu_rot_y[0] = 0;
      out->imu_rot_z[0] = 0;
      out->imu_time[0] = currentImuTime;
      ++imuPointerCur;
      continue;
    }
    double angular_x = thisImuMsg.angular_velocity[0], angular_y = thisImuMsg.angular_velocity[1],
           angular_z = thisImuMsg.angular_velocity[2];
    double timeDiff = currentImuTime - out->imu_time[imuPointerCur - 1];
    out->imu_rot_x[imuPointerCur] = out->imu_rot_x[imuPointerCur - 1] + angular_x * timeDiff;
    out->imu_rot_y[imuPointerCur] = out->imu_rot_y[imuPointerCur - 1] + angular_y * timeDiff;
    out->imu_rot_z[imuPointerCur] = out->imu_rot_z[imuPointerCur - 1] + angular_z * timeDiff;
    out->imu_time[imuPointerCur] = currentImuTime;
    ++imuPointerCur;
  }
  --imuPointerCur;
  out->imu_pointer_cur = imuPointerCur < 0 ? 0 : imuPointerCur;  // (-1 in the reference: unused then)
  if (imuPointerCur <= 0) return 0;
  out->imu_available = 1;
  return 0;
}

// Small-solver probes for unit tests.
void orc_jacobi(float* A, int n, float* W, float* V) { cv_jacobi(A, n, W, V); }
int orc_qr_solve(float* A, int n, float* b) { return cv_qr_solve(A, n, b); }
void orc_colpiv_solve(const float* A15, const float* b5, float* x3) {
  float A[5][3];
  std::memcpy(A, A15, sizeof(A));
  eigen_colpiv_solve(A, b5, x3);
}
int orc_knn5(const fbr_point_xyzi* map, int64_t n, const fbr_point_xyzi* q, int64_t nq, int32_t* idx, float* d2) {
  KDTree kd;
  kd.build(map, (int)n);
  for (int64_t i = 0; i < nq; ++i) {
    KDTree::Res r = kd.knn5(q[i]);
    for (int j = 0; j < 5; ++j) {
      idx[i * 5 + j] = j < r.cnt ? r.i[j] : -1;
      d2[i * 5 + j] = j < r.cnt ? r.d[j] : INFINITY;
    }
  }
  return 0;
}
// Sort probe: libstdc++ std::sort of smoothness_t by value; writes the resulting ind order.
void orc_sort_smoothness(const float* values, int64_t n, int64_t* ind_out) {
  std::vector<smoothness_t> v(n);
  for (int64_t i = 0; i < n; ++i) v[i] = smoothness_t{values[i], (size_t)i};
  std::sort(v.begin(), v.end(), by_value());
  for (int64_t i = 0; i < n; ++i) ind_out[i] = (int64_t)v[i].ind;
}
// Sort probe: libstdc++ std::sort of PCL's cloud_point_index_idx {idx, i} by idx (VoxelGrid,
// voxel_grid.cpp); writes the resulting cloud_point_index order.
void orc_sort_voxel_pairs(const uint32_t* keys, int64_t n, int64_t* ind_out) {
  std::vector<cloud_point_index_idx> v(n);
  for (int64_t i = 0; i < n; ++i) v[i] = cloud_point_index_idx{keys[i], (unsigned)i};
  std::sort(v.begin(), v.end(), std::less<cloud_point_index_idx>());
  for (int64_t i = 0; i < n; ++i) ind_out[i] = (int64_t)v[i].cloud_point_index;
}
int orc_num_threads_max(void) { return omp_get_max_threads(); }

// Accumulated per-stage wall time (ms) of process_scan / register calls since the last reset:
// [A2/A4 projection, A6-A9 features, A11 CropBox, A12 downsampleCurrentScan, A13 KD-tree builds,
//  A13-A18 Gauss-Newton iterations].
void orc_stage_ms(double out[6], int reset) {
  for (int k = 0; k < 6; ++k) {
    if (out) out[k] = (double)g_stage_ns[k].load(std::memory_order_relaxed) * 1e-6;
    if (reset) g_stage_ns[k].store(0, std::memory_order_relaxed);
  }
}

}  // extern "C"
