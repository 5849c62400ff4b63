// fbr_imu.h — IMU deskew arithmetic, shared by the host table builder
// (fbr_imu.cpp) and the device kernels (k_project.hip: deskewPoint, k_register.hip: the IMU half
// of transformUpdate).  Restated in the reference's operation order:
//   findRotation             /root/reference/src/imageProjection.cpp:494-526 (double)
//   deskewPoint              :545-580 (float; findPosition is all-zero, :528-542)
//   pcl::getTransformation   pcl/common/impl/eigen.hpp (float)
//   Affine3f::inverse        Eigen 3.3 Transform::inverse(Affine): 3x3 cofactor inverse
//                            (InverseImpl.h compute_inverse<..., 3>), t' = (-L^-1) * t
//   Affine3f * Affine3f      Eigen 3.3 transform_transform_product_impl: L = L1 * L2,
//                            t = L1 * t2 + t1
//   Eigen 3-term sums        fixed-size coefficient products reduce as x0 + (x1 + x2)
//                            (redux_novec_unroller splits 3 into 1 + 2)
//   tf::Quaternion::setRPY / slerp / angleShortestPath, tf::Matrix3x3(q).getRPY
//                            (tf/LinearMath/Quaternion.h, Matrix3x3.h; tfScalar = double)
// Float sin/cos are glibc's sinf/cosf restated bit for bit (fbr_sincosf.h), on the host and the
// device alike.
#pragma once
#include <math.h>
#include <stdint.h>

#include "fbr.h"
#include "fbr_sincosf.h"

#if defined(__HIPCC__)
#define FBR_HD __host__ __device__
#else
#define FBR_HD
#endif

namespace fbr {

// desk_mode bits of a job (fbr_set_deskew)
constexpr int kDeskPoints = 1;  // deskewPoint active: deskewFlag != -1 && imuAvailable (:548)
constexpr int kDeskImu = 2;     // cloudInfo.imuAvailable: transformUpdate's IMU slerp (:1447)

struct Rot3 {
  float m[3][3];
};

// sinf / cosf as glibc 2.35 computes them on an FMA-capable x86-64 host (fbr_sincosf.h).
FBR_HD inline float fsin(float x) { return gl_sinf(x); }
FBR_HD inline float fcos(float x) { return gl_cosf(x); }

// findRotation (:494-526)
FBR_HD inline void find_rotation(const fbr_deskew_table& T, double pointTime, float* rx, float* ry, float* rz) {
  int f = 0;
  while (f < T.imu_pointer_cur) {
    if (pointTime < T.imu_time[f]) break;
    ++f;
  }
  if (pointTime > T.imu_time[f] || f == 0) {
    *rx = (float)T.imu_rot_x[f];
    *ry = (float)T.imu_rot_y[f];
    *rz = (float)T.imu_rot_z[f];
  } else {
    const int b = f - 1;
    const double ratioFront = (pointTime - T.imu_time[b]) / (T.imu_time[f] - T.imu_time[b]);
    const double ratioBack = (T.imu_time[f] - pointTime) / (T.imu_time[f] - T.imu_time[b]);
    *rx = (float)(T.imu_rot_x[f] * ratioFront + T.imu_rot_x[b] * ratioBack);
    *ry = (float)(T.imu_rot_y[f] * ratioFront + T.imu_rot_y[b] * ratioBack);
    *rz = (float)(T.imu_rot_z[f] * ratioFront + T.imu_rot_z[b] * ratioBack);
  }
}

// Linear part of pcl::getTransformation(0, 0, 0, roll, pitch, yaw).
FBR_HD inline Rot3 rot_rpy(float roll, float pitch, float yaw) {
  const float A = fcos(yaw), B = fsin(yaw), C = fcos(pitch), D = fsin(pitch), E = fcos(roll), F = fsin(roll);
  const float DE = D * E, DF = D * F;
  Rot3 r;
  r.m[0][0] = A * C; r.m[0][1] = A * DF - B * E; r.m[0][2] = B * F + A * DE;
  r.m[1][0] = B * C; r.m[1][1] = A * E + B * DF; r.m[1][2] = B * DE - A * F;
  r.m[2][0] = -D;    r.m[2][1] = C * F;          r.m[2][2] = C * E;
  return r;
}

FBR_HD inline float sum3(float x0, float x1, float x2) { return x0 + (x1 + x2); }

// Eigen cofactor_3x3<i,j>: m(i1,j1) m(i2,j2) - m(i1,j2) m(i2,j1) with i1 = (i+1)%3, i2 = (i+2)%3.
FBR_HD inline float cof3(const Rot3& a, int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return a.m[i1][j1] * a.m[i2][j2] - a.m[i1][j2] * a.m[i2][j1];
}

// Affine3f::inverse() of a transform with zero translation: the inverse linear part, and
// t' = (-L^-1) * 0 with the signed zeros Eigen produces.
FBR_HD inline void affine_inverse(const Rot3& a, Rot3& inv, float t[3]) {
  const float c0 = cof3(a, 0, 0), c1 = cof3(a, 1, 0), c2 = cof3(a, 2, 0);
  const float det = sum3(c0 * a.m[0][0], c1 * a.m[1][0], c2 * a.m[2][0]);
  const float invdet = 1.0f / det;
  inv.m[0][0] = c0 * invdet;
  inv.m[0][1] = c1 * invdet;
  inv.m[0][2] = c2 * invdet;
  inv.m[1][0] = cof3(a, 0, 1) * invdet;
  inv.m[1][1] = cof3(a, 1, 1) * invdet;
  inv.m[1][2] = cof3(a, 2, 1) * invdet;
  inv.m[2][0] = cof3(a, 0, 2) * invdet;
  inv.m[2][1] = cof3(a, 1, 2) * invdet;
  inv.m[2][2] = cof3(a, 2, 2) * invdet;
  for (int r = 0; r < 3; ++r) t[r] = sum3(-inv.m[r][0] * 0.0f, -inv.m[r][1] * 0.0f, -inv.m[r][2] * 0.0f);
}

// transBt = transStartInverse * transFinal with transFinal = (R, 0): L1 * R and L1 * 0 + t1.
FBR_HD inline void compose(const Rot3& l1, const float t1[3], const Rot3& r, Rot3& out, float tout[3]) {
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) out.m[i][j] = sum3(l1.m[i][0] * r.m[0][j], l1.m[i][1] * r.m[1][j], l1.m[i][2] * r.m[2][j]);
    tout[i] = sum3(l1.m[i][0] * 0.0f, l1.m[i][1] * 0.0f, l1.m[i][2] * 0.0f) + t1[i];
  }
}

// deskewPoint's transform of one point (:574-577).
FBR_HD inline void apply_affine(const Rot3& r, const float t[3], float x, float y, float z, float* o) {
  o[0] = r.m[0][0] * x + r.m[0][1] * y + r.m[0][2] * z + t[0];
  o[1] = r.m[1][0] * x + r.m[1][1] * y + r.m[1][2] * z + t[1];
  o[2] = r.m[2][0] * x + r.m[2][1] * y + r.m[2][2] * z + t[2];
}

// ---- tf LinearMath (double) ----
struct TfQuat {
  double x, y, z, w;
};

FBR_HD inline TfQuat tf_set_rpy(double roll, double pitch, double yaw) {  // Quaternion::setRPY
  const double halfYaw = yaw * 0.5, halfPitch = pitch * 0.5, halfRoll = roll * 0.5;
  const double cosYaw = cos(halfYaw), sinYaw = sin(halfYaw);
  const double cosPitch = cos(halfPitch), sinPitch = sin(halfPitch);
  const double cosRoll = cos(halfRoll), sinRoll = sin(halfRoll);
  TfQuat q;
  q.x = sinRoll * cosPitch * cosYaw - cosRoll * sinPitch * sinYaw;
  q.y = cosRoll * sinPitch * cosYaw + sinRoll * cosPitch * sinYaw;
  q.z = cosRoll * cosPitch * sinYaw - sinRoll * sinPitch * cosYaw;
  q.w = cosRoll * cosPitch * cosYaw + sinRoll * sinPitch * sinYaw;
  return q;
}

FBR_HD inline double tf_dot(const TfQuat& a, const TfQuat& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

FBR_HD inline double tf_acos(double x) {  // tfAcos clamps to [-1, 1]
  if (x < -1.0) x = -1.0;
  if (x > 1.0) x = 1.0;
  return acos(x);
}
FBR_HD inline double tf_asin(double x) {  // tfAsin clamps to [-1, 1]
  if (x < -1.0) x = -1.0;
  if (x > 1.0) x = 1.0;
  return asin(x);
}

// Quaternion::slerp(q, t), with angleShortestPath
FBR_HD inline TfQuat tf_slerp(const TfQuat& a, const TfQuat& q, double t) {
  const double s = sqrt(tf_dot(a, a) * tf_dot(q, q));
  double ang;
  if (tf_dot(a, q) < 0) {
    const TfQuat nq{-q.x, -q.y, -q.z, -q.w};
    ang = tf_acos(tf_dot(a, nq) / s) * 2.0;
  } else {
    ang = tf_acos(tf_dot(a, q) / s) * 2.0;
  }
  const double theta = ang / 2.0;
  if (theta != 0.0) {
    const double d = 1.0 / sin(theta);
    const double s0 = sin((1.0 - t) * theta);
    const double s1 = sin(t * theta);
    if (tf_dot(a, q) < 0)
      return TfQuat{(a.x * s0 + -q.x * s1) * d, (a.y * s0 + -q.y * s1) * d, (a.z * s0 + -q.z * s1) * d,
                    (a.w * s0 + -q.w * s1) * d};
    return TfQuat{(a.x * s0 + q.x * s1) * d, (a.y * s0 + q.y * s1) * d, (a.z * s0 + q.z * s1) * d,
                  (a.w * s0 + q.w * s1) * d};
  }
  return a;
}

// tf::Matrix3x3(q).getRPY(roll, pitch, yaw): setRotation(q), then getEulerYPR (solution 1).
FBR_HD inline void tf_get_rpy(const TfQuat& q, double* roll, double* pitch, double* yaw) {
  const double d = tf_dot(q, q);
  const double s = 2.0 / d;
  const double xs = q.x * s, ys = q.y * s, zs = q.z * s;
  const double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
  const double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
  const double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
  const double m00 = 1.0 - (yy + zz), m10 = xy + wz, m20 = xz - wy, m21 = yz + wx, m22 = 1.0 - (xx + yy);
  if (fabs(m20) >= 1) {  // pitch at a singularity
    const double delta = atan2(m21, m22);
    *yaw = 0;
    *pitch = m20 < 0 ? 3.1415926535897932384626433832795029 / 2.0 : -3.1415926535897932384626433832795029 / 2.0;
    *roll = delta;
  } else {
    const double p = -tf_asin(m20);
    *pitch = p;
    *roll = atan2(m21 / cos(p), m22 / cos(p));
    *yaw = atan2(m10 / cos(p), m00 / cos(p));
  }
}

// The IMU half of transformUpdate (mapOptmization.h:1447-1474) on transformTobeMapped[0..1].
FBR_HD inline void imu_slerp_update(float tr[6], float imu_roll_init, float imu_pitch_init) {
  if (fabsf(imu_pitch_init) < 1.4) {
    const double imuWeight = 0.05;
    double rollMid, pitchMid, yawMid;
    TfQuat tq = tf_set_rpy(tr[0], 0, 0), iq = tf_set_rpy(imu_roll_init, 0, 0);
    tf_get_rpy(tf_slerp(tq, iq, imuWeight), &rollMid, &pitchMid, &yawMid);
    tr[0] = (float)rollMid;
    tq = tf_set_rpy(0, tr[1], 0);
    iq = tf_set_rpy(0, imu_pitch_init, 0);
    tf_get_rpy(tf_slerp(tq, iq, imuWeight), &rollMid, &pitchMid, &yawMid);
    tr[1] = (float)pitchMid;
  }
}

}  // namespace fbr
