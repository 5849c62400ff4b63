// fbr_imu.cpp — host side of the IMU deskew path.
//
// Reference: imuConverter (include/utility.h:219-253), which ImageProjection::imuHandler applies to
// every IMU message before queueing it (src/imageProjection.cpp:148-156), and deskewInfo +
// imuDeskewInfo (:303-393), which turn the queued samples into the per-scan rotation table that
// deskewPoint interpolates (:494-580; on the device in k_project.hip).  imuDeskewInfo is a serial
// pass over the ~20 samples of one scan (200 Hz IMU, 10 Hz lidar) and stays on the host, as in the
// reference.  Third-party semantics restated (double):
//   Eigen 3.3 Matrix3d * Vector3d     coefficient-based product, row sums x0 + (x1 + x2)
//   Eigen Quaterniond(Matrix3d)       quaternionbase_assign_impl<Other, 3, 3>
//   Eigen quaternion product          the generic quat_product formula (the SSE2 specialisation
//                                     groups the same products differently: rounding-level)
//   tf::quaternionMsgToTF             normalises when |length2 - 1| > QUATERNION_TOLERANCE (0.1)
//   tf::Matrix3x3(q).getRPY           fbr_imu.h
#include <cmath>
#include <cstring>

#include "fbr.h"
#include "fbr_imu.h"

namespace {

double sum3d(double a, double b, double c) { return a + (b + c); }

// Eigen Quaterniond(const Matrix3d&); q = {x, y, z, w}
void quat_from_matrix(const double m[9], double q[4]) {
  auto M = [&](int r, int c) { return m[3 * r + c]; };
  double t = sum3d(M(0, 0), M(1, 1), M(2, 2));  // trace()
  if (t > 0.0) {
    t = std::sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (M(2, 1) - M(1, 2)) * t;
    q[1] = (M(0, 2) - M(2, 0)) * t;
    q[2] = (M(1, 0) - M(0, 1)) * t;
  } else {
    int i = 0;
    if (M(1, 1) > M(0, 0)) i = 1;
    if (M(2, 2) > M(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (M(k, j) - M(j, k)) * t;
    q[j] = (M(j, i) + M(i, j)) * t;
    q[k] = (M(k, i) + M(i, k)) * t;
  }
}

// Eigen a * b, {x, y, z, w}
void quat_mul(const double a[4], const double b[4], double o[4]) {
  o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

// imuRPY2rosRPY (utility.h:292-303): tf::quaternionMsgToTF, then Matrix3x3::getRPY
void imu_rpy(const fbr_imu_sample& s, double* roll, double* pitch, double* yaw) {
  fbr::TfQuat q{s.orientation[0], s.orientation[1], s.orientation[2], s.orientation[3]};
  const double l2 = fbr::tf_dot(q, q);
  if (std::fabs(l2 - 1) > 0.1f) {  // QUATERNION_TOLERANCE: normalize() = *this *= 1 / length()
    const double inv = 1.0 / std::sqrt(l2);
    q.x *= inv;
    q.y *= inv;
    q.z *= inv;
    q.w *= inv;
  }
  fbr::tf_get_rpy(q, roll, pitch, yaw);
}

}  // namespace

extern "C" {

int fbr_imu_convert(const fbr_imu_extrinsics* ext, const fbr_imu_sample* in, fbr_imu_sample* out) {
  if (!ext || !in || !out) return FBR_ERR_INVALID_ARG;
  fbr_imu_sample o = *in;
  const double* R = ext->ext_rot;
  for (int r = 0; r < 3; ++r) {  // acc = extRot * acc; gyr = extRot * gyr (:224-234)
    o.linear_acceleration[r] = sum3d(R[3 * r] * in->linear_acceleration[0], R[3 * r + 1] * in->linear_acceleration[1],
                                     R[3 * r + 2] * in->linear_acceleration[2]);
    o.angular_velocity[r] = sum3d(R[3 * r] * in->angular_velocity[0], R[3 * r + 1] * in->angular_velocity[1],
                                  R[3 * r + 2] * in->angular_velocity[2]);
  }
  double qe[4], qf[4];
  quat_from_matrix(ext->ext_rpy, qe);             // extQRPY = Quaterniond(extRPY) (utility.h:178)
  quat_mul(qe, in->orientation, qf);              // q_final = extQRPY * q_from (:238-243)
  for (int k = 0; k < 4; ++k) o.orientation[k] = qf[k];
  if (std::sqrt(qf[0] * qf[0] + qf[1] * qf[1] + qf[2] * qf[2] + qf[3] * qf[3]) < 0.1)  // :246-250
    return FBR_ERR_INVALID_ARG;
  *out = o;
  return FBR_OK;
}

int fbr_imu_deskew_info(const fbr_imu_sample* q, int64_t n, double timeScanCur, double timeScanNext,
                        fbr_deskew_table* out, int64_t* n_pop) {
  if (!out || n < 0 || (n && !q)) return FBR_ERR_INVALID_ARG;
  // everything but the carried cloudInfo.imu*Init fields
  const float ri = out->imu_roll_init, pi = out->imu_pitch_init, yi = out->imu_yaw_init;
  std::memset(out, 0, sizeof(*out));
  out->imu_roll_init = ri;
  out->imu_pitch_init = pi;
  out->imu_yaw_init = yi;
  out->time_scan_cur = timeScanCur;
  if (n_pop) *n_pop = 0;
  // deskewInfo (:308-314)
  if (n == 0 || q[0].stamp > timeScanCur || q[n - 1].stamp < timeScanNext) {
    out->status = FBR_DESKEW_WAIT_IMU;
    return FBR_OK;
  }
  out->status = FBR_DESKEW_READY;
  // imuDeskewInfo (:323-393)
  int64_t b = 0;
  while (b < n && q[b].stamp < timeScanCur - 0.01) ++b;  // pop_front (:328-335)
  if (n_pop) *n_pop = b;
  if (b == n) return FBR_OK;
  int cur = 0;
  for (int64_t i = b; i < n; ++i) {
    const double currentImuTime = q[i].stamp;
    if (currentImuTime <= timeScanCur) {  // imuRPY2rosRPY into cloudInfo.imu*Init (float)
      double r, p, y;
      imu_rpy(q[i], &r, &p, &y);
      out->imu_roll_init = (float)r;
      out->imu_pitch_init = (float)p;
      out->imu_yaw_init = (float)y;
    }
    if (currentImuTime > timeScanNext + 0.01) break;
    if (cur >= FBR_IMU_QUEUE) return FBR_ERR_CAPACITY;
    if (cur == 0) {
      out->imu_rot_x[0] = 0;
      out->imu_rot_y[0] = 0;
      out->imu_rot_z[0] = 0;
      out->imu_time[0] = currentImuTime;
      ++cur;
      continue;
    }
    const double timeDiff = currentImuTime - out->imu_time[cur - 1];
    out->imu_rot_x[cur] = out->imu_rot_x[cur - 1] + q[i].angular_velocity[0] * timeDiff;
    out->imu_rot_y[cur] = out->imu_rot_y[cur - 1] + q[i].angular_velocity[1] * timeDiff;
    out->imu_rot_z[cur] = out->imu_rot_z[cur - 1] + q[i].angular_velocity[2] * timeDiff;
    out->imu_time[cur] = currentImuTime;
    ++cur;
  }
  --cur;
  out->imu_pointer_cur = cur < 0 ? 0 : cur;
  if (cur <= 0) return FBR_OK;
  out->imu_available = 1;
  return FBR_OK;
}

}  // extern "C"
