/* fbr.hpp — header-only C++ host mirror of the reference's operator interface for the hot path,
 * layered on the C-ABI in fbr.h (libfbr_hip.so).  No ROS, PCL or Eigen types: the cloud_info
 * message is mirrored by fbr::CloudInfo (msg/cloud_info.msg fields on the path) and
 * Eigen::Affine3f by fbr::Affine3f (row-major 4x4 float, Eigen's matrix() element order).
 *
 *   reference (file:line)                                         mirror
 *   ImageProjection::cloudHandler / projectPointCloud /             fbr::ImageProjection::cloudHandler
 *     cloudExtraction (src/imageProjection.cpp:182-226, 583-670)    (+ the static pose chain :206-218)
 *   FeatureExtraction::featureExtra (src/featureExtraction.h:79)    fbr::FeatureExtraction::featureExtra
 *   mapOptimization::registration (src/mapOptmization.h:263-343)    fbr::MapOptimization::registration
 *
 * Error behaviour follows the reference: a scan that fails the cachePointCloud checks is dropped
 * (cloudHandler returns false); too few features leave the pose untouched (status in lastStats()).
 * Device or argument errors, which the reference has no analogue for, throw fbr::Error.
 *
 * The three objects share one fbr::Context (one HIP device + stream), because the device keeps the
 * projection, feature state and map resident between the stages — the reference's objects are
 * also members of one node (imageProjection.cpp:96-97).
 */
#ifndef FBR_HPP_
#define FBR_HPP_

#include <cstdint>
#include <cstdlib>
#include <deque>
#include <stdexcept>
#include <string>
#include <vector>

#include "fbr.h"

namespace fbr {

struct Error : std::runtime_error {
  int status;
  Error(int s, const char* what) : std::runtime_error(std::string(what) + ": " + fbr_strerror(s)), status(s) {}
};

inline void check(int s, const char* what) {
  if (s != FBR_OK) throw Error(s, what);
}

/* Eigen::Affine3f as a row-major 4x4 float matrix. */
struct Affine3f {
  float m[16];
  static Affine3f Identity() {
    Affine3f a{};
    a.m[0] = a.m[5] = a.m[10] = a.m[15] = 1.0f;
    return a;
  }
  /* pcl::getTransformation(x, y, z, roll, pitch, yaw) */
  static Affine3f fromPose(const float rpyxyz[6]) {
    Affine3f a;
    fbr_affine_from_pose(rpyxyz, a.m);
    return a;
  }
  /* pcl::getTranslationAndEulerAngles -> [roll, pitch, yaw, x, y, z] */
  void toPose(float rpyxyz[6]) const { fbr_pose_from_affine(m, rpyxyz); }
  float x() const { return m[3]; }
  float y() const { return m[7]; }
  float z() const { return m[11]; }
};

/* The cloud_info fields the path reads or writes (msg/cloud_info.msg:5-9, 32-34), plus the
 * feature mask (FeatureExtraction::cloudLabel, featureExtraction.h:41). */
struct CloudInfo {
  double stamp = 0.0;                         // header.stamp.toSec()
  std::vector<int32_t> startRingIndex;        // [N_SCAN]
  std::vector<int32_t> endRingIndex;          // [N_SCAN]
  std::vector<int32_t> pointColInd;           // [n]
  std::vector<float> pointRange;              // [n]
  std::vector<fbr_point_xyzi> cloud_deskewed; // [n] extractedCloud
  std::vector<fbr_point_xyzi> cloud_corner;   // cornerCloud (visit order)
  std::vector<fbr_point_xyzi> cloud_surface;  // surfaceCloud (per-ring DS, ring order)
  std::vector<int8_t> cloudLabel;             // [n] 1 corner, -1 picked surf, 0
};

/* One HIP device + stream + device-resident state (RAII over fbr_ctx). */
class Context {
 public:
  explicit Context(const fbr_params& p, int hip_device = 0) : p_(p) {
    check(fbr_create(&ctx_, &p_, hip_device), "fbr_create");
  }
  ~Context() {
    if (ctx_) fbr_destroy(ctx_);
  }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  fbr_ctx* get() const { return ctx_; }
  const fbr_params& params() const { return p_; }

 private:
  fbr_params p_;
  fbr_ctx* ctx_ = nullptr;
};

/* sensor_msgs/PointCloud2 as the node receives it (an owned copy: what cloudQueue holds,
 * imageProjection.cpp:233). */
struct PointCloud2 {
  struct Field {
    std::string name;
    uint32_t offset = 0;
    uint8_t datatype = FBR_PF_FLOAT32;
    uint32_t count = 1;
  };
  double stamp = 0.0;  // header.stamp.toSec()
  uint32_t height = 1, width = 0, point_step = 0, row_step = 0;
  bool is_bigendian = false, is_dense = true;
  std::vector<Field> fields;
  std::vector<uint8_t> data;
};

/* ImageProjection (imageProjection.cpp:29): projectPointCloud + cloudExtraction on the device. */
class ImageProjection {
 public:
  explicit ImageProjection(Context& c) : c_(c) {}
  ImageProjection(const ImageProjection&) = delete;

  /* cloudHandler's projection half (:197-199).  Returns false where cachePointCloud drops the
   * scan (:229-301: a ring outside [0, N_SCAN) is not an error there, only points are skipped;
   * an empty cloud yields an empty CloudInfo). */
  bool cloudHandler(const fbr_point_xyzirt* pts, int64_t n, double stamp, CloudInfo& info) {
    const int H = c_.params().n_scan;
    info.stamp = stamp;
    info.startRingIndex.assign(H, 0);
    info.endRingIndex.assign(H, 0);
    info.pointColInd.resize(n);
    info.pointRange.resize(n);
    info.cloud_deskewed.resize(n);
    int64_t n_out = 0;
    check(fbr_project(c_.get(), pts, n, info.startRingIndex.data(), info.endRingIndex.data(),
                      info.pointColInd.data(), info.pointRange.data(), info.cloud_deskewed.data(), &n_out),
          "fbr_project");
    info.pointColInd.resize(n_out);
    info.pointRange.resize(n_out);
    info.cloud_deskewed.resize(n_out);
    info.cloud_corner.clear();
    info.cloud_surface.clear();
    info.cloudLabel.clear();
    return true;
  }

  /* cachePointCloud (:229-301): the 2-message delay queue; returns false while it fills, else
   * makes the oldest message current (timeScanCur = its stamp). */
  bool cachePointCloud(const PointCloud2& msg) {
    cloudQueue_.push_back(msg);
    if (cloudQueue_.size() <= 2) return false;
    current_ = std::move(cloudQueue_.front());
    cloudQueue_.pop_front();
    return true;
  }

  /* cloudHandler's projection half on a raw message: the cache queue, then the message bytes are
   * unpacked on the device (fromROSMsg), checked (is_dense / ring -> fbr::Error with FBR_ERR_MSG
   * where the reference calls ros::shutdown()), and projected.  msgFlags() reports the warnings
   * (FBR_MSG_NO_TIME: the reference's "deskew function disabled" ROS_WARN). */
  bool cloudHandler(const PointCloud2& msg, CloudInfo& info) {
    if (!cachePointCloud(msg)) return false;
    std::vector<fbr_point_field> f(current_.fields.size());
    for (size_t k = 0; k < f.size(); ++k)
      f[k] = fbr_point_field{current_.fields[k].name.c_str(), current_.fields[k].offset, current_.fields[k].datatype,
                             current_.fields[k].count};
    fbr_pointcloud2 m;
    m.height = current_.height;
    m.width = current_.width;
    m.fields = f.data();
    m.n_fields = (int32_t)f.size();
    m.is_bigendian = current_.is_bigendian;
    m.point_step = current_.point_step;
    m.row_step = current_.row_step;
    m.data = current_.data.data();
    m.data_size = current_.data.size();
    m.is_dense = current_.is_dense;
    const int H = c_.params().n_scan;
    const int64_t n = (int64_t)current_.width * current_.height;
    info.stamp = current_.stamp;
    info.startRingIndex.assign(H, 0);
    info.endRingIndex.assign(H, 0);
    info.pointColInd.resize(n);
    info.pointRange.resize(n);
    info.cloud_deskewed.resize(n);
    int64_t n_out = 0;
    check(fbr_project_msg(c_.get(), &m, info.startRingIndex.data(), info.endRingIndex.data(), info.pointColInd.data(),
                          info.pointRange.data(), info.cloud_deskewed.data(), &n_out, &msg_flags_),
          "fbr_project_msg");
    info.pointColInd.resize(n_out);
    info.pointRange.resize(n_out);
    info.cloud_deskewed.resize(n_out);
    info.cloud_corner.clear();
    info.cloud_surface.clear();
    info.cloudLabel.clear();
    return true;
  }
  int msgFlags() const { return msg_flags_; }

  /* deskewInfo() enabled (imageProjection.cpp:189-191 uncommented): the table fbr_imu_deskew_info
   * built for the next scan; deskewPoint then runs inside the device compaction. */
  void setDeskew(const fbr_deskew_table& t) { check(fbr_set_deskew(c_.get(), &t, 1), "fbr_set_deskew"); }
  void clearDeskew() { check(fbr_set_deskew(c_.get(), nullptr, 0), "fbr_set_deskew"); }

 private:
  Context& c_;
  std::deque<PointCloud2> cloudQueue_;
  PointCloud2 current_;
  int msg_flags_ = 0;
};

/* FeatureExtraction (featureExtraction.h:19): featureExtra(cloud_info) on the projection the
 * context holds (the same scan ImageProjection just handled). */
class FeatureExtraction {
 public:
  explicit FeatureExtraction(Context& c) : c_(c) {}

  void featureExtra(CloudInfo& info) {
    const int64_t n = (int64_t)info.pointColInd.size();
    const int64_t corner_cap = 20 * 6 * (int64_t)c_.params().n_scan;
    info.cloudLabel.resize(n);
    info.cloud_corner.resize(corner_cap);
    info.cloud_surface.resize(n);
    int64_t nc = 0, ns = 0;
    check(fbr_extract_features(c_.get(), info.cloudLabel.data(), info.cloud_corner.data(), &nc,
                               info.cloud_surface.data(), &ns),
          "fbr_extract_features");
    info.cloud_corner.resize(nc);
    info.cloud_surface.resize(ns);
  }

 private:
  Context& c_;
};

/* mapOptimization (mapOptmization.h:54): prior map + registration(cloud_info, Affine3f&). */
class MapOptimization {
 public:
  explicit MapOptimization(Context& c) : c_(c) {}

  /* corner_GlobalMap / surf_GlobalMap as loaded from the PCDs (:245-260; the start-up VoxelGrid is
   * applied on the device). */
  void setGlobalMap(const std::vector<fbr_point_xyzi>& corner, const std::vector<fbr_point_xyzi>& surf) {
    check(fbr_set_map(c_.get(), corner.data(), (int64_t)corner.size(), surf.data(), (int64_t)surf.size()),
          "fbr_set_map");
  }

  /* The start-up block itself (:245-260): loadPCDFile(getenv("HOME") + savePCDDirectory +
   * "cloudCorner.pcd" / "cloudSurf.pcd") then the DS.  Unlike the reference (which ignores
   * loadPCDFile's return value and runs with an empty map), an unreadable file throws. */
  void loadGlobalMap(const std::string& savePCDDirectory) {
    const char* home = std::getenv("HOME");
    const std::string dir = std::string(home ? home : "") + savePCDDirectory;
    loadGlobalMapFiles(dir + "cloudCorner.pcd", dir + "cloudSurf.pcd");
  }
  void loadGlobalMapFiles(const std::string& corner_pcd, const std::string& surf_pcd) {
    check(fbr_load_map(c_.get(), corner_pcd.c_str(), surf_pcd.c_str()), "fbr_load_map");
  }

  /* registration (:263-343): mappingProcessInterval gate, getTranslationAndEulerAngles of the
   * guess, CropBox + DS + scan2MapOptimization on the device, getTransformation of the result. */
  void registration(const CloudInfo& info, Affine3f& pose_guess) {
    stats_ = fbr_reg_stats{};
    if (!(info.stamp - timeLastProcessing_ >= c_.params().mapping_process_interval)) {
      stats_.status = FBR_REG_SKIPPED_INTERVAL;
      return;
    }
    timeLastProcessing_ = info.stamp;
    float pose[6];
    pose_guess.toPose(pose);
    check(fbr_register(c_.get(), info.cloud_corner.data(), (int64_t)info.cloud_corner.size(),
                       info.cloud_surface.data(), (int64_t)info.cloud_surface.size(), pose, &stats_),
          "fbr_register");
    pose_guess = Affine3f::fromPose(pose);
  }

  const fbr_reg_stats& lastStats() const { return stats_; }

  /* LIO-SAM keyframe back-end (mapOptmization.h:857-978, 1667-1770): the caller's GTSAM step pushes
   * each key pose with its DS'd feature clouds and corrects poses after a loop closure;
   * extractSurroundingKeyFrames then makes the keyframe local map the registration map. */
  void addKeyFrame(const fbr_keypose& pose, const std::vector<fbr_point_xyzi>& corner,
                   const std::vector<fbr_point_xyzi>& surf) {
    check(fbr_keyframes_add(c_.get(), &pose, corner.data(), (int64_t)corner.size(), surf.data(), (int64_t)surf.size()),
          "fbr_keyframes_add");
  }
  void correctPose(int64_t index, const fbr_keypose& pose) {
    check(fbr_keyframes_set_pose(c_.get(), index, &pose), "fbr_keyframes_set_pose");
  }
  void extractSurroundingKeyFrames(double timeLaserCloudInfoLast, const fbr_keyframe_params& kp) {
    check(fbr_extract_surrounding_keyframes(c_.get(), timeLaserCloudInfoLast, &kp, nullptr, nullptr, nullptr),
          "fbr_extract_surrounding_keyframes");
  }

 private:
  Context& c_;
  double timeLastProcessing_ = -1.0;  // mapOptmization.h:135 (timeLastProcessing = -1)
  fbr_reg_stats stats_{};
};

/* The node-level chain of cloudHandler (:182-226): project -> featureExtra -> registration with
 * the static pose (step = identity, so pose = pose * step = pose). */
class Node {
 public:
  explicit Node(Context& c) : proj_(c), feat_(c), map_(c), pose_(Affine3f::Identity()) {}
  MapOptimization& matcher() { return map_; }
  const Affine3f& pose() const { return pose_; }
  void setPose(const Affine3f& p) { pose_ = p; }
  const CloudInfo& cloudInfo() const { return info_; }

  bool cloudHandler(const fbr_point_xyzirt* pts, int64_t n, double stamp) {
    if (!proj_.cloudHandler(pts, n, stamp, info_)) return false;
    feat_.featureExtra(info_);
    map_.registration(info_, pose_);
    return true;
  }
  /* The reference's entry point proper: cloudHandler(const sensor_msgs::PointCloud2ConstPtr&)
   * (:182-226), including the 2-message cache queue (returns false while it fills). */
  bool cloudHandler(const PointCloud2& msg) {
    if (!proj_.cloudHandler(msg, info_)) return false;
    feat_.featureExtra(info_);
    map_.registration(info_, pose_);
    return true;
  }
  ImageProjection& projection() { return proj_; }

 private:
  ImageProjection proj_;
  FeatureExtraction feat_;
  MapOptimization map_;
  Affine3f pose_;
  CloudInfo info_;
};

}  // namespace fbr

#endif /* FBR_HPP_ */
