// fbr_msg.cpp — sensor_msgs/PointCloud2 wire adapter on the host side of the boundary
// (SURVEY §8(f) row 2).
//
// Reference: ImageProjection::cachePointCloud (src/imageProjection.cpp:229-301) converts the
// message with pcl::fromROSMsg into PointXYZIRT (:253, layout :8-21), rejects non-dense clouds
// (:256-260) and clouds without a "ring" field (:264-281), and warns when there is no "time" field
// (:285-298).  publishCloud (include/utility.h:255-264) goes the other way with pcl::toROSMsg of a
// PointXYZI cloud.  PCL (1.8) semantics restated here:
//   * a point-type field is mapped from the message field with the same name, the same datatype,
//     and count equal to the type's count (or 0 for a scalar); otherwise it stays 0 (the points are
//     value-initialised by vector::resize);
//   * points are read row-major: point (r, c) at data[r * row_step + c * point_step];
//   * is_bigendian is not consulted.
#include <cstring>

#include "fbr.h"
#include "fbr_msg.h"

namespace fbr {

namespace {

struct Want {
  const char* name;
  uint8_t datatype;
  int size;
};
constexpr Want kWant[kMsgFields] = {{"x", FBR_PF_FLOAT32, 4},         {"y", FBR_PF_FLOAT32, 4},
                                    {"z", FBR_PF_FLOAT32, 4},         {"intensity", FBR_PF_FLOAT32, 4},
                                    {"ring", FBR_PF_UINT16, 2},       {"time", FBR_PF_FLOAT32, 4}};

}  // namespace

int resolve_msg(const fbr_pointcloud2* m, MsgLayout* L) {
  if (!m || !L || m->n_fields < 0 || (m->n_fields && !m->fields)) return FBR_ERR_INVALID_ARG;
  L->width = m->width;
  L->height = m->height;
  L->point_step = m->point_step;
  L->row_step = m->row_step;
  L->n = (int64_t)m->width * (int64_t)m->height;
  L->flags = 0;
  L->bytes = 0;
  bool has_ring = false, has_time = false;
  for (int k = 0; k < kMsgFields; ++k) L->off[k] = -1;
  for (int f = 0; f < m->n_fields; ++f) {
    const fbr_point_field& F = m->fields[f];
    if (!F.name) return FBR_ERR_INVALID_ARG;
    if (!std::strcmp(F.name, "ring")) has_ring = true;
    if (!std::strcmp(F.name, "time")) has_time = true;
    for (int k = 0; k < kMsgFields; ++k) {
      if (L->off[k] >= 0 || std::strcmp(F.name, kWant[k].name)) continue;
      if (F.datatype != kWant[k].datatype || (F.count != 1 && F.count != 0)) continue;
      if ((uint64_t)F.offset + kWant[k].size > m->point_step) return FBR_ERR_INVALID_ARG;
      L->off[k] = (int32_t)F.offset;
    }
  }
  // cachePointCloud's checks, in the reference's order
  if (!m->is_dense) return FBR_ERR_MSG;
  if (!has_ring) return FBR_ERR_MSG;
  if (!has_time) L->flags |= FBR_MSG_NO_TIME;
  if (L->off[kMsgRing] < 0) L->flags |= FBR_MSG_RING_UNMAPPED;
  if (L->off[kMsgX] < 0 || L->off[kMsgY] < 0 || L->off[kMsgZ] < 0 || L->off[kMsgI] < 0)
    L->flags |= FBR_MSG_XYZI_UNMAPPED;
  if (L->n > 0) {
    if ((uint64_t)m->width * m->point_step > m->row_step && m->height > 1) return FBR_ERR_INVALID_ARG;
    L->bytes = (uint64_t)(m->height - 1) * m->row_step + (uint64_t)m->width * m->point_step;
    if (!m->data || m->data_size < L->bytes) return FBR_ERR_INVALID_ARG;
  }
  return FBR_OK;
}

}  // namespace fbr

extern "C" {

int fbr_msg_to_points(const fbr_pointcloud2* msg, fbr_point_xyzirt* out, int64_t cap, int64_t* n,
                      int32_t* msg_flags) {
  if (!n) return FBR_ERR_INVALID_ARG;
  fbr::MsgLayout L;
  const int rc = fbr::resolve_msg(msg, &L);
  if (rc) return rc;
  *n = L.n;
  if (msg_flags) *msg_flags = L.flags;
  if (!out) return FBR_OK;
  if (cap < L.n) return FBR_ERR_CAPACITY;
  for (uint32_t r = 0; r < L.height; ++r) {
    for (uint32_t c = 0; c < L.width; ++c) {
      const uint8_t* p = msg->data + (uint64_t)r * L.row_step + (uint64_t)c * L.point_step;
      fbr_point_xyzirt q;
      std::memset(&q, 0, sizeof(q));
      float* xyzi = &q.x;
      for (int k = 0; k < 4; ++k)
        if (L.off[k] >= 0) std::memcpy(xyzi + k, p + L.off[k], 4);
      if (L.off[fbr::kMsgRing] >= 0) std::memcpy(&q.ring, p + L.off[fbr::kMsgRing], 2);
      if (L.off[fbr::kMsgTime] >= 0) std::memcpy(&q.time, p + L.off[fbr::kMsgTime], 4);
      out[(int64_t)r * L.width + c] = q;
    }
  }
  return FBR_OK;
}

int fbr_points_to_msg_data(const fbr_point_xyzi* pts, int64_t n, uint8_t* data) {
  if (n < 0 || (n && (!pts || !data))) return FBR_ERR_INVALID_ARG;
  const float one = 1.0f;
  for (int64_t i = 0; i < n; ++i) {
    uint8_t* d = data + 32 * i;
    std::memset(d, 0, 32);
    std::memcpy(d, &pts[i].x, 12);
    std::memcpy(d + 12, &one, 4);  // PCL_ADD_POINT4D's data[3]
    std::memcpy(d + 16, &pts[i].intensity, 4);
  }
  return FBR_OK;
}

}  // extern "C"
