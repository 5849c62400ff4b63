// fbr_msg.h — internal: PointCloud2 -> PointXYZIRT field mapping shared by the host converter
// (fbr_msg.cpp) and the device unpack path (fbr_api.hip / k_project.hip).
#pragma once
#include <cstdint>

#include "fbr.h"

namespace fbr {

// Byte offsets inside one message point of the PointXYZIRT fields (-1 = unmapped, read as 0).
enum { kMsgX = 0, kMsgY, kMsgZ, kMsgI, kMsgRing, kMsgTime, kMsgFields };

struct MsgLayout {
  int64_t n;              // width * height
  uint32_t width, height, point_step, row_step;
  int32_t off[kMsgFields];
  int32_t flags;          // FBR_MSG_*
  uint64_t bytes;         // bytes of data the points span ((height-1)*row_step + width*point_step)
};

// pcl::fromROSMsg's createMapping (name + datatype + count) and cachePointCloud's checks.
// Returns FBR_OK, FBR_ERR_INVALID_ARG (inconsistent sizes) or FBR_ERR_MSG.
int resolve_msg(const fbr_pointcloud2* msg, MsgLayout* L);

}  // namespace fbr
