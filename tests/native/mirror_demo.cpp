// mirror_demo.cpp — drives the C++ host mirror (include/fbr.hpp) the way the reference's node
// drives its objects: ImageProjection::cloudHandler -> FeatureExtraction::featureExtra ->
// mapOptimization::registration with the static Affine3f pose chain (imageProjection.cpp:182-226).
// Test harness only: tests/test_cpp_mirror.py writes the input file, runs this program and
// checks the output file against the CPU oracle.
//
// input : int32 H, W, n_scans; int64 n_corner_map, n_surf_map; map points (16 B each);
//         float pose0[6]; per scan { double stamp; int64 n; n x 24 B fbr_point_xyzirt }
// output: per scan { int64 n_out; int32 start[H], end[H]; int32 col[n_out]; float range[n_out];
//         int8 label[n_out]; int64 nc; nc x 16 B; int64 ns; ns x 16 B; float affine[16];
//         fbr_reg_stats }
// options: --pcd DIR  the map is loaded from $HOME<DIR>cloudCorner.pcd / cloudSurf.pcd
//                      (MapOptimization::loadGlobalMap, mapOptmization.h:245-260) instead of from
//                      the input file's map points;
//          --msg       each scan is sent as a sensor_msgs/PointCloud2 (Velodyne 32-B records)
//                      through Node::cloudHandler(msg) with the 2-message cache queue; two extra
//                      messages after the last scan flush the queue, so the output still holds
//                      one record per input scan, in input order.
// exit  : 0 ok, 2 bad input, 3 fbr::Error (prints the status)
#include <cstdio>
#include <cstring>
#include <vector>

#include "fbr.hpp"

namespace {
template <class T>
bool rd(FILE* f, T* p, size_t n = 1) {
  return fread(p, sizeof(T), n, f) == n;
}
template <class T>
void wr(FILE* f, const T* p, size_t n = 1) {
  if (n) fwrite(p, sizeof(T), n, f);
}

void write_record(FILE* out, fbr::Node& node, int H) {
  const fbr::CloudInfo& ci = node.cloudInfo();
  const int64_t n_out = (int64_t)ci.pointColInd.size();
  wr(out, &n_out);
  wr(out, ci.startRingIndex.data(), H);
  wr(out, ci.endRingIndex.data(), H);
  wr(out, ci.pointColInd.data(), n_out);
  wr(out, ci.pointRange.data(), n_out);
  wr(out, ci.cloudLabel.data(), n_out);
  const int64_t nc = (int64_t)ci.cloud_corner.size(), ns = (int64_t)ci.cloud_surface.size();
  wr(out, &nc);
  wr(out, ci.cloud_corner.data(), nc);
  wr(out, &ns);
  wr(out, ci.cloud_surface.data(), ns);
  wr(out, node.pose().m, 16);
  const fbr_reg_stats st = node.matcher().lastStats();
  wr(out, &st);
}

// PointXYZIRT as a Velodyne driver publishes it: x y z @0/4/8, intensity @16, ring u16 @20,
// time @24, 32-B records.
fbr::PointCloud2 velodyne_msg(const std::vector<fbr_point_xyzirt>& pts, double stamp) {
  fbr::PointCloud2 m;
  m.stamp = stamp;
  m.width = (uint32_t)pts.size();
  m.point_step = 32;
  m.row_step = 32 * m.width;
  m.fields = {{"x", 0, FBR_PF_FLOAT32, 1}, {"y", 4, FBR_PF_FLOAT32, 1}, {"z", 8, FBR_PF_FLOAT32, 1},
              {"intensity", 16, FBR_PF_FLOAT32, 1}, {"ring", 20, FBR_PF_UINT16, 1}, {"time", 24, FBR_PF_FLOAT32, 1}};
  m.data.assign(32 * pts.size(), 0);
  for (size_t i = 0; i < pts.size(); ++i) {
    uint8_t* d = m.data.data() + 32 * i;
    memcpy(d, &pts[i].x, 12);
    memcpy(d + 16, &pts[i].intensity, 4);
    memcpy(d + 20, &pts[i].ring, 2);
    memcpy(d + 24, &pts[i].time, 4);
  }
  return m;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: mirror_demo <in> <out> [--pcd DIR] [--msg]\n");
    return 2;
  }
  const char* pcd_dir = nullptr;
  bool as_msg = false;
  for (int a = 3; a < argc; ++a) {
    if (!strcmp(argv[a], "--pcd") && a + 1 < argc)
      pcd_dir = argv[++a];
    else if (!strcmp(argv[a], "--msg"))
      as_msg = true;
    else
      return 2;
  }
  FILE* in = fopen(argv[1], "rb");
  if (!in) return 2;
  int32_t H, W, n_scans;
  int64_t nc_map, ns_map;
  if (!rd(in, &H) || !rd(in, &W) || !rd(in, &n_scans) || !rd(in, &nc_map) || !rd(in, &ns_map)) return 2;
  std::vector<fbr_point_xyzi> cmap(nc_map), smap(ns_map);
  float pose0[6];
  if (!rd(in, cmap.data(), cmap.size()) || !rd(in, smap.data(), smap.size()) || !rd(in, pose0, 6)) return 2;
  FILE* out = fopen(argv[2], "wb");
  if (!out) return 2;
  try {
    fbr_params p;
    fbr_params_default(&p);
    p.n_scan = H;
    p.horizon_scan = W;
    fbr::Context ctx(p, 0);
    fbr::Node node(ctx);
    if (pcd_dir)
      node.matcher().loadGlobalMap(pcd_dir);
    else
      node.matcher().setGlobalMap(cmap, smap);
    std::vector<fbr::PointCloud2> msgs;
    node.setPose(fbr::Affine3f::fromPose(pose0));
    for (int s = 0; s < n_scans; ++s) {
      double stamp;
      int64_t n;
      if (!rd(in, &stamp) || !rd(in, &n)) return 2;
      std::vector<fbr_point_xyzirt> pts(n);
      if (!rd(in, pts.data(), pts.size())) return 2;
      if (!as_msg) {
        node.cloudHandler(pts.data(), n, stamp);
        write_record(out, node, H);
        continue;
      }
      msgs.push_back(velodyne_msg(pts, stamp));
      if (node.cloudHandler(msgs.back())) write_record(out, node, H);
    }
    for (int k = 0; as_msg && k < 2; ++k) {  // flush the cache queue
      fbr::PointCloud2 m = msgs.back();
      m.stamp += 1.0 + k;
      if (node.cloudHandler(m)) write_record(out, node, H);
    }
  } catch (const fbr::Error& e) {
    fprintf(stderr, "fbr::Error %d: %s\n", e.status, e.what());
    fclose(out);
    return 3;
  }
  fclose(out);
  fclose(in);
  return 0;
}


