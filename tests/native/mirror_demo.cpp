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
// argv[3] (optional): savePCDDirectory — the map is then loaded from $HOME<dir>cloudCorner.pcd /
//         cloudSurf.pcd (MapOptimization::loadGlobalMap, mapOptmization.h:245-260) instead of
//         from the input file's map points.
// exit  : 0 ok, 2 bad input, 3 fbr::Error (prints the status)
#include <cstdio>
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
}  // namespace

int main(int argc, char** argv) {
  if (argc != 3 && argc != 4) {
    fprintf(stderr, "usage: mirror_demo <in> <out> [savePCDDirectory]\n");
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
    if (argc == 4)
      node.matcher().loadGlobalMap(argv[3]);
    else
      node.matcher().setGlobalMap(cmap, smap);
    node.setPose(fbr::Affine3f::fromPose(pose0));
    for (int s = 0; s < n_scans; ++s) {
      double stamp;
      int64_t n;
      if (!rd(in, &stamp) || !rd(in, &n)) return 2;
      std::vector<fbr_point_xyzirt> pts(n);
      if (!rd(in, pts.data(), pts.size())) return 2;
      node.cloudHandler(pts.data(), n, stamp);
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
  } catch (const fbr::Error& e) {
    fprintf(stderr, "fbr::Error %d: %s\n", e.status, e.what());
    fclose(out);
    return 3;
  }
  fclose(out);
  fclose(in);
  return 0;
}
