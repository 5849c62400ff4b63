// fbr_synth.cpp — deterministic synthetic lidar scans and prior feature maps (host C++).
//
// Input generator for tests and bench.py (BASELINE.md "Configs as concrete synthetic inputs",
// SURVEY.md §8d).  Not part of the registration hot path.  A procedural scene (ground plane,
// yaw-rotated box buildings, box cars, thin vertical poles) is ray-cast analytically for a
// multi-beam spinning lidar; points are emitted in firing order (column-major) with azimuth
// jitter, N(0, 1 cm) range noise, 5 % dropouts and 0.5 % sub-1 m returns, exactly the shape the
// reference's projectPointCloud() consumes (imageProjection.cpp:583-640).  The prior map is
// sampled from the same scene surfaces (surf) and vertical edges / pole axes (corner), in the
// world frame, like the cloudCorner.pcd / cloudSurf.pcd the reference loads
// (mapOptmization.h:247-248).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/fbr.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) {}
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  double uni(double a, double b) { return a + (b - a) * uni(); }
  double normal() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
};

struct Box {  // yaw-rotated box standing on the ground
  double cx, cy, hx, hy, h, yaw, c, s;
};
struct Pole {
  double x, y, r, h;
};
struct Tree {  // canopy sphere on a pole trunk
  double x, y, z, r;
};

struct Scene {
  std::vector<Box> boxes;  // buildings then cars
  int n_buildings = 0;
  std::vector<Pole> poles;
  std::vector<Tree> trees;
  double radius = 60.0;
};

bool hit_box(const Box& b, const double o[3], const double d[3], double& t) {
  // ray into the box frame (rotate by -yaw about the box centre)
  double ox = o[0] - b.cx, oy = o[1] - b.cy;
  double lx = b.c * ox + b.s * oy, ly = -b.s * ox + b.c * oy, lz = o[2];
  double dx = b.c * d[0] + b.s * d[1], dy = -b.s * d[0] + b.c * d[1], dz = d[2];
  double tmin = 0.0, tmax = 1e30;
  const double lo[3] = {-b.hx, -b.hy, 0.0}, hi[3] = {b.hx, b.hy, b.h};
  const double oo[3] = {lx, ly, lz}, dd[3] = {dx, dy, dz};
  for (int a = 0; a < 3; ++a) {
    if (std::fabs(dd[a]) < 1e-12) {
      if (oo[a] < lo[a] || oo[a] > hi[a]) return false;
    } else {
      double t1 = (lo[a] - oo[a]) / dd[a], t2 = (hi[a] - oo[a]) / dd[a];
      if (t1 > t2) std::swap(t1, t2);
      if (t1 > tmin) tmin = t1;
      if (t2 < tmax) tmax = t2;
      if (tmin > tmax) return false;
    }
  }
  if (tmin <= 1e-6) return false;  // origin inside or behind
  t = tmin;
  return true;
}

bool hit_pole(const Pole& p, const double o[3], const double d[3], double& t) {
  double ox = o[0] - p.x, oy = o[1] - p.y;
  double a = d[0] * d[0] + d[1] * d[1];
  if (a < 1e-12) return false;
  double b = 2 * (ox * d[0] + oy * d[1]);
  double c = ox * ox + oy * oy - p.r * p.r;
  double disc = b * b - 4 * a * c;
  if (disc < 0) return false;
  double tt = (-b - std::sqrt(disc)) / (2 * a);
  if (tt <= 1e-6) return false;
  double z = o[2] + tt * d[2];
  if (z < 0 || z > p.h) return false;
  t = tt;
  return true;
}

bool hit_sphere(const Tree& s, const double o[3], const double d[3], double& t) {
  double ox = o[0] - s.x, oy = o[1] - s.y, oz = o[2] - s.z;
  double b = ox * d[0] + oy * d[1] + oz * d[2];
  double c = ox * ox + oy * oy + oz * oz - s.r * s.r;
  double disc = b * b - c;
  if (disc < 0) return false;
  double tt = -b - std::sqrt(disc);
  if (tt <= 1e-6) return false;
  t = tt;
  return true;
}

void build_scene(uint64_t seed, Scene& sc) {
  Rng rng(seed ^ 0x5CE4E5CE4Eull);
  sc.boxes.clear();
  sc.poles.clear();
  sc.trees.clear();
  // buildings in an annulus 18..55 m around the origin
  const int nb = 36;
  for (int i = 0; i < nb; ++i) {
    double ang = 2 * M_PI * (i + rng.uni(0.1, 0.9)) / nb;
    double rr = rng.uni(15.0, 38.0);
    Box b;
    b.hx = rng.uni(2.5, 7.0);
    b.hy = rng.uni(2.5, 7.0);
    b.h = rng.uni(6.0, 20.0);
    b.cx = rr * std::cos(ang);
    b.cy = rr * std::sin(ang);
    b.yaw = rng.uni(-M_PI, M_PI);
    b.c = std::cos(b.yaw);
    b.s = std::sin(b.yaw);
    sc.boxes.push_back(b);
  }
  sc.n_buildings = nb;
  // cars 9..16 m
  for (int i = 0; i < 30; ++i) {
    double ang = rng.uni(-M_PI, M_PI), rr = rng.uni(10.0, 16.0);
    Box b;
    b.hx = 2.25;
    b.hy = 0.9;
    b.h = 1.5;
    b.cx = rr * std::cos(ang);
    b.cy = rr * std::sin(ang);
    b.yaw = rng.uni(-M_PI, M_PI);
    b.c = std::cos(b.yaw);
    b.s = std::sin(b.yaw);
    sc.boxes.push_back(b);
  }
  // poles 4..45 m
  for (int i = 0; i < 50; ++i) {
    double ang = rng.uni(-M_PI, M_PI), rr = rng.uni(9.5, 45.0);
    Pole p;
    p.x = rr * std::cos(ang);
    p.y = rr * std::sin(ang);
    p.r = rng.uni(0.05, 0.15);
    p.h = rng.uni(3.0, 8.0);
    sc.poles.push_back(p);
  }
  // trees 10..40 m: trunk pole + canopy sphere
  for (int i = 0; i < 30; ++i) {
    double ang = rng.uni(-M_PI, M_PI), rr = rng.uni(10.0, 40.0);
    Pole p;
    p.x = rr * std::cos(ang);
    p.y = rr * std::sin(ang);
    p.r = rng.uni(0.12, 0.25);
    p.h = rng.uni(2.5, 3.5);
    sc.poles.push_back(p);
    Tree t{p.x, p.y, p.h + rng.uni(1.2, 2.5), rng.uni(1.5, 2.8)};
    sc.trees.push_back(t);
  }
}

void beam_table(int H, std::vector<double>& el) {
  el.resize(H);
  if (H == 16) {
    for (int r = 0; r < H; ++r) el[r] = -15.0 + 2.0 * r;
  } else if (H == 64) {
    for (int r = 0; r < H; ++r) el[r] = -24.8 + (2.0 + 24.8) * r / (H - 1);  // kitti2bag.py:242-243
  } else if (H == 128) {
    for (int r = 0; r < H; ++r) el[r] = -22.5 + 45.0 * r / (H - 1);
  } else {
    for (int r = 0; r < H; ++r) el[r] = -25.0 + 40.0 * r / (H > 1 ? H - 1 : 1);
  }
}

// R = Rz(yaw) Ry(pitch) Rx(roll), double precision
void rot(const double rpy[3], double R[3][3]) {
  double A = std::cos(rpy[2]), B = std::sin(rpy[2]), C = std::cos(rpy[1]), D = std::sin(rpy[1]),
         E = std::cos(rpy[0]), F = std::sin(rpy[0]);
  R[0][0] = A * C; R[0][1] = A * D * F - B * E; R[0][2] = B * F + A * D * E;
  R[1][0] = B * C; R[1][1] = A * E + B * D * F; R[1][2] = B * D * E - A * F;
  R[2][0] = -D;    R[2][1] = C * F;             R[2][2] = C * E;
}

}  // namespace

extern "C" {

struct fbr_synth_opts {
  double range_noise;     // 0.01 m
  double dropout;         // 0.05
  double short_return;    // 0.005
  double max_range;       // 100 m
  double az_offset;       // 0.42 cells: some jittered azimuths round into the next column
  double az_jitter;       // 0.1 cells (0.02 deg at 1800 columns)
};

void fbr_synth_default_opts(fbr_synth_opts* o) {
  o->range_noise = 0.01;
  o->dropout = 0.05;
  o->short_return = 0.005;
  o->max_range = 100.0;
  o->az_offset = 0.42;
  o->az_jitter = 0.1;
}

// Ray-cast one scan of an H x W spinning lidar at world pose [roll,pitch,yaw,x,y,z].
// out must hold H*W points; returns the number emitted.
int64_t fbr_synth_scan(uint64_t scene_seed, int H, int W, const double pose[6], uint64_t seed,
                       const fbr_synth_opts* opts, fbr_point_xyzirt* out) {
  Scene sc;
  build_scene(scene_seed, sc);
  fbr_synth_opts o;
  if (opts) o = *opts; else fbr_synth_default_opts(&o);
  std::vector<double> el;
  beam_table(H, el);
  double R[3][3];
  rot(pose, R);
  const double org[3] = {pose[3], pose[4], pose[5]};
  Rng rng(seed);
  int64_t n = 0;
  const double cell = 2 * M_PI / W;
  for (int c = 0; c < W; ++c) {
    for (int r = 0; r < H; ++r) {
      double az = (c + o.az_offset + rng.uni(-o.az_jitter, o.az_jitter)) * cell;
      double e = el[r] * M_PI / 180.0;
      double dl[3] = {std::cos(e) * std::cos(az), std::cos(e) * std::sin(az), std::sin(e)};
      double dw[3];
      for (int i = 0; i < 3; ++i) dw[i] = R[i][0] * dl[0] + R[i][1] * dl[1] + R[i][2] * dl[2];
      double best = 1e30, t;
      if (dw[2] < -1e-9) {
        t = -org[2] / dw[2];
        if (t > 0 && t < best) best = t;
      }
      for (const Box& b : sc.boxes)
        if (hit_box(b, org, dw, t) && t < best) best = t;
      for (const Pole& p : sc.poles)
        if (hit_pole(p, org, dw, t) && t < best) best = t;
      for (const Tree& tr : sc.trees)
        if (hit_sphere(tr, org, dw, t) && t < best) best = t;
      double u_drop = rng.uni(), u_short = rng.uni(), nz = rng.normal(), inten = rng.uni(0.0, 255.0);
      if (best > o.max_range) continue;
      if (u_drop < o.dropout) continue;
      double rg = best + o.range_noise * nz;
      if (u_short < o.short_return) rg = 0.3 + 0.69 * rng.uni();
      fbr_point_xyzirt& q = out[n++];
      q.x = (float)(rg * dl[0]);
      q.y = (float)(rg * dl[1]);
      q.z = (float)(rg * dl[2]);
      q.intensity = (float)inten;
      q.ring = (uint16_t)r;
      q.pad_ = 0;
      q.time = (float)(0.1 * c / W);
    }
  }
  return n;
}

// Sample a prior feature map of the scene in the world frame.  surf: ground disk + building and
// car faces at `surf_density` points/m^2; corner: building vertical edges and pole axes at
// `corner_density` points/m.  Returns counts through n_corner / n_surf; pass NULL buffers to query
// the counts first (the same seed gives the same counts).
int fbr_synth_map(uint64_t scene_seed, uint64_t seed, double map_radius, double surf_density,
                  double corner_density, fbr_point_xyzi* corner, int64_t* n_corner,
                  fbr_point_xyzi* surf, int64_t* n_surf) {
  Scene sc;
  build_scene(scene_seed, sc);
  Rng rng(seed);
  int64_t nc = 0, ns = 0;
  auto put_s = [&](double x, double y, double z) {
    if (surf) surf[ns] = fbr_point_xyzi{(float)x, (float)y, (float)z, (float)rng.uni(0.0, 255.0)};
    else rng.next();
    ++ns;
  };
  auto put_c = [&](double x, double y, double z) {
    if (corner) corner[nc] = fbr_point_xyzi{(float)x, (float)y, (float)z, (float)rng.uni(0.0, 255.0)};
    else rng.next();
    ++nc;
  };
  auto count_of = [&](double expected) {
    int64_t k = (int64_t)std::floor(expected);
    if (rng.uni() < expected - k) ++k;
    return k;
  };
  auto inside_any_box = [&](double x, double y) {
    for (const Box& b : sc.boxes) {
      double ox = x - b.cx, oy = y - b.cy;
      double lx = b.c * ox + b.s * oy, ly = -b.s * ox + b.c * oy;
      if (std::fabs(lx) < b.hx && std::fabs(ly) < b.hy) return true;
    }
    return false;
  };
  // ground disk
  {
    int64_t k = count_of(M_PI * map_radius * map_radius * surf_density);
    for (int64_t i = 0; i < k; ++i) {
      double rr = map_radius * std::sqrt(rng.uni()), a = rng.uni(-M_PI, M_PI);
      double x = rr * std::cos(a), y = rr * std::sin(a);
      double zn = 0.01 * rng.normal();
      if (inside_any_box(x, y)) { rng.next(); continue; }
      put_s(x, y, zn);
    }
  }
  // box faces (4 vertical faces; cars also their roof)
  for (size_t bi = 0; bi < sc.boxes.size(); ++bi) {
    const Box& b = sc.boxes[bi];
    if (std::hypot(b.cx, b.cy) > map_radius + 10) continue;
    for (int f = 0; f < 4; ++f) {
      double len = (f < 2) ? 2 * b.hy : 2 * b.hx;
      int64_t k = count_of(len * b.h * surf_density);
      for (int64_t i = 0; i < k; ++i) {
        double u = rng.uni(-0.5, 0.5) * len, z = rng.uni(0.0, b.h), w = 0.01 * rng.normal();
        double lx, ly;
        if (f == 0) lx = b.hx + w, ly = u;
        else if (f == 1) lx = -b.hx - w, ly = u;
        else if (f == 2) lx = u, ly = b.hy + w;
        else lx = u, ly = -b.hy - w;
        put_s(b.cx + b.c * lx - b.s * ly, b.cy + b.s * lx + b.c * ly, z);
      }
    }
    if ((int)bi >= sc.n_buildings) {
      int64_t k = count_of(4 * b.hx * b.hy * surf_density);
      for (int64_t i = 0; i < k; ++i) {
        double lx = rng.uni(-b.hx, b.hx), ly = rng.uni(-b.hy, b.hy);
        put_s(b.cx + b.c * lx - b.s * ly, b.cy + b.s * lx + b.c * ly, b.h + 0.01 * rng.normal());
      }
    }
    // vertical edges -> corner map
    for (int e = 0; e < 4; ++e) {
      double lx = (e & 1) ? b.hx : -b.hx, ly = (e & 2) ? b.hy : -b.hy;
      double ex = b.cx + b.c * lx - b.s * ly, ey = b.cy + b.s * lx + b.c * ly;
      int64_t k = count_of(b.h * corner_density);
      for (int64_t i = 0; i < k; ++i)
        put_c(ex + 0.03 * rng.normal(), ey + 0.03 * rng.normal(), rng.uni(0.0, b.h));
    }
  }
  for (const Tree& tr : sc.trees) {  // canopy surfaces
    if (std::hypot(tr.x, tr.y) > map_radius + 10) continue;
    int64_t k = count_of(4 * M_PI * tr.r * tr.r * surf_density);
    for (int64_t i = 0; i < k; ++i) {
      double zc = rng.uni(-1.0, 1.0), a = rng.uni(-M_PI, M_PI), rr = tr.r + 0.01 * rng.normal();
      double sxy = std::sqrt(1 - zc * zc);
      put_s(tr.x + rr * sxy * std::cos(a), tr.y + rr * sxy * std::sin(a), tr.z + rr * zc);
    }
  }
  for (const Pole& p : sc.poles) {
    if (std::hypot(p.x, p.y) > map_radius + 10) continue;
    int64_t k = count_of(p.h * corner_density);
    for (int64_t i = 0; i < k; ++i) {
      double a = rng.uni(-M_PI, M_PI), rr = p.r * rng.uni();
      put_c(p.x + rr * std::cos(a), p.y + rr * std::sin(a), rng.uni(0.0, p.h));
    }
  }
  if (n_corner) *n_corner = nc;
  if (n_surf) *n_surf = ns;
  return 0;
}

}  // extern "C"
