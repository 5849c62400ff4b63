// fbr_pcd.cpp — PCD file I/O for the prior global map.
//
// Reference: src/mapOptmization.h:245-260 loads cloudCorner.pcd / cloudSurf.pcd with
// pcl::io::loadPCDFile into PointXYZI clouds and VoxelGrid-filters them; :495-519 writes the maps
// with pcl::io::savePCDFileASCII.  This is a dependency-free restatement of the PCD v0.7 format
// as PCL 1.8 reads and writes it:
//   * header: VERSION / FIELDS / SIZE / TYPE / COUNT / WIDTH / HEIGHT / VIEWPOINT / POINTS / DATA
//     (case-insensitive keys, '#' comments);
//   * DATA ascii (whitespace separated, "nan" allowed), binary (packed records), and
//     binary_compressed (uint32 compressed size, uint32 raw size, LZF stream of the fields laid
//     out one after another: all values of field 0, then field 1, ...);
//   * x, y, z and intensity are taken by name from any field layout (other fields, e.g. "_"
//     padding, rgb or normals, are skipped; a missing intensity reads as 0); F4/F8/U/I types.
// Writers: ASCII with PCL's default precision of 8 significant digits (as savePCDFileASCII), and
// binary (exact floats).
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fbr.h"

namespace {

struct Field {
  std::string name;
  int size = 4, count = 1;
  char type = 'F';
  int offset = 0;  // byte offset inside a binary record
};

struct Header {
  std::vector<Field> fields;
  int64_t width = 0, height = 1, points = -1;
  std::string data;
  int record = 0;  // bytes per point
};

std::string lower(std::string s) {
  for (char& ch : s) ch = (char)std::tolower((unsigned char)ch);
  return s;
}

std::vector<std::string> split(const std::string& line) {
  std::vector<std::string> out;
  size_t i = 0;
  while (i < line.size()) {
    while (i < line.size() && std::isspace((unsigned char)line[i])) ++i;
    size_t j = i;
    while (j < line.size() && !std::isspace((unsigned char)line[j])) ++j;
    if (j > i) out.push_back(line.substr(i, j - i));
    i = j;
  }
  return out;
}

// Reads the header; leaves `pos` at the first byte of the data section.
int parse_header(const std::vector<unsigned char>& buf, Header& h, size_t& pos) {
  pos = 0;
  std::vector<int> sizes, counts;
  std::vector<char> types;
  while (pos < buf.size()) {
    size_t e = pos;
    while (e < buf.size() && buf[e] != '\n') ++e;
    std::string line((const char*)buf.data() + pos, e - pos);
    pos = e < buf.size() ? e + 1 : e;
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty() || line[0] == '#') continue;
    std::vector<std::string> t = split(line);
    if (t.empty()) continue;
    const std::string key = lower(t[0]);
    if (key == "version") {
      continue;
    } else if (key == "fields" || key == "columns") {
      h.fields.clear();
      for (size_t k = 1; k < t.size(); ++k) {
        Field f;
        f.name = t[k];
        h.fields.push_back(f);
      }
    } else if (key == "size") {
      for (size_t k = 1; k < t.size(); ++k) sizes.push_back(std::atoi(t[k].c_str()));
    } else if (key == "type") {
      for (size_t k = 1; k < t.size(); ++k) types.push_back((char)std::toupper((unsigned char)t[k][0]));
    } else if (key == "count") {
      for (size_t k = 1; k < t.size(); ++k) counts.push_back(std::atoi(t[k].c_str()));
    } else if (key == "width" && t.size() > 1) {
      h.width = std::atoll(t[1].c_str());
    } else if (key == "height" && t.size() > 1) {
      h.height = std::atoll(t[1].c_str());
    } else if (key == "viewpoint") {
      continue;
    } else if (key == "points" && t.size() > 1) {
      h.points = std::atoll(t[1].c_str());
    } else if (key == "data" && t.size() > 1) {
      h.data = lower(t[1]);
      break;
    } else {
      return FBR_ERR_INVALID_ARG;
    }
  }
  if (h.data.empty() || h.fields.empty()) return FBR_ERR_INVALID_ARG;
  if (sizes.size() != h.fields.size() || types.size() != h.fields.size()) return FBR_ERR_INVALID_ARG;
  int off = 0;
  for (size_t k = 0; k < h.fields.size(); ++k) {
    Field& f = h.fields[k];
    f.size = sizes[k];
    f.type = types[k];
    f.count = k < counts.size() ? counts[k] : 1;
    if (f.size != 1 && f.size != 2 && f.size != 4 && f.size != 8) return FBR_ERR_INVALID_ARG;
    if (f.count < 1) return FBR_ERR_INVALID_ARG;
    f.offset = off;
    off += f.size * f.count;
  }
  h.record = off;
  if (h.points < 0) h.points = h.width * h.height;
  if (h.points < 0 || h.points != h.width * h.height) return FBR_ERR_INVALID_ARG;
  return FBR_OK;
}

double load_value(const unsigned char* p, const Field& f) {
  switch (f.type) {
    case 'F':
      if (f.size == 4) {
        float v;
        std::memcpy(&v, p, 4);
        return v;
      } else if (f.size == 8) {
        double v;
        std::memcpy(&v, p, 8);
        return v;
      }
      return 0.0;
    case 'U':
      if (f.size == 1) return (double)*p;
      if (f.size == 2) { uint16_t v; std::memcpy(&v, p, 2); return v; }
      if (f.size == 4) { uint32_t v; std::memcpy(&v, p, 4); return v; }
      { uint64_t v; std::memcpy(&v, p, 8); return (double)v; }
    default:  // 'I'
      if (f.size == 1) return (double)(int8_t)*p;
      if (f.size == 2) { int16_t v; std::memcpy(&v, p, 2); return v; }
      if (f.size == 4) { int32_t v; std::memcpy(&v, p, 4); return v; }
      { int64_t v; std::memcpy(&v, p, 8); return (double)v; }
  }
}

// LZF decompression (liblzf's lzf_decompress, the codec PCL uses for binary_compressed).
bool lzf_decompress(const unsigned char* in, size_t in_len, unsigned char* out, size_t out_len) {
  size_t ip = 0, op = 0;
  while (ip < in_len) {
    unsigned ctrl = in[ip++];
    if (ctrl < 32) {  // literal run of ctrl + 1 bytes
      const size_t len = ctrl + 1;
      if (ip + len > in_len || op + len > out_len) return false;
      std::memcpy(out + op, in + ip, len);
      ip += len;
      op += len;
    } else {  // back reference
      size_t len = ctrl >> 5;
      if (len == 7) {
        if (ip >= in_len) return false;
        len += in[ip++];
      }
      if (ip >= in_len) return false;
      const size_t back = ((ctrl & 0x1f) << 8) + in[ip++] + 1;
      len += 2;
      if (back > op || op + len > out_len) return false;
      for (size_t k = 0; k < len; ++k, ++op) out[op] = out[op - back];  // may overlap
    }
  }
  return op == out_len;
}

int find_field(const Header& h, const char* name) {
  for (size_t k = 0; k < h.fields.size(); ++k)
    if (h.fields[k].name == name) return (int)k;
  return -1;
}

int read_file(const char* path, std::vector<unsigned char>& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return FBR_ERR_INVALID_ARG;
  std::fseek(f, 0, SEEK_END);
  const long sz = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (sz < 0) {
    std::fclose(f);
    return FBR_ERR_INVALID_ARG;
  }
  buf.resize((size_t)sz);
  const size_t got = sz ? std::fread(buf.data(), 1, (size_t)sz, f) : 0;
  std::fclose(f);
  return got == (size_t)sz ? FBR_OK : FBR_ERR_INVALID_ARG;
}

}  // namespace

extern "C" {

int fbr_pcd_read(const char* path, fbr_point_xyzi* out, int64_t cap, int64_t* n_out) {
  if (!path || !n_out) return FBR_ERR_INVALID_ARG;
  std::vector<unsigned char> buf;
  int rc = read_file(path, buf);
  if (rc) return rc;
  Header h;
  size_t pos = 0;
  rc = parse_header(buf, h, pos);
  if (rc) return rc;
  const int64_t n = h.points;
  *n_out = n;
  if (!out) return FBR_OK;  // size query
  if (cap < n) return FBR_ERR_CAPACITY;
  const int fi[4] = {find_field(h, "x"), find_field(h, "y"), find_field(h, "z"), find_field(h, "intensity")};
  if (fi[0] < 0 || fi[1] < 0 || fi[2] < 0) return FBR_ERR_INVALID_ARG;
  auto put = [&](int64_t i, int c, double v) {
    float* dst = &out[i].x;
    dst[c] = (float)v;
  };
  for (int64_t i = 0; i < n; ++i) out[i] = fbr_point_xyzi{0.f, 0.f, 0.f, 0.f};
  if (h.data == "ascii") {
    // tokens per point = sum of counts; each line one point
    int64_t i = 0;
    size_t p = pos;
    while (i < n && p < buf.size()) {
      size_t e = p;
      while (e < buf.size() && buf[e] != '\n') ++e;
      std::string line((const char*)buf.data() + p, e - p);
      p = e < buf.size() ? e + 1 : e;
      std::vector<std::string> t = split(line);
      if (t.empty()) continue;
      size_t tok = 0;
      for (size_t k = 0; k < h.fields.size(); ++k) {
        for (int c = 0; c < h.fields[k].count; ++c, ++tok) {
          if (tok >= t.size()) return FBR_ERR_INVALID_ARG;
          if (c != 0) continue;
          for (int q = 0; q < 4; ++q)
            if ((int)k == fi[q]) {
              const std::string& s = t[tok];
              const std::string ls = lower(s);
              const double v = (ls == "nan" || ls == "-nan") ? std::nan("") : std::strtod(s.c_str(), nullptr);
              put(i, q, v);
            }
        }
      }
      ++i;
    }
    return i == n ? FBR_OK : FBR_ERR_INVALID_ARG;
  }
  if (h.data == "binary") {
    if (pos + (size_t)n * h.record > buf.size()) return FBR_ERR_INVALID_ARG;
    const unsigned char* base = buf.data() + pos;
    for (int64_t i = 0; i < n; ++i)
      for (int q = 0; q < 4; ++q)
        if (fi[q] >= 0) put(i, q, load_value(base + i * h.record + h.fields[fi[q]].offset, h.fields[fi[q]]));
    return FBR_OK;
  }
  if (h.data == "binary_compressed") {
    if (pos + 8 > buf.size()) return FBR_ERR_INVALID_ARG;
    uint32_t csize, usize;
    std::memcpy(&csize, buf.data() + pos, 4);
    std::memcpy(&usize, buf.data() + pos + 4, 4);
    if (pos + 8 + (size_t)csize > buf.size() || (int64_t)usize != n * h.record) return FBR_ERR_INVALID_ARG;
    std::vector<unsigned char> raw(usize);
    if (usize && !lzf_decompress(buf.data() + pos + 8, csize, raw.data(), usize)) return FBR_ERR_INVALID_ARG;
    // fields are stored one after another: field k occupies n * size * count bytes
    size_t foff = 0;
    for (size_t k = 0; k < h.fields.size(); ++k) {
      const Field& f = h.fields[k];
      for (int q = 0; q < 4; ++q)
        if ((int)k == fi[q])
          for (int64_t i = 0; i < n; ++i) put(i, q, load_value(raw.data() + foff + (size_t)i * f.size * f.count, f));
      foff += (size_t)n * f.size * f.count;
    }
    return FBR_OK;
  }
  return FBR_ERR_INVALID_ARG;
}

static int write_header(FILE* f, int64_t n, const char* data) {
  return std::fprintf(f,
                      "# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\n"
                      "SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\nWIDTH %lld\nHEIGHT 1\n"
                      "VIEWPOINT 0 0 0 1 0 0 0\nPOINTS %lld\nDATA %s\n",
                      (long long)n, (long long)n, data) > 0;
}

int fbr_pcd_write_ascii(const char* path, const fbr_point_xyzi* pts, int64_t n) {
  if (!path || n < 0 || (n && !pts)) return FBR_ERR_INVALID_ARG;
  FILE* f = std::fopen(path, "wb");
  if (!f) return FBR_ERR_INVALID_ARG;
  bool ok = write_header(f, n, "ascii");
  for (int64_t i = 0; i < n && ok; ++i) {
    const float v[4] = {pts[i].x, pts[i].y, pts[i].z, pts[i].intensity};
    for (int c = 0; c < 4 && ok; ++c) {
      // savePCDFileASCII: precision 8 (%.8g), "nan" for NaN, space separated
      if (std::isnan(v[c])) ok = std::fputs("nan", f) >= 0;
      else ok = std::fprintf(f, "%.8g", (double)v[c]) > 0;
      if (ok) ok = std::fputc(c < 3 ? ' ' : '\n', f) != EOF;
    }
  }
  ok = (std::fclose(f) == 0) && ok;
  return ok ? FBR_OK : FBR_ERR_INVALID_ARG;
}

int fbr_pcd_write_binary(const char* path, const fbr_point_xyzi* pts, int64_t n) {
  if (!path || n < 0 || (n && !pts)) return FBR_ERR_INVALID_ARG;
  FILE* f = std::fopen(path, "wb");
  if (!f) return FBR_ERR_INVALID_ARG;
  bool ok = write_header(f, n, "binary");
  if (ok && n) ok = std::fwrite(pts, sizeof(fbr_point_xyzi), (size_t)n, f) == (size_t)n;
  ok = (std::fclose(f) == 0) && ok;
  return ok ? FBR_OK : FBR_ERR_INVALID_ARG;
}

int fbr_load_map(fbr_ctx* ctx, const char* corner_pcd, const char* surf_pcd) {
  if (!ctx || !corner_pcd || !surf_pcd) return FBR_ERR_INVALID_ARG;
  int64_t nc = 0, ns = 0;
  int rc = fbr_pcd_read(corner_pcd, nullptr, 0, &nc);
  if (!rc) rc = fbr_pcd_read(surf_pcd, nullptr, 0, &ns);
  if (rc) return rc;
  std::vector<fbr_point_xyzi> c((size_t)nc), s((size_t)ns);
  rc = fbr_pcd_read(corner_pcd, c.data(), nc, &nc);
  if (!rc) rc = fbr_pcd_read(surf_pcd, s.data(), ns, &ns);
  if (!rc) rc = fbr_set_map(ctx, c.data(), nc, s.data(), ns);
  return rc;
}

}  // extern "C"
