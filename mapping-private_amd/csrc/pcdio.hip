// pcdio.hip -- host-side wire formats of the path: PCD point clouds as
// the reference's tools load them (pcl::io::loadPCDFile: calc_scene_auto_threshold.cpp:89,
// extract_c3_hlac_scene.cpp, the ROS bag dumps), and the ASCII feature PCD of
// readFeature / writeFeature (c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:46-113).
// No device code: these feed c3h_voxelize and store c3h_get_features output.
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/c3hlac_mi355x.h"

namespace {

struct PcdHeader {
  std::vector<std::string> fields;
  std::vector<int> size, count;
  std::vector<char> type;
  long long points = -1, width = -1, height = 1;
  int data = -1;  // 0 ascii, 1 binary
  long header_end = 0;
};

std::vector<std::string> split(const char* s) {
  std::vector<std::string> v;
  const char* p = s;
  while (*p) {
    while (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n') ++p;
    if (!*p) break;
    const char* q = p;
    while (*q && *q != ' ' && *q != '\t' && *q != '\r' && *q != '\n') ++q;
    v.emplace_back(p, q - p);
    p = q;
  }
  return v;
}

int read_header(FILE* fp, PcdHeader& h) {
  char line[4096];
  while (fgets(line, sizeof(line), fp)) {
    std::vector<std::string> t = split(line);
    if (t.empty() || t[0][0] == '#') continue;
    const std::string& k = t[0];
    if (k == "FIELDS" || k == "COLUMNS") {
      h.fields.assign(t.begin() + 1, t.end());
    } else if (k == "SIZE") {
      for (size_t i = 1; i < t.size(); ++i) h.size.push_back(atoi(t[i].c_str()));
    } else if (k == "TYPE") {
      for (size_t i = 1; i < t.size(); ++i) h.type.push_back(t[i][0]);
    } else if (k == "COUNT") {
      for (size_t i = 1; i < t.size(); ++i) h.count.push_back(atoi(t[i].c_str()));
    } else if (k == "WIDTH" && t.size() > 1) {
      h.width = atoll(t[1].c_str());
    } else if (k == "HEIGHT" && t.size() > 1) {
      h.height = atoll(t[1].c_str());
    } else if (k == "POINTS" && t.size() > 1) {
      h.points = atoll(t[1].c_str());
    } else if (k == "DATA" && t.size() > 1) {
      h.data = t[1] == "ascii" ? 0 : t[1] == "binary" ? 1 : 2;
      h.header_end = ftell(fp);
      return 0;
    }
  }
  return -1;
}

}  // namespace

extern "C" {

int c3h_pcd_read_xyzrgb(const char* path, float* out, int64_t* n) {
  if (!path || !n) return C3H_ERR_ARG;
  FILE* fp = fopen(path, "rb");
  if (!fp) return C3H_ERR_NOTFOUND;
  PcdHeader h;
  const int rc = read_header(fp, h);
  const size_t nf = h.fields.size();
  if (rc != 0 || nf == 0 || h.data < 0 || h.data > 1) {
    fclose(fp);
    return C3H_ERR_FORMAT;
  }
  if (h.size.empty()) h.size.assign(nf, 4);
  if (h.count.empty()) h.count.assign(nf, 1);
  if (h.type.empty()) h.type.assign(nf, 'F');
  if (h.points < 0) h.points = h.width * h.height;
  int ix = -1, iy = -1, iz = -1, ic = -1;
  long off[64];
  long stride = 0;
  bool ok = nf <= 64 && h.size.size() == nf && h.count.size() == nf && h.type.size() == nf && h.points >= 0;
  for (size_t f = 0; ok && f < nf; ++f) {
    off[f] = stride;
    stride += (long)h.size[f] * h.count[f];
    const std::string& nm = h.fields[f];
    if (nm == "x") ix = (int)f;
    if (nm == "y") iy = (int)f;
    if (nm == "z") iz = (int)f;
    if (nm == "rgb" || nm == "rgba") ic = (int)f;
  }
  const int need[4] = {ix, iy, iz, ic};
  for (int k = 0; ok && k < 4; ++k)
    ok = need[k] >= 0 && h.size[need[k]] == 4 && h.count[need[k]] == 1 && (k == 3 || h.type[need[k]] == 'F');
  if (!ok) {
    fclose(fp);
    return C3H_ERR_ARG;  // not an x y z rgb cloud of 4-byte scalars
  }
  if (!out) {
    *n = h.points;
    fclose(fp);
    return C3H_OK;
  }
  if (*n < h.points) {
    fclose(fp);
    return C3H_ERR_ARG;
  }
  int ret = C3H_OK;
  if (h.data == 1) {
    // binary: ROS-era PCL writers put the data at the next 4096-byte page after the header
    // (the demo clouds), current ones right after it; the file size tells which
    fseek(fp, 0, SEEK_END);
    const long fsize = ftell(fp);
    const long bytes = stride * (long)h.points;
    const long page = (h.header_end + 4095) / 4096 * 4096;
    long start = -1;
    if (fsize == h.header_end + bytes) start = h.header_end;
    else if (fsize == page + bytes) start = page;
    else if (fsize > h.header_end + bytes) start = fsize - bytes;  // trailing-aligned writers
    std::vector<unsigned char> buf((size_t)bytes);
    if (start < 0 || fseek(fp, start, SEEK_SET) != 0 || fread(buf.data(), 1, buf.size(), fp) != buf.size()) {
      ret = C3H_ERR_FORMAT;
    } else {
      for (long long i = 0; i < h.points; ++i)
        for (int k = 0; k < 4; ++k) memcpy(&out[4 * i + k], &buf[(size_t)(i * stride + off[need[k]])], 4);
    }
  } else {
    // ascii: one point per line, fields in header order; rgb as PCL prints it (a float whose
    // bits are the packed colour, or an unsigned integer for TYPE U)
    fseek(fp, h.header_end, SEEK_SET);
    std::vector<char> line(64 + 32 * stride);
    for (long long i = 0; i < h.points && ret == C3H_OK; ++i) {
      if (!fgets(line.data(), (int)line.size(), fp)) {
        ret = C3H_ERR_FORMAT;
        break;
      }
      std::vector<std::string> t = split(line.data());
      if (t.size() < nf) {
        ret = C3H_ERR_FORMAT;
        break;
      }
      for (int k = 0; k < 4; ++k) {
        const std::string& s = t[need[k]];
        if (k == 3 && h.type[ic] != 'F') {
          const uint32_t u = (uint32_t)strtoul(s.c_str(), nullptr, 10);
          memcpy(&out[4 * i + 3], &u, 4);
        } else {
          out[4 * i + k] = strtof(s.c_str(), nullptr);
        }
      }
    }
  }
  fclose(fp);
  if (ret == C3H_OK) *n = h.points;
  return ret;
}

// readFeature (c3_hlac_tools.hpp:46-71): COUNT = dim, POINTS = rows, then "%f " scans
int c3h_feature_pcd_read(const char* path, float* out, int64_t* rows, int32_t* dim) {
  if (!path || !rows || !dim) return C3H_ERR_ARG;
  FILE* fp = fopen(path, "r");
  if (!fp) return C3H_ERR_NOTFOUND;
  int d = -1, ns = -1;
  char line[4096];
  bool data = false;
  while (fgets(line, sizeof(line), fp)) {
    if (strncmp(line, "COUNT", 5) == 0) sscanf(line, "COUNT %d", &d);
    else if (strncmp(line, "POINTS", 6) == 0) sscanf(line, "POINTS %d", &ns);
    else if (strncmp(line, "DATA", 4) == 0) {
      data = true;
      break;
    }
  }
  if (!data || d < 0 || ns < 0) {
    fclose(fp);
    return C3H_ERR_FORMAT;
  }
  if (!out) {
    *rows = ns;
    *dim = d;
    fclose(fp);
    return C3H_OK;
  }
  if (*rows < ns || *dim < d) {
    fclose(fp);
    return C3H_ERR_ARG;
  }
  for (long long i = 0; i < (long long)ns * d; ++i)
    if (fscanf(fp, "%f ", &out[i]) == EOF) {
      fclose(fp);
      return C3H_ERR_FORMAT;
    }
  fclose(fp);
  *rows = ns;
  *dim = d;
  return C3H_OK;
}

// writeFeature (c3_hlac_tools.hpp:83-113; grsd_colorCHLAC_tools.hpp:32-58 writes FIELDS vfh)
int c3h_feature_pcd_write(const char* path, const float* feat, int64_t rows, int32_t dim, int32_t remove_zero,
                          const char* fields) {
  if (!path || (!feat && rows > 0) || rows < 0 || dim < 1) return C3H_ERR_ARG;
  auto zero = [&](int64_t r) {
    for (int t = 0; t < dim; ++t)
      if (feat[r * dim + t] != 0) return false;
    return true;
  };
  int64_t kept = rows;
  if (remove_zero)
    for (int64_t r = 0; r < rows; ++r)
      if (zero(r)) --kept;
  FILE* fp = fopen(path, "w");
  if (!fp) return C3H_ERR_NOTFOUND;
  fprintf(fp, "# .PCD v.7 - Point Cloud Data file format\n");
  fprintf(fp, "FIELDS %s\n", fields ? fields : "descriptor");
  fprintf(fp, "SIZE 4\n");
  fprintf(fp, "TYPE F\n");
  fprintf(fp, "COUNT %d\n", dim);
  fprintf(fp, "WIDTH %d\n", (int)kept);
  fprintf(fp, "HEIGHT 1\n");
  fprintf(fp, "POINTS %d\n", (int)kept);
  fprintf(fp, "DATA ascii\n");
  for (int64_t r = 0; r < rows; ++r) {
    if (remove_zero && zero(r)) continue;
    for (int t = 0; t < dim; ++t) fprintf(fp, "%f ", feat[r * dim + t]);
    fprintf(fp, "\n");
  }
  return fclose(fp) == 0 ? C3H_OK : C3H_ERR_FORMAT;
}

}  // extern "C"
