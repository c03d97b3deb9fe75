// ASan/UBSan run of the product library's host-side code: the wire
// formats of pcdio.hip (PCD clouds, feature PCDs) and pca.hip (PCA::write, the
// rotateFeature90 maps), compiled with the sanitizers on the host side only (no GPU is
// touched).  argv: feature-pcd output dir, then PCD clouds and reference PCA files.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/c3hlac_mi355x.h"

static int check_pcd(const char* path) {
  int64_t n = 0;
  const int q = c3h_pcd_read_xyzrgb(path, nullptr, &n);
  if (q == C3H_ERR_FORMAT || q == C3H_ERR_ARG) return 0;  // e.g. a feature PCD: the error path runs too
  if (q != C3H_OK) return 1;
  std::vector<float> pts((size_t)(n ? n : 1) * 4);
  int64_t cap = n;
  if (c3h_pcd_read_xyzrgb(path, pts.data(), &cap) != C3H_OK || cap != n) return 2;
  return 0;
}

static int check_pca(const char* path, const std::string& out) {
  FILE* fp = fopen(path, "rb");  // PCA::read's binary layout (the reader lives in capi.hip)
  int dim = 0;
  if (!fp || fread(&dim, 4, 1, fp) != 1 || dim <= 0 || dim > 4096) return 3;
  std::vector<float> a((size_t)dim * dim), v(dim), m(dim);
  const bool ok = fread(a.data(), 4, a.size(), fp) == a.size() && fread(v.data(), 4, dim, fp) == (size_t)dim;
  const int hm = ok && fread(m.data(), 4, dim, fp) == (size_t)dim;
  fclose(fp);
  if (!ok) return 4;
  for (int ascii = 0; ascii < 2; ++ascii)
    if (c3h_pca_write(out.c_str(), ascii, dim, a.data(), v.data(), hm ? m.data() : nullptr) != C3H_OK) return 5;
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 64;
  const std::string dir = argv[1];
  for (int dim : {981, 495, 486})
    for (int mode = 0; mode < 4; ++mode) {
      std::vector<int32_t> map(dim);
      if (c3h_rotate_map(dim, mode, map.data()) != C3H_OK) return 6;
    }
  std::vector<int32_t> bad(117);
  if (c3h_rotate_map(117, 0, bad.data()) != C3H_ERR_ARG) return 7;
  // feature PCD round trip, with zero rows dropped and the "vfh" FIELDS name
  const int rows = 37, dim = 137;
  std::vector<float> f((size_t)rows * dim);
  for (size_t i = 0; i < f.size(); ++i) f[i] = (i % 11 == 0 || (i / dim) % 5 == 0) ? 0.f : (float)(i % 97) / 7.f;
  const std::string fp = dir + "/feat.pcd";
  for (int rz = 0; rz < 2; ++rz) {
    if (c3h_feature_pcd_write(fp.c_str(), f.data(), rows, dim, rz, rz ? "vfh" : nullptr) != C3H_OK) return 8;
    int64_t r = 0;
    int32_t d = 0;
    if (c3h_feature_pcd_read(fp.c_str(), nullptr, &r, &d) != C3H_OK || d != dim) return 9;
    std::vector<float> back((size_t)r * d);
    if (c3h_feature_pcd_read(fp.c_str(), back.data(), &r, &d) != C3H_OK) return 10;
  }
  for (int i = 2; i < argc; ++i) {
    const char* p = argv[i];
    const size_t L = strlen(p);
    const int rc = (L > 4 && !strcmp(p + L - 4, ".pcd")) ? check_pcd(p) : check_pca(p, dir + "/pca_out");
    if (rc) {
      fprintf(stderr, "%s: failed (%d)\n", p, rc);
      return 20 + rc;
    }
  }
  printf("host_check ok\n");
  return 0;
}
