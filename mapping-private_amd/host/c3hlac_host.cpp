// c3hlac_host.cpp -- the reference-named C++ facade over the C-ABI (see c3hlac_host.h).
#include "c3hlac_host.h"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

namespace c3hlac {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void grid_info(const Context& ctx, c3h_grid_info* info) {
  ctx.check(c3h_get_grid_info(ctx.get(), info), "c3h_get_grid_info");
}

Vector3i v3(const int32_t* p) {
  Vector3i v;
  v[0] = p[0];
  v[1] = p[1];
  v[2] = p[2];
  return v;
}

// extractC3HLACSignature{981,117} body (c3_hlac_tools.hpp:134-160, 169-195): the silent
// empty cases of setVoxelFilter / computeFeature leave `feature` empty and still return
// getSubdivNum().
Vector3i extract(VoxelGrid& grid, int variant, std::vector<std::vector<float> >& feature, int thr_r,
                 int thr_g, int thr_b, float voxel_size, int subdiv, int ox, int oy, int oz,
                 int color_mode) {
  feature.resize(0);
  if (grid.leaf() != 0.0f && voxel_size != grid.leaf())
    throw Error(C3H_ERR_ARG, "extractC3HLACSignature: voxel_size differs from the grid's leaf size");
  c3h_extract_params p;
  p.variant = variant;
  p.thr[0] = thr_r;
  p.thr[1] = thr_g;
  p.thr[2] = thr_b;
  p.subdiv = subdiv;
  p.offset[0] = ox;
  p.offset[1] = oy;
  p.offset[2] = oz;
  p.color_mode = color_mode;
  int32_t sb[3];
  int64_t hist_num = 0;
  const Context& ctx = grid.context();
  ctx.check(c3h_extract(ctx.get(), &p, sb, &hist_num), "c3h_extract");
  if (hist_num > 0) {
    std::vector<float> flat((size_t)hist_num * variant);
    ctx.check(c3h_get_features(ctx.get(), flat.data(), 0), "c3h_get_features");
    feature.resize((size_t)hist_num);
    for (int64_t h = 0; h < hist_num; ++h)
      feature[h].assign(flat.begin() + h * variant, flat.begin() + (h + 1) * variant);
  }
  return v3(sb);
}

// Param::readParam (param.cpp:200-222): first "key value" pair whose key matches.
template <typename T>
bool read_param(const char* filename, const char* key, T& val) {
  std::ifstream in(filename);
  if (!in) return false;
  std::string tok;
  while (in >> tok) {
    if (tok == key) {
      std::string v;
      if (!(in >> v)) return false;
      std::istringstream vs(v);
      return (bool)(vs >> val);
    }
  }
  return false;
}

}  // namespace

// ------------------------------------------------------------------------- Context
Context::Context(int hip_device) {
  c3h_ctx* c = nullptr;
  const int rc = c3h_create(hip_device, &c);
  if (rc != C3H_OK) throw Error(rc, "c3h_create failed (no HIP device or library not built?)");
  ctx_.reset(c, c3h_destroy);
}

void Context::check(int rc, const char* what) const {
  if (rc < 0) {
    const char* m = c3h_last_error(ctx_.get());
    throw Error(rc, std::string(what) + ": " + (m ? m : ""));
  }
}

void Context::setStream(void* s) { check(c3h_set_stream(get(), s), "c3h_set_stream"); }
void Context::synchronize() { check(c3h_synchronize(get()), "c3h_synchronize"); }

// ------------------------------------------------------------------------- VoxelGrid
void VoxelGrid::setLeafSize(float lx, float ly, float lz) {
  if (lx != ly || ly != lz) throw Error(C3H_ERR_ARG, "VoxelGrid: anisotropic leaves are not supported");
  leaf_ = lx;
}

Vector3i VoxelGrid::getNrDivisions() const {
  c3h_grid_info i;
  grid_info(ctx_, &i);
  return v3(i.div_b);
}
Vector3i VoxelGrid::getMinBoxCoordinates() const {
  c3h_grid_info i;
  grid_info(ctx_, &i);
  return v3(i.min_b);
}
Vector3i VoxelGrid::getMaxBoxCoordinates() const {
  c3h_grid_info i;
  grid_info(ctx_, &i);
  return v3(i.max_b);
}

std::vector<int> VoxelGrid::getLeafLayout() const {
  const Vector3i d = getNrDivisions();
  std::vector<int> out((size_t)d[0] * d[1] * d[2]);
  ctx_.check(c3h_get_leaf_layout(ctx_.get(), out.data(), 0), "c3h_get_leaf_layout");
  return out;
}

void VoxelGrid::setPackedGrid(const uint32_t* words, const Vector3i& div_b, const Vector3i& min_b,
                              float leaf, bool on_device) {
  ctx_.check(c3h_set_grid(ctx_.get(), words, div_b.v, min_b.v, leaf, on_device ? 1 : 0), "c3h_set_grid");
  leaf_ = leaf;
}

std::vector<uint32_t> VoxelGrid::getPackedGrid() const {
  const Vector3i d = getNrDivisions();
  std::vector<uint32_t> out((size_t)d[0] * d[1] * d[2]);
  ctx_.check(c3h_get_grid(ctx_.get(), out.data(), 0), "c3h_get_grid");
  return out;
}

void getVoxelGrid(VoxelGrid& grid, const std::vector<PointXYZRGB>& input,
                  std::vector<PointXYZRGB>& output, float voxel_size, float z_limit) {
  static_assert(sizeof(PointXYZRGB) == 16, "xyzrgb record must be 4 floats");
  grid.leaf_ = voxel_size;
  c3h_grid_info info;
  grid.ctx_.check(c3h_voxelize(grid.ctx_.get(), reinterpret_cast<const float*>(input.data()),
                               (int64_t)input.size(), 0, voxel_size, z_limit, &info),
                  "c3h_voxelize");
  output.resize((size_t)info.n_occ);
  if (info.n_occ > 0)
    grid.ctx_.check(c3h_get_downsampled(grid.ctx_.get(), reinterpret_cast<float*>(output.data()), 0),
                    "c3h_get_downsampled");
}

int loadPCDFile(const std::string& file_name, std::vector<PointXYZRGB>& cloud) {
  int64_t n = 0;
  if (c3h_pcd_read_xyzrgb(file_name.c_str(), nullptr, &n) != C3H_OK) return -1;
  cloud.resize((size_t)n);
  if (n > 0 && c3h_pcd_read_xyzrgb(file_name.c_str(), reinterpret_cast<float*>(cloud.data()), &n) != C3H_OK)
    return -1;
  return 0;
}

void readFeature(const char* name, std::vector<std::vector<float> >& feature) {
  feature.resize(0);
  int64_t rows = 0;
  int32_t dim = 0;
  int rc = c3h_feature_pcd_read(name, nullptr, &rows, &dim);
  if (rc != C3H_OK) throw Error(rc, std::string("readFeature: ") + name);
  std::vector<float> buf((size_t)rows * dim);
  if (!buf.empty()) {
    rc = c3h_feature_pcd_read(name, buf.data(), &rows, &dim);
    if (rc != C3H_OK) throw Error(rc, std::string("readFeature: ") + name);
  }
  for (int64_t r = 0; r < rows; ++r) feature.emplace_back(buf.begin() + r * dim, buf.begin() + (r + 1) * dim);
}

void readFeature(const char* name, std::vector<float>& feature) {
  std::vector<std::vector<float> > features;
  readFeature(name, features);
  if (features.size() != 1)
    std::cerr << "Warning in readFeature(): the number of features in " << name << " is not 1. ("
              << features.size() << ")" << std::endl;
  feature = features.empty() ? std::vector<float>() : features[0];
}

void writeFeature(const char* name, const std::vector<std::vector<float> > feature, bool remove_0_flg) {
  if (feature.empty()) throw Error(C3H_ERR_ARG, "writeFeature: no rows");
  const size_t dim = feature[0].size();
  std::vector<float> buf;
  buf.reserve(feature.size() * dim);
  for (const auto& row : feature) {
    if (row.size() != dim) throw Error(C3H_ERR_ARG, "writeFeature: ragged rows");
    buf.insert(buf.end(), row.begin(), row.end());
  }
  const int rc = c3h_feature_pcd_write(name, buf.data(), (int64_t)feature.size(), (int32_t)dim, remove_0_flg ? 1 : 0,
                                       nullptr);
  if (rc != C3H_OK) throw Error(rc, std::string("writeFeature: ") + name);
}

void writeFeature(const char* name, const std::vector<float> feature, bool remove_0_flg) {
  writeFeature(name, std::vector<std::vector<float> >(1, feature), remove_0_flg);
}

void ColorThreshold::addScene(const VoxelGrid& grid) {
  grid.context().check(c3h_color_histogram(grid.context().get(), hist_, 1), "c3h_color_histogram");
}

void ColorThreshold::compute(int threshold[3], double total_average[3]) const {
  int32_t t[3];
  const int rc = c3h_auto_threshold(hist_, t, total_average);
  if (rc != C3H_OK) throw Error(rc, "ColorThreshold::compute: no occupied voxels");
  for (int i = 0; i < 3; ++i) threshold[i] = t[i];
}

void getVoxelGrid(VoxelGrid& grid, const std::vector<PointXYZRGBNormal>& input,
                  std::vector<PointXYZRGBNormal>& output, float voxel_size, float z_limit) {
  static_assert(sizeof(PointXYZRGBNormal) == 32, "xyzrgb + normal record must be 8 floats");
  std::vector<PointXYZRGB> xyz(input.size()), cent;
  for (size_t i = 0; i < input.size(); ++i) xyz[i] = PointXYZRGB{input[i].x, input[i].y, input[i].z, input[i].rgb};
  getVoxelGrid(grid, xyz, cent, voxel_size, z_limit);
  output.assign(cent.size(), PointXYZRGBNormal());
  if (cent.empty()) return;
  // VoxelGrid::filter averages every float field of the voxel's points: the normal and the
  // curvature in fp32, input order, times 1 / n as Eigen 3.0 divides (the centroid's xyz and
  // colour come from the device, with the same arithmetic)
  const std::vector<int> layout = grid.getLeafLayout();
  const Vector3i mn = grid.getMinBoxCoordinates(), dv = grid.getNrDivisions();
  const float inv = 1.0f / voxel_size;
  std::vector<float> acc(cent.size() * 4, 0.0f);
  std::vector<int> cnt(cent.size(), 0);
  for (const PointXYZRGBNormal& p : input) {
    if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z) || !(p.z < z_limit)) continue;
    const int cx = (int)std::floor(p.x * inv) - mn[0], cy = (int)std::floor(p.y * inv) - mn[1],
              cz = (int)std::floor(p.z * inv) - mn[2];
    const int o = layout[(size_t)cx + (size_t)dv[0] * ((size_t)cy + (size_t)dv[1] * cz)];
    float* a = &acc[(size_t)o * 4];
    a[0] += p.normal_x;
    a[1] += p.normal_y;
    a[2] += p.normal_z;
    a[3] += p.curvature;
    ++cnt[o];
  }
  for (size_t o = 0; o < cent.size(); ++o) {
    const float rn = 1.0f / (float)cnt[o];
    output[o] = PointXYZRGBNormal{cent[o].x, cent[o].y, cent[o].z, cent[o].rgb, acc[4 * o] * rn, acc[4 * o + 1] * rn,
                                  acc[4 * o + 2] * rn, acc[4 * o + 3] * rn};
  }
}

namespace detail {

bool voxel_filter(const VoxelGrid& grid, int subdiv, const int off[3], Vector3i& subdiv_b) {
  if (subdiv > 0) {
    const Vector3i div = grid.getNrDivisions();
    if (div[0] <= off[0] || div[1] <= off[1] || div[2] <= off[2]) {
      std::cerr << "(In setVoxelFilter) offset values (" << off[0] << "," << off[1] << "," << off[2]
                << ") exceed voxel grid size (" << div[0] << "," << div[1] << "," << div[2] << ")." << std::endl;
      return false;
    }
    const float inv = 1.0 / subdiv;  // inverse_subdivision_size, float as there
    for (int a = 0; a < 3; ++a) subdiv_b[a] = (int)std::ceil((div[a] - off[a]) * inv);
  } else if (subdiv < 0) {
    std::cerr << "(In setVoxelFilter) Invalid subdivision size: " << subdiv << std::endl;
    return false;
  }
  return true;
}

int64_t compute_feature(VoxelGrid& grid, int dim, const int thr[3], int subdiv, const int off[3], int color_mode,
                        std::vector<float>& flat) {
  if (thr[0] < 0 || thr[1] < 0 || thr[2] < 0) {  // computeFeature's silent return (c3_hlac.cpp:306-309)
    std::cerr << "Invalid color_threshold: " << thr[0] << " " << thr[1] << " " << thr[2] << std::endl;
    flat.clear();
    return 0;
  }
  std::vector<std::vector<float> > rows;
  extract(grid, dim, rows, thr[0], thr[1], thr[2], grid.leaf(), subdiv, off[0], off[1], off[2], color_mode);
  flat.resize(rows.size() * (size_t)dim);
  for (size_t h = 0; h < rows.size(); ++h) std::copy(rows[h].begin(), rows[h].end(), flat.begin() + h * dim);
  return (int64_t)rows.size();
}

int64_t grid_occupied(const VoxelGrid& grid) {
  c3h_grid_info i;
  grid_info(grid.context(), &i);
  return i.n_occ;
}

}  // namespace detail

// the explicit instantiations of c3_hlac.cpp:418-426
template class C3HLAC117Estimation<PointXYZRGB, C3HLACSignature117>;
template class C3HLAC117Estimation<PointXYZRGB, C3HLACSignature981>;
template class C3HLAC981Estimation<PointXYZRGB, C3HLACSignature117>;
template class C3HLAC981Estimation<PointXYZRGB, C3HLACSignature981>;
template class C3HLAC117Estimation<PointXYZRGBNormal, C3HLACSignature117>;
template class C3HLAC117Estimation<PointXYZRGBNormal, C3HLACSignature981>;
template class C3HLAC981Estimation<PointXYZRGBNormal, C3HLACSignature117>;
template class C3HLAC981Estimation<PointXYZRGBNormal, C3HLACSignature981>;
template class ColorCHLAC_RI_Estimation<PointXYZRGB, C3HLACSignature117>;
template class ColorCHLACEstimation<PointXYZRGB, C3HLACSignature981>;
template class ColorCHLAC_RI_Estimation<PointXYZRGBNormal, C3HLACSignature117>;
template class ColorCHLACEstimation<PointXYZRGBNormal, C3HLACSignature981>;

Vector3i extractC3HLACSignature981(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int r,
                                   int g, int b, float voxel_size, int subdiv, int ox, int oy, int oz,
                                   int color_mode) {
  return extract(grid, C3H_VARIANT_981, feature, r, g, b, voxel_size, subdiv, ox, oy, oz, color_mode);
}
void extractC3HLACSignature981(VoxelGrid& grid, std::vector<float>& feature, int r, int g, int b,
                               float voxel_size, int color_mode) {
  std::vector<std::vector<float> > tmp;
  extract(grid, C3H_VARIANT_981, tmp, r, g, b, voxel_size, 0, 0, 0, 0, color_mode);
  feature = tmp.empty() ? std::vector<float>() : tmp[0];
}
Vector3i extractC3HLACSignature117(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int r,
                                   int g, int b, float voxel_size, int subdiv, int ox, int oy, int oz,
                                   int color_mode) {
  return extract(grid, C3H_VARIANT_117, feature, r, g, b, voxel_size, subdiv, ox, oy, oz, color_mode);
}
void extractC3HLACSignature117(VoxelGrid& grid, std::vector<float>& feature, int r, int g, int b,
                               float voxel_size, int color_mode) {
  std::vector<std::vector<float> > tmp;
  extract(grid, C3H_VARIANT_117, tmp, r, g, b, voxel_size, 0, 0, 0, 0, color_mode);
  feature = tmp.empty() ? std::vector<float>() : tmp[0];
}

// extractColorCHLACSignature981/117 (color_chlac/include/color_chlac/grsd_colorCHLAC_tools.hpp:
// 680-747): the same flow with ColorCHLAC{,_RI}Estimation, whose setColor is (v, 255 - v)
Vector3i extractColorCHLACSignature981(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int r,
                                       int g, int b, float voxel_size, int subdiv, int ox, int oy, int oz) {
  return extract(grid, C3H_VARIANT_981, feature, r, g, b, voxel_size, subdiv, ox, oy, oz, C3H_COLOR_CHLAC);
}
void extractColorCHLACSignature981(VoxelGrid& grid, std::vector<float>& feature, int r, int g, int b,
                                   float voxel_size) {
  extractC3HLACSignature981(grid, feature, r, g, b, voxel_size, C3H_COLOR_CHLAC);
}
Vector3i extractColorCHLACSignature117(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int r,
                                       int g, int b, float voxel_size, int subdiv, int ox, int oy, int oz) {
  return extract(grid, C3H_VARIANT_117, feature, r, g, b, voxel_size, subdiv, ox, oy, oz, C3H_COLOR_CHLAC);
}
void extractColorCHLACSignature117(VoxelGrid& grid, std::vector<float>& feature, int r, int g, int b,
                                   float voxel_size) {
  extractC3HLACSignature117(grid, feature, r, g, b, voxel_size, C3H_COLOR_CHLAC);
}

// ------------------------------------------------------------------------- VOSCH / GRSD
void computeNormal(VoxelGrid& grid, double radius) {
  const Context& ctx = grid.context();
  ctx.check(c3h_compute_normals(ctx.get(), (float)radius, nullptr), "c3h_compute_normals");
}

std::vector<float> getNormals(const VoxelGrid& grid) {
  const Context& ctx = grid.context();
  c3h_grid_info gi;
  grid_info(ctx, &gi);
  std::vector<float> out((size_t)gi.n_valid * 4);
  ctx.check(c3h_get_normals(ctx.get(), out.data(), 0), "c3h_get_normals");
  return out;
}

static Vector3i grsd_like(VoxelGrid& grid, std::vector<std::vector<float> >& feature, float voxel_size, int subdiv,
                          int ox, int oy, int oz, bool normalize, const int* thr) {
  feature.resize(0);
  if (grid.leaf() != 0.0f && voxel_size != grid.leaf())
    throw Error(C3H_ERR_ARG, "extractGRSDSignature21: voxel_size differs from the grid's leaf size");
  const Context& ctx = grid.context();
  c3h_grsd_params p;
  p.subdiv = subdiv;
  p.offset[0] = ox;
  p.offset[1] = oy;
  p.offset[2] = oz;
  p.rsd_radius = (float)rsd_radius_search;
  p.normalize = normalize ? 1 : 0;
  int32_t sb[3] = {0, 0, 0};
  int64_t H = 0;
  auto run = [&] {
    return thr ? c3h_extract_vosch(ctx.get(), &p, thr, 1, sb, &H) : c3h_extract_grsd(ctx.get(), &p, sb, &H);
  };
  int rc = run();
  if (rc == C3H_ERR_STATE) {  // no normals yet: computeNormal with the reference's radius
    computeNormal(grid);
    rc = run();
  }
  ctx.check(rc, thr ? "c3h_extract_vosch" : "c3h_extract_grsd");
  const int F = thr ? 137 : 20;
  if (H > 0) {
    std::vector<float> flat((size_t)H * F);
    ctx.check(c3h_get_features(ctx.get(), flat.data(), 0), "c3h_get_features");
    feature.resize((size_t)H);
    for (int64_t h = 0; h < H; ++h) feature[h].assign(flat.begin() + h * F, flat.begin() + (h + 1) * F);
  }
  return v3(sb);
}

Vector3i extractGRSDSignature21(VoxelGrid& grid, std::vector<std::vector<float> >& feature, float voxel_size,
                                int subdiv, int ox, int oy, int oz, bool is_normalize) {
  return grsd_like(grid, feature, voxel_size, subdiv, ox, oy, oz, is_normalize, nullptr);
}

Vector3i extractVOSCH(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int thR, int thG, int thB,
                      float voxel_size, int subdiv, int ox, int oy, int oz, bool is_normalize) {
  const int thr[3] = {thR, thG, thB};
  return grsd_like(grid, feature, voxel_size, subdiv, ox, oy, oz, is_normalize, thr);
}

// ------------------------------------------------------------------------- PCA
void PCA::read(const char* filename, bool ascii) {
  // c3h_pca_read returns the axis column-major (eigenvector i contiguous), as the file
  int32_t has_mean = 0;
  int dim = c3h_pca_read(filename, ascii ? 1 : 0, nullptr, nullptr, nullptr, &has_mean, 0);
  if (dim < 0) throw Error(dim, std::string("PCA::read: cannot read ") + filename);
  std::vector<float> col((size_t)dim * dim), var(dim), mean(dim);
  dim = c3h_pca_read(filename, ascii ? 1 : 0, col.data(), var.data(), mean.data(), &has_mean, dim);
  if (dim < 0) throw Error(dim, std::string("PCA::read: malformed ") + filename);
  axis_ = MatrixXf(dim, dim);
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) axis_(j, i) = col[(size_t)i * dim + j];
  variance_ = var;
  mean_flg_ = has_mean != 0;
  if (mean_flg_) mean_ = mean;
  else mean_.clear();
}

const std::vector<float>& PCA::getMean() const {
  if (!mean_flg_) throw Error(C3H_ERR_STATE, "PCA::getMean: There is no mean vector (mean_flg=false).");
  return mean_;
}

namespace {
constexpr size_t kPcaBatchRows = 4096;  // host rows per c3h_pca_add_data call
}

PCA::~PCA() { c3h_pca_destroy(h_); }

c3h_pca* PCA::handle() {
  if (!h_) {
    int rc = c3h_pca_create(device_, mean_flg_ ? 1 : 0, &h_);
    if (rc != C3H_OK) throw Error(rc, "PCA: c3h_pca_create failed");
  }
  return h_;
}

void PCA::flush(bool rotated) {
  std::vector<float>& r = rows_[rotated ? 1 : 0];
  if (r.empty()) return;
  const int64_t n = (int64_t)(r.size() / F_);
  int rc = c3h_pca_add_data(handle(), r.data(), n, F_, F_, rotated ? 1 : 0, 0);
  r.clear();
  if (rc != C3H_OK) throw Error(rc, std::string("PCA::addData: ") + c3h_pca_last_error(h_));
}

void PCA::addData(const std::vector<float>& feature) {
  if (F_ == -1) F_ = (int)feature.size();
  if ((int)feature.size() != F_) throw Error(C3H_ERR_ARG, "PCA::addData: vector size differs");
  rows_[0].insert(rows_[0].end(), feature.begin(), feature.end());
  if (rows_[0].size() >= kPcaBatchRows * F_) flush(false);
}

void PCA::addDataRotated24(const std::vector<float>& feature) {
  if (F_ == -1) F_ = (int)feature.size();
  if ((int)feature.size() != F_) throw Error(C3H_ERR_ARG, "PCA::addData: vector size differs");
  rows_[1].insert(rows_[1].end(), feature.begin(), feature.end());
  if (rows_[1].size() >= kPcaBatchRows * F_) flush(true);
}

void PCA::setCompress(const MatrixXf& axis, const std::vector<float>& variance, int dim, bool whitening) {
  const int F = axis.rows;
  if (dim <= 0 || dim > axis.cols || (whitening && (int)variance.size() < dim))
    throw Error(C3H_ERR_ARG, "PCA::setCompress: bad dimension");
  std::vector<float> col((size_t)F * dim);  // column d contiguous
  for (int d = 0; d < dim; ++d)
    for (int f = 0; f < F; ++f) col[(size_t)d * F + f] = axis(f, d);
  int rc = c3h_pca_set_compress(handle(), col.data(), whitening ? variance.data() : nullptr, F, dim);
  if (rc != C3H_OK) throw Error(rc, std::string("PCA::setCompress: ") + c3h_pca_last_error(h_));
}

void PCA::solve(bool regularization_flg, float regularization_nolm) {
  flush(false);
  flush(true);
  c3h_pca* h = handle();
  int rc = c3h_pca_solve(h, regularization_flg ? 1 : 0, regularization_nolm);
  if (rc != C3H_OK) throw Error(rc, std::string("PCA::solve: ") + c3h_pca_last_error(h));
  const int dim = c3h_pca_get(h, nullptr, nullptr, nullptr, nullptr, 0);
  if (dim < 0) throw Error(dim, "PCA::solve: get");
  std::vector<float> col((size_t)dim * dim);
  variance_.assign(dim, 0.f);
  mean_.assign(mean_flg_ ? dim : 0, 0.f);
  rc = c3h_pca_get(h, col.data(), variance_.data(), mean_flg_ ? mean_.data() : nullptr, nullptr, 0);
  if (rc < 0) throw Error(rc, "PCA::solve: get");
  axis_ = MatrixXf(dim, dim);
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) axis_(j, i) = col[(size_t)i * dim + j];
}

void PCA::write(const char* filename, bool ascii) const {
  const int dim = (int)variance_.size();
  std::vector<float> col((size_t)dim * dim);
  for (int i = 0; i < dim; ++i)
    for (int j = 0; j < dim; ++j) col[(size_t)i * dim + j] = axis_(j, i);
  int rc = c3h_pca_write(filename, ascii ? 1 : 0, dim, col.data(), variance_.data(),
                         mean_flg_ ? mean_.data() : nullptr);
  if (rc != C3H_OK) throw Error(rc, std::string("PCA::write: cannot write ") + filename);
}

void rotateFeature90(std::vector<float>& output, const std::vector<float>& input, RotateMode mode) {
  const int dim = (int)input.size();
  std::vector<int32_t> map(dim);
  int rc = c3h_rotate_map(dim, (int32_t)mode, map.data());
  if (rc != C3H_OK) throw Error(rc, "rotateFeature90: improper dimension");
  output.resize(dim);
  for (int o = 0; o < dim; ++o) output[o] = input[map[o]];
}

// ------------------------------------------------------------------------- Param
float Param::readVoxelSize(const char* f) {
  float v;
  return read_param(f, "voxel_size:", v) && v > 0 ? v : -1.0f;
}
int Param::readDim(const char* f) {
  int v;
  return read_param(f, "dim:", v) && v >= 1 ? v : -1;
}
int Param::readBoxSizeScene(const char* f) {
  int v;
  return read_param(f, "box_size(scene):", v) && v >= 1 ? v : -1;
}
int Param::readBoxSizeModel(const char* f) {
  int v;
  return read_param(f, "box_size(model):", v) && v >= 1 ? v : -1;
}
int Param::readRotateNum(const char* f) {
  int v;
  return read_param(f, "rotate_num:", v) && v >= 1 ? v : -1;
}
int Param::readC3HLACFlag(const char* f) {
  int v;
  return read_param(f, "c3_hlac_flg:", v) ? v : -1;
}
void Param::readColorThreshold(int& r, int& g, int& b, const char* f) {
  std::ifstream in(f);
  if (!in || !(in >> r >> g >> b)) throw Error(C3H_ERR_NOTFOUND, std::string("Param::readColorThreshold: ") + f);
}

// ------------------------------------------------------------------------- SearchObj
void SearchObj::setRange(int r1, int r2, int r3) {
  range_[0] = r1;
  range_[1] = r2;
  range_[2] = r3;
}

void SearchObj::setRank(int rank_num) {
  rank_ = rank_num;
  ctx_.check(c3h_set_rank(ctx_.get(), rank_num), "c3h_set_rank");
  dets_.assign((size_t)model_num_ * rank_, c3h_det{0.0, 0, 0, 0, C3H_S_MODE_1});
}

// readAxis (search.cpp:153-165): the first dim_model eigenvectors as rows; rows i >= 1
// scaled by sqrt(var_i)/sqrt(var_0) over the first `dim` columns (double arithmetic).
static MatrixXf read_model_axis(const char* filename, int dim, int dim_model, bool ascii, bool ms) {
  PCA pca;
  pca.read(filename, ascii);
  const MatrixXf& a = pca.getAxis();
  if (dim_model > a.cols) throw Error(C3H_ERR_ARG, "readAxis: dim_model exceeds the PCA dimension");
  MatrixXf q(dim_model, a.rows);
  for (int i = 0; i < dim_model; ++i)
    for (int j = 0; j < a.rows; ++j) q(i, j) = a(j, i);
  if (ms) {
    const std::vector<float>& v = pca.getVariance();
    for (int i = 1; i < dim_model; ++i)
      for (int j = 0; j < dim && j < a.rows; ++j)
        q(i, j) = (float)((double)q(i, j) * std::sqrt((double)v[i]) / std::sqrt((double)v[0]));
  }
  return q;
}

void SearchObj::readAxis(const char* filename, int dim, int dim_model, bool ascii, bool ms) {
  axis_q_.assign(1, read_model_axis(filename, dim, dim_model, ascii, ms));
  model_dim_ = dim_model;
  setup_dirty_ = true;
}

void SearchObj::getRange(int& xr, int& yr, int& zr, SearchMode mode) const {
  xr = xRange(mode);
  yr = yRange(mode);
  zr = zRange(mode);
}

// xRange / yRange / zRange (search.cpp:260-317)
int SearchObj::xRange(SearchMode m) const {
  switch (m) {
    case S_MODE_1: case S_MODE_2: return range_[0];
    case S_MODE_3: case S_MODE_4: return range_[1];
    case S_MODE_5: case S_MODE_6: return range_[2];
  }
  return 0;
}
int SearchObj::yRange(SearchMode m) const {
  switch (m) {
    case S_MODE_3: case S_MODE_5: return range_[0];
    case S_MODE_1: case S_MODE_6: return range_[1];
    case S_MODE_2: case S_MODE_4: return range_[2];
  }
  return 0;
}
int SearchObj::zRange(SearchMode m) const {
  switch (m) {
    case S_MODE_4: case S_MODE_6: return range_[0];
    case S_MODE_2: case S_MODE_5: return range_[1];
    case S_MODE_1: case S_MODE_3: return range_[2];
  }
  return 0;
}

const c3h_det& SearchObj::det(int m, int num) const {
  const size_t i = (size_t)m * rank_ + num;
  if (m < 0 || m >= model_num_ || num < 0 || num >= rank_ || i >= dets_.size())
    throw Error(C3H_ERR_ARG, "SearchObj: detection index out of range");
  return dets_[i];
}

void SearchObj::setSceneAxis(const MatrixXf& axis) {
  axis_p_ = axis;
  compress_ = true;
  setup_dirty_ = true;
}

// setSceneAxis with whitening (search.cpp:701-712): row i scaled by float(1/sqrt(var_i))
void SearchObj::setSceneAxis(const MatrixXf& axis, const std::vector<float>& var, int dim) {
  (void)dim;
  if ((int)var.size() < axis.rows) throw Error(C3H_ERR_ARG, "setSceneAxis: variance shorter than the axis");
  axis_p_ = axis;
  for (int i = 0; i < axis.rows; ++i) {
    const float s = (float)(1 / std::sqrt((double)var[i]));
    for (int j = 0; j < axis.cols; ++j) axis_p_(i, j) = s * axis_p_(i, j);
  }
  compress_ = true;
  setup_dirty_ = true;
}

void SearchObj::setNormalizeVal(const char* filename) {
  std::ifstream in(filename);
  if (!in) throw Error(C3H_ERR_NOTFOUND, std::string("setNormalizeVal: ") + filename);
  float v;
  while (in >> v) feature_max_.push_back(v);
  setup_dirty_ = true;
}

void SearchObj::cleanMax() {
  ctx_.check(c3h_clean_max(ctx_.get()), "c3h_clean_max");
  for (auto& d : dets_) {
    d.score = 0.0;
    d.x = d.y = d.z = 0;
  }
}

void SearchObj::cleanData() {
  xn_ = yn_ = zn_ = 0;
  cleanMax();
}

void SearchObj::ensureSetup(int F) {
  if (!setup_dirty_) return;
  if (axis_q_.empty()) throw Error(C3H_ERR_STATE, "SearchObj: readAxis has not been called");
  const int M = (int)axis_q_.size(), r = model_dim_;
  const int D = compress_ ? axis_p_.rows : F;
  if (compress_ && axis_p_.cols != F)
    throw Error(C3H_ERR_ARG, "SearchObj: scene axis width differs from the feature dimension");
  std::vector<float> q((size_t)M * r * D, 0.0f);
  for (int m = 0; m < M; ++m) {
    if (axis_q_[m].cols < D) throw Error(C3H_ERR_ARG, "SearchObj: model axis narrower than D");
    for (int i = 0; i < r; ++i)
      for (int d = 0; d < D; ++d) q[((size_t)m * r + i) * D + d] = axis_q_[m](i, d);
  }
  ctx_.check(c3h_search_setup(ctx_.get(), compress_ ? axis_p_.data.data() : nullptr, nullptr, D, F,
                              q.data(), M, r, feature_max_.empty() ? nullptr : feature_max_.data(),
                              (int)feature_max_.size()),
             "c3h_search_setup");
  if (rank_ < 1) setRank(1);
  else ctx_.check(c3h_set_rank(ctx_.get(), rank_), "c3h_set_rank");
  dets_.assign((size_t)model_num_ * rank_, c3h_det{0.0, 0, 0, 0, C3H_S_MODE_1});
  setup_dirty_ = false;
}

void SearchObj::readData(const char* filenameF, const char* filenameN, int dim, bool ascii) {
  if (dim < 1) throw Error(C3H_ERR_ARG, "readData: dim");
  FILE* fp = fopen(filenameF, ascii ? "r" : "rb");
  FILE* fp2 = fopen(filenameN, ascii ? "r" : "rb");
  if (!fp || !fp2) {
    if (fp) fclose(fp);
    if (fp2) fclose(fp2);
    throw Error(C3H_ERR_NOTFOUND, "readData: cannot open the integral tables");
  }
  int n3[3] = {0, 0, 0};
  bool ok = ascii ? fscanf(fp, "%d %d %d\n", &n3[0], &n3[1], &n3[2]) == 3 : fread(n3, sizeof(int), 3, fp) == 3;
  ok = ok && n3[0] > 0 && n3[1] > 0 && n3[2] > 0;
  const int64_t H = ok ? (int64_t)n3[0] * n3[1] * n3[2] : 0;
  std::vector<double> I((size_t)H * dim);
  std::vector<int64_t> E((size_t)H);
  for (int64_t n = 0; n < H && ok; ++n) {
    for (int j = 0; j < dim && ok; ++j) {
      double v;
      if (ascii) {
        int idx;
        ok = fscanf(fp, "%d:%lf ", &idx, &v) == 2;
      } else {
        ok = fread(&v, sizeof(double), 1, fp) == 1;
      }
      I[(size_t)n * dim + j] = (double)(float)v;  // integral_features is VectorXf
    }
    int e = 0;
    ok = ok && (ascii ? fscanf(fp2, "%d\n", &e) == 1 : fread(&e, sizeof(int), 1, fp2) == 1);
    E[(size_t)n] = e;
  }
  fclose(fp);
  fclose(fp2);
  if (!ok) throw Error(C3H_ERR_FORMAT, "readData: malformed integral tables");
  // per-subdivision values: 3-D differences of the summed-volume tables (search.cpp:579-653)
  const int X = n3[0], Y = n3[1];
  auto at = [&](int x, int y, int z) -> int64_t { return x < 0 || y < 0 || z < 0 ? -1 : x + (int64_t)X * (y + (int64_t)Y * z); };
  std::vector<float> cell((size_t)H * dim);
  std::vector<int32_t> ex((size_t)H);
  for (int z = 0; z < n3[2]; ++z)
    for (int y = 0; y < Y; ++y)
      for (int x = 0; x < X; ++x) {
        const int64_t id[8] = {at(x, y, z), at(x - 1, y, z), at(x, y - 1, z), at(x - 1, y - 1, z),
                               at(x, y, z - 1), at(x - 1, y, z - 1), at(x, y - 1, z - 1), at(x - 1, y - 1, z - 1)};
        const int sg[8] = {1, -1, -1, 1, -1, 1, 1, -1};
        const int64_t h = id[0];
        int64_t e = 0;
        for (int k = 0; k < 8; ++k)
          if (id[k] >= 0) e += sg[k] * E[(size_t)id[k]];
        ex[(size_t)h] = (int32_t)e;
        for (int j = 0; j < dim; ++j) {
          double v = 0;
          for (int k = 0; k < 8; ++k)
            if (id[k] >= 0) v += sg[k] * I[(size_t)id[k] * dim + j];
          cell[(size_t)h * dim + j] = (float)v;
        }
      }
  compress_ = false;  // the tables hold compressed features already
  axis_p_ = MatrixXf();
  setup_dirty_ = true;
  ensureSetup(dim);
  const int32_t sb[3] = {n3[0], n3[1], n3[2]};
  ctx_.check(c3h_set_features(ctx_.get(), cell.data(), sb, dim, ex.data(), 0, 0), "c3h_set_features");
  setDataFromContext(Vector3i{n3[0], n3[1], n3[2]});
}

void SearchObj::setDataFromContext(const Vector3i& subdiv_b) {
  xn_ = subdiv_b[0];
  yn_ = subdiv_b[1];
  zn_ = subdiv_b[2];
}

void SearchObj::run(bool rotate, bool remove_overlap) {
  const double t0 = now_s();
  const int M = (int)axis_q_.size();
  std::vector<c3h_det> out((size_t)std::max(M, 1) * std::max(rank_, 1));
  const int rc = c3h_search(ctx_.get(), range_, threshold_, rotate ? 1 : 0, remove_overlap ? 1 : 0,
                            out.data());
  ctx_.check(rc, "c3h_search");
  if (rc > 0) dets_ = out;
  search_time = now_s() - t0;
}

void SearchObj::search() { run(true, false); }
void SearchObj::searchWithoutRotation() { run(false, false); }

// writeResult (search.cpp:662-679)
void SearchObj::writeResult(const char* filename, int box_size) {
  FILE* fp = fopen(filename, "w");
  if (!fp) throw Error(C3H_ERR_NOTFOUND, std::string("writeResult: ") + filename);
  for (int r = 0; r < rank_; ++r) {
    const c3h_det& d = det(0, r);
    if (d.score == 0) break;
    int xr, yr, zr;
    getRange(xr, yr, zr, (SearchMode)d.mode);
    fprintf(fp, "%d %d %d %d %d %d %f\n", d.x * box_size, xr * box_size, d.y * box_size,
            yr * box_size, d.z * box_size, zr * box_size, d.score);
  }
  fprintf(fp, "time: %f\n", search_time);
  fclose(fp);
}

// ------------------------------------------------------------------------- SearchObjMulti
void SearchObjMulti::setRank(int rank_num) { SearchObj::setRank(rank_num); }

void SearchObjMulti::readAxis(char** filename, int dim, int dim_model, bool ascii, bool ms) {
  axis_q_.clear();
  for (int m = 0; m < model_num_; ++m)
    axis_q_.push_back(read_model_axis(filename[m], dim, dim_model, ascii, ms));
  model_dim_ = dim_model;
  setup_dirty_ = true;
}

// removeOverlap (search.cpp:972-992) on the lists of the last search
void SearchObjMulti::removeOverlap() {
  if (dets_.empty()) return;
  ctx_.check(c3h_remove_overlap(model_num_, rank_, range_, dets_.data()), "c3h_remove_overlap");
}

// SearchObjMulti::cleanData (search.cpp:760-770) keeps the lists
void SearchObjMulti::cleanData() { xn_ = yn_ = zn_ = 0; }

// ------------------------------------------------------------------------- setC3HLAC
static void set_c3hlac(SearchObj& so, int F, int thr_r, int thr_g, int thr_b, const VoxelGrid& grid,
                       double voxel_size, int subdiv) {
  const Context& ctx = so.context();
  // bind the grid's device buffer into the search context without a copy
  const uint32_t* words = nullptr;
  grid.context().check(c3h_grid_device_ptr(grid.context().get(), &words), "c3h_grid_device_ptr");
  c3h_grid_info gi;
  grid_info(grid.context(), &gi);
  if ((float)voxel_size != gi.leaf)
    throw Error(C3H_ERR_ARG, "setC3HLAC: voxel_size differs from the grid's leaf size");
  ctx.check(c3h_set_grid(ctx.get(), words, gi.div_b, gi.min_b, gi.leaf, 1), "c3h_set_grid");
  c3h_extract_params p;
  p.variant = F;
  p.thr[0] = thr_r;
  p.thr[1] = thr_g;
  p.thr[2] = thr_b;
  p.subdiv = subdiv;
  p.offset[0] = p.offset[1] = p.offset[2] = 0;
  p.color_mode = C3H_COLOR_C3_DOUBLE;
  int32_t sb[3];
  int64_t hist_num = 0;
  ctx.check(c3h_extract(ctx.get(), &p, sb, &hist_num), "c3h_extract");
  so.setDataFromContext(v3(sb));
}

void SearchC3HLAC::setC3HLAC(int dim, int r, int g, int b, const VoxelGrid& grid, double voxel_size,
                             int subdiv) {
  (void)dim;
  ensureSetup(C3H_VARIANT_981);
  set_c3hlac(*this, C3H_VARIANT_981, r, g, b, grid, voxel_size, subdiv);
}

void SearchC3HLACMulti::setC3HLAC(int dim, int r, int g, int b, const VoxelGrid& grid,
                                  double voxel_size, int subdiv) {
  (void)dim;
  ensureSetup(C3H_VARIANT_981);
  set_c3hlac(*this, C3H_VARIANT_981, r, g, b, grid, voxel_size, subdiv);
}

// setVOSCH / setGRSD (search_new.h:34-76): features on the grid's context, handed to the
// search context with their exist rule (setData)
static void set_external(SearchObj& so, VoxelGrid& grid, double voxel_size, int subdiv, const int* thr) {
  std::vector<std::vector<float> > f;
  const Vector3i sb = grsd_like(grid, f, (float)voxel_size, subdiv, 0, 0, 0, false, thr);
  const int F = thr ? 137 : 20;
  std::vector<float> flat;
  flat.reserve(f.size() * F);
  for (const auto& row : f) flat.insert(flat.end(), row.begin(), row.end());
  const int32_t sbv[3] = {sb[0], sb[1], sb[2]};
  const Context& ctx = so.context();
  ctx.check(c3h_set_features(ctx.get(), flat.empty() ? nullptr : flat.data(), sbv, F, nullptr,
                             thr ? C3H_EXIST_VOSCH : C3H_EXIST_GRSD, 0),
            "c3h_set_features");
  so.setDataFromContext(sb);
}

void SearchVOSCH::setVOSCH(int dim, int r, int g, int b, VoxelGrid& grid, double voxel_size, int subdiv) {
  (void)dim;
  ensureSetup(137);
  const int thr[3] = {r, g, b};
  set_external(*this, grid, voxel_size, subdiv, thr);
}

void SearchVOSCHMulti::setVOSCH(int dim, int r, int g, int b, VoxelGrid& grid, double voxel_size, int subdiv) {
  (void)dim;
  ensureSetup(137);
  const int thr[3] = {r, g, b};
  set_external(*this, grid, voxel_size, subdiv, thr);
}

void SearchGRSD::setGRSD(int dim, VoxelGrid& grid, double voxel_size, int subdiv) {
  (void)dim;
  ensureSetup(20);
  set_external(*this, grid, voxel_size, subdiv, nullptr);
}

}  // namespace c3hlac
