// c3hlac_host.h -- C++ facade with the reference's API names over the C-ABI
// (include/c3hlac_mi355x.h).  A caller of the reference's
//   getVoxelGrid / extractC3HLACSignature981/117   (c3_hlac/include/c3_hlac/c3_hlac_tools.h:53-89)
//   SearchObj / SearchObjMulti                     (color_voxel_recognition/include/color_voxel_recognition/search.h:53-270)
//   SearchC3HLAC / SearchC3HLACMulti               (.../search_c3_hlac.h:44-88)
//   PCA::read                                      (.../pca.h:60-72, src/pca.cpp:119-185)
//   Param                                          (.../param.h, src/param.cpp:43-222)
// switches by replacing the PCL/Eigen types with the small value types below.
//
// Differences that are deliberate (documented in INTEGRATION.md):
//   - the voxel grid lives on the GPU: `VoxelGrid` owns a device context, and the
//     downsampled cloud is only materialised when asked for (getVoxelGrid's `output`);
//   - errors raise c3hlac::Error instead of exit()/stderr, except where the reference
//     reports through a return value (setVoxelFilter's bool -> empty features, Param's -1);
//   - SearchObj::search_time is measured on the host around the whole search call.
#ifndef C3HLAC_HOST_H_
#define C3HLAC_HOST_H_

#include <algorithm>
#include <cmath>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "c3hlac_mi355x.h"

namespace c3hlac {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

// pcl::PointXYZRGB as stored in binary PCD files: rgb is the packed 0x00RRGGBB in the
// float's bits (pcl_cloud layout minus the SSE padding).
struct PointXYZRGB {
  float x, y, z, rgb;
};

struct Vector3i {  // Eigen::Vector3i
  int v[3] = {0, 0, 0};
  int& operator[](int i) { return v[i]; }
  int operator[](int i) const { return v[i]; }
  int x() const { return v[0]; }
  int y() const { return v[1]; }
  int z() const { return v[2]; }
};

// Row-major dense float matrix (stand-in for Eigen::MatrixXf in the search API).
struct MatrixXf {
  int rows = 0, cols = 0;
  std::vector<float> data;
  MatrixXf() = default;
  MatrixXf(int r, int c) : rows(r), cols(c), data((size_t)r * c, 0.0f) {}
  float& operator()(int r, int c) { return data[(size_t)r * cols + c]; }
  float operator()(int r, int c) const { return data[(size_t)r * cols + c]; }
};

// One device + one HIP stream (c3h_ctx); shared by the objects bound to it.
class Context {
 public:
  explicit Context(int hip_device = 0);
  c3h_ctx* get() const { return ctx_.get(); }
  void check(int rc, const char* what) const;
  void setStream(void* hip_stream);
  void synchronize();

 private:
  std::shared_ptr<c3h_ctx> ctx_;
};

// pcl::VoxelGrid<PointXYZRGB> after filter(): the packed colour/occupancy grid on the GPU.
class VoxelGrid {
 public:
  explicit VoxelGrid(int hip_device = 0) : ctx_(hip_device) {}
  explicit VoxelGrid(const Context& ctx) : ctx_(ctx) {}
  void setLeafSize(float lx, float ly, float lz);
  void setSaveLeafLayout(bool) {}  // the leaf layout is always derivable (getLeafLayout)
  Vector3i getNrDivisions() const;
  Vector3i getMinBoxCoordinates() const;
  Vector3i getMaxBoxCoordinates() const;
  std::vector<int> getLeafLayout() const;
  // the grid of an external producer (same packing as c3h_get_grid)
  void setPackedGrid(const uint32_t* words, const Vector3i& div_b, const Vector3i& min_b, float leaf,
                     bool on_device);
  std::vector<uint32_t> getPackedGrid() const;
  const Context& context() const { return ctx_; }
  float leaf() const { return leaf_; }

 private:
  friend void getVoxelGrid(VoxelGrid&, const std::vector<PointXYZRGB>&, std::vector<PointXYZRGB>&,
                           float, float);
  Context ctx_;
  float leaf_ = 0.0f;
};

// getVoxelGrid (c3_hlac_tools.hpp:124-130), with detect_object.cpp's limitPoint
// (z >= z_limit or non-finite points dropped) folded in.
void getVoxelGrid(VoxelGrid& grid, const std::vector<PointXYZRGB>& input,
                  std::vector<PointXYZRGB>& output, float voxel_size,
                  float z_limit = std::numeric_limits<float>::infinity());

// extractC3HLACSignature981/117 (c3_hlac_tools.hpp:134-202).  `color_mode` selects the
// setColor table (C3H_COLOR_*: C3 sin/cos in double -- the reference build's default -- or
// float; C3H_COLOR_CHLAC is extractColorCHLACSignature*'s, below).
Vector3i extractC3HLACSignature981(VoxelGrid& grid, std::vector<std::vector<float> >& feature,
                                   int color_threshold_r, int color_threshold_g,
                                   int color_threshold_b, float voxel_size,
                                   int subdivision_size = 0, int offset_x = 0, int offset_y = 0,
                                   int offset_z = 0, int color_mode = C3H_COLOR_C3_DOUBLE);
void extractC3HLACSignature981(VoxelGrid& grid, std::vector<float>& feature, int color_threshold_r,
                               int color_threshold_g, int color_threshold_b, float voxel_size,
                               int color_mode = C3H_COLOR_C3_DOUBLE);
Vector3i extractC3HLACSignature117(VoxelGrid& grid, std::vector<std::vector<float> >& feature,
                                   int color_threshold_r, int color_threshold_g,
                                   int color_threshold_b, float voxel_size,
                                   int subdivision_size = 0, int offset_x = 0, int offset_y = 0,
                                   int offset_z = 0, int color_mode = C3H_COLOR_C3_DOUBLE);
void extractC3HLACSignature117(VoxelGrid& grid, std::vector<float>& feature, int color_threshold_r,
                               int color_threshold_g, int color_threshold_b, float voxel_size,
                               int color_mode = C3H_COLOR_C3_DOUBLE);

// ---- the pcl::Feature-style estimators (c3_hlac/include/c3_hlac/c3_hlac.h:42-220) -----
const int DIM_C3HLAC_981_1_3 = 495;
const int DIM_C3HLAC_981_BIN_1_3 = 486;
const int DIM_C3HLAC_981_1_3_ALL = 981;
const int DIM_C3HLAC_117_1_3 = 63;
const int DIM_C3HLAC_117_BIN_1_3 = 54;
const int DIM_C3HLAC_117_1_3_ALL = 117;
struct C3HLACSignature117 {  // c3_hlac.h:50-53
  float histogram[117];
};
struct C3HLACSignature981 {  // c3_hlac.h:61-64
  float histogram[981];
};

// pcl::PointXYZRGBNormal (the estimators' second point type, c3_hlac.cpp:423-426): 8 floats
// here (x, y, z, rgb bits, normal, curvature; no SSE padding)
struct PointXYZRGBNormal {
  float x, y, z, rgb;
  float normal_x, normal_y, normal_z, curvature;
};
// getVoxelGrid for PointXYZRGBNormal clouds: the grid and the centroids' xyz and colour are
// those of the xyzrgb part (c3h_voxelize); normals and curvature are averaged per voxel in
// fp32 in input order, as VoxelGrid::filter averages every float field.
void getVoxelGrid(VoxelGrid& grid, const std::vector<PointXYZRGBNormal>& input,
                  std::vector<PointXYZRGBNormal>& output, float voxel_size,
                  float z_limit = std::numeric_limits<float>::infinity());

namespace detail {
// setVoxelFilter (c3_hlac.cpp:204-231): the offset check and getSubdivNum arithmetic
bool voxel_filter(const VoxelGrid& grid, int subdiv, const int off[3], Vector3i& subdiv_b);
// computeFeature (c3_hlac.cpp:303-324, 395-416) on the grid's device context: hist_num rows
// of `dim` floats (0 rows for the silent-empty cases)
int64_t compute_feature(VoxelGrid& grid, int dim, const int thr[3], int subdiv, const int off[3],
                        int color_mode, std::vector<float>& flat);
int64_t grid_occupied(const VoxelGrid& grid);  // n_occ of the grid (-1: not from getVoxelGrid)
}  // namespace detail

// C3HLAC117Estimation<PointT, PointOutT> (c3_hlac.h:79-155): rotation-invariant C3-HLAC of
// the subdivisions of a voxel grid.  The input cloud is the grid's downsampled cloud (as
// extractC3HLACSignature117 passes it, c3_hlac_tools.hpp:169-195); the grid on the device
// already holds its voxels' colours and centroids, so compute() checks the cloud's size
// against the grid and reads nothing else from it.  Deviations: setVoxelFilter keeps a copy
// of the VoxelGrid handle, which shares the device grid (re-voxelising into the same
// VoxelGrid changes what compute() sees); compute() without a successful setVoxelFilter
// throws; the silent-empty cases (a negative threshold) leave `output` empty where PCL's
// Feature::compute leaves indices_->size() uninitialised points.
template <typename PointT, typename PointOutT>
class C3HLAC117Estimation {
 public:
  C3HLAC117Estimation() : feature_name_("C3HLAC117Estimation") {}
  virtual ~C3HLAC117Estimation() = default;
  // setColorThreshold (c3_hlac.h:92)
  void setColorThreshold(int threshold_r, int threshold_g, int threshold_b) {
    thr_[0] = threshold_r;
    thr_[1] = threshold_g;
    thr_[2] = threshold_b;
  }
  // setVoxelFilter (c3_hlac.h:102, c3_hlac.cpp:204-231): false when an offset reaches the
  // grid size or the subdivision size is negative
  bool setVoxelFilter(const VoxelGrid& grid, int subdivision_size = 0, int offset_x = 0, int offset_y = 0,
                      int offset_z = 0, float voxel_size = 0.01f) {
    grid_ = std::make_shared<VoxelGrid>(grid);
    subdiv_ = subdivision_size;
    off_[0] = offset_x;
    off_[1] = offset_y;
    off_[2] = offset_z;
    voxel_size_ = voxel_size;
    filter_ok_ = detail::voxel_filter(grid, subdivision_size, off_, subdiv_b_);
    return filter_ok_;
  }
  Vector3i getSubdivNum() const { return subdiv_b_; }  // c3_hlac.h:105
  void setInputCloud(const std::vector<PointT>& cloud) { cloud_ = &cloud; }
  // the radius search extractC3HLACSignature* sets is "not used actually" (c3_hlac_tools.hpp:140-141)
  void setRadiusSearch(double) {}
  template <class Tree>
  void setSearchMethod(const Tree&) {}
  // setColor's sin/cos evaluation (double = the reference build's, see c3h_extract_params)
  void setLUTDouble(bool lut_double) { color_mode_ = lut_double ? C3H_COLOR_C3_DOUBLE : C3H_COLOR_C3_FLOAT; }
  void setColorMode(int color_mode) { color_mode_ = color_mode; }  // C3H_COLOR_*
  const std::string& getFeatureName() const { return feature_name_; }
  // Feature::compute -> computeFeature: one PointOutT per subdivision (hist_num of them)
  void compute(std::vector<PointOutT>& output) {
    if (!grid_ || !filter_ok_) throw Error(C3H_ERR_STATE, feature_name_ + "::compute: no valid setVoxelFilter");
    if (grid_->leaf() != 0.0f && voxel_size_ != grid_->leaf())
      throw Error(C3H_ERR_ARG, feature_name_ + "::compute: voxel_size differs from the grid's leaf size");
    const int64_t nocc = detail::grid_occupied(*grid_);
    if (cloud_ && nocc >= 0 && (int64_t)cloud_->size() != nocc)
      throw Error(C3H_ERR_ARG, feature_name_ + "::compute: the input cloud is not the grid's downsampled cloud");
    const int d = dim();
    if ((size_t)d * sizeof(float) > sizeof(PointOutT))  // c3_hlac.cpp:422 instantiates 981 -> Signature117
      throw Error(C3H_ERR_ARG, feature_name_ + "::compute: the output type holds fewer than " + std::to_string(d) +
                                   " floats");
    std::vector<float> flat;
    const int64_t hn = detail::compute_feature(*grid_, d, thr_, subdiv_, off_, color_mode_, flat);
    output.assign((size_t)hn, PointOutT());
    for (int64_t h = 0; h < hn; ++h) {
      float* dst = reinterpret_cast<float*>(&output[h]);
      std::fill(dst, dst + sizeof(PointOutT) / sizeof(float), 0.0f);
      std::copy(flat.begin() + h * d, flat.begin() + (h + 1) * d, dst);
    }
  }

 protected:
  virtual int dim() const { return DIM_C3HLAC_117_1_3_ALL; }
  std::string feature_name_;
  std::shared_ptr<VoxelGrid> grid_;
  const std::vector<PointT>* cloud_ = nullptr;
  int thr_[3] = {-1, -1, -1};  // the constructor's -1 (c3_hlac.cpp:178): compute() then returns empty
  int subdiv_ = 0, off_[3] = {0, 0, 0};
  float voxel_size_ = 0.0f;
  bool filter_ok_ = false;
  int color_mode_ = C3H_COLOR_C3_DOUBLE;
  Vector3i subdiv_b_;
};

// C3HLAC981Estimation<PointT, PointOutT> (c3_hlac.h:158-220): rotation-variant, 981 bins
template <typename PointT, typename PointOutT>
class C3HLAC981Estimation : public C3HLAC117Estimation<PointT, PointOutT> {
 public:
  C3HLAC981Estimation() { this->feature_name_ = "C3HLAC981Estimation"; }

 protected:
  int dim() const override { return DIM_C3HLAC_981_1_3_ALL; }
};

// ColorCHLAC_RI_Estimation / ColorCHLACEstimation (color_chlac/include/color_chlac/
// color_chlac.h): the same estimators with ColorCHLAC's setColor (r_ = 255 - r,
// color_chlac.hpp:148-153); bins and normalisation constants are the C3 ones.
template <typename PointT, typename PointOutT>
class ColorCHLAC_RI_Estimation : public C3HLAC117Estimation<PointT, PointOutT> {
 public:
  ColorCHLAC_RI_Estimation() {
    this->feature_name_ = "ColorCHLAC_RI_Estimation";
    this->color_mode_ = C3H_COLOR_CHLAC;
  }
};
template <typename PointT, typename PointOutT>
class ColorCHLACEstimation : public C3HLAC117Estimation<PointT, PointOutT> {
 public:
  ColorCHLACEstimation() {
    this->feature_name_ = "ColorCHLACEstimation";
    this->color_mode_ = C3H_COLOR_CHLAC;
  }

 protected:
  int dim() const override { return DIM_C3HLAC_981_1_3_ALL; }
};
// extractColorCHLACSignature981/117 (grsd_colorCHLAC_tools.hpp:680-747)
Vector3i extractColorCHLACSignature981(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int thR,
                                       int thG, int thB, float voxel_size, int subdivision_size = 0,
                                       int offset_x = 0, int offset_y = 0, int offset_z = 0);
void extractColorCHLACSignature981(VoxelGrid& grid, std::vector<float>& feature, int thR, int thG, int thB,
                                   float voxel_size);
Vector3i extractColorCHLACSignature117(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int thR,
                                       int thG, int thB, float voxel_size, int subdivision_size = 0,
                                       int offset_x = 0, int offset_y = 0, int offset_z = 0);
void extractColorCHLACSignature117(VoxelGrid& grid, std::vector<float>& feature, int thR, int thG, int thB,
                                   float voxel_size);

// VOSCH / GRSD (color_chlac/include/color_chlac/grsd_colorCHLAC_tools.h:27-32, .hpp:63-296,
// 832-843) on the grid's cloud: computeNormal (radius normals_radius_search) runs on the
// points the grid was built from (PCL's normals are not a field of PointXYZRGB here: they
// stay on the device); extractGRSDSignature21 computes them first when needed.
const double rsd_radius_search = 0.01;
const double normals_radius_search = 0.02;
void computeNormal(VoxelGrid& grid, double radius = normals_radius_search);
std::vector<float> getNormals(const VoxelGrid& grid);  // n x 4: nx, ny, nz, curvature
Vector3i extractGRSDSignature21(VoxelGrid& grid, std::vector<std::vector<float> >& feature, float voxel_size,
                                int subdivision_size = 0, int offset_x = 0, int offset_y = 0, int offset_z = 0,
                                bool is_normalize = false);
Vector3i extractVOSCH(VoxelGrid& grid, std::vector<std::vector<float> >& feature, int thR, int thG, int thB,
                      float voxel_size, int subdivision_size = 0, int offset_x = 0, int offset_y = 0,
                      int offset_z = 0, bool is_normalize = false);

// pcl::io::loadPCDFile for x y z rgb clouds (c3h_pcd_read_xyzrgb): 0 on success, -1 when
// the file cannot be opened or parsed, as PCL returns.
int loadPCDFile(const std::string& file_name, std::vector<PointXYZRGB>& cloud);

// readFeature / writeFeature (c3_hlac_tools.hpp:46-113): ASCII feature PCD files.
void readFeature(const char* name, std::vector<std::vector<float> >& feature);
void readFeature(const char* name, std::vector<float>& feature);
void writeFeature(const char* name, const std::vector<std::vector<float> > feature, bool remove_0_flg = true);
void writeFeature(const char* name, const std::vector<float> feature, bool remove_0_flg = true);

// calc_scene_auto_threshold.cpp:84-146 as a class: addScene() per voxelised scene frame
// (histograms of its voxel colours, on the GPU), compute() the RGB binarisation thresholds.
class ColorThreshold {
 public:
  void addScene(const VoxelGrid& grid);
  void compute(int threshold[3], double total_average[3] = nullptr) const;
  const int64_t* histogram() const { return hist_; }  // [c * 256 + v], c = r, g, b

 private:
  int64_t hist_[768] = {};
};

// PCA file reader (pca.cpp:119-185).  getAxis() is dim x dim with eigenvector i in
// column i, as Eigen holds it.
class PCA {
 public:
  // PCA(bool _mean_flg = true) (pca.h:49); training runs on HIP device `hip_device`
  explicit PCA(bool mean_flg = true, int hip_device = 0) : mean_flg_(mean_flg), device_(hip_device) {}
  ~PCA();
  PCA(const PCA&) = delete;
  PCA& operator=(const PCA&) = delete;
  // addData (pca.cpp:48-69): rows are batched on the host and accumulated on the GPU
  void addData(const std::vector<float>& feature);
  // pca_models.cpp's training in one call: compressFeature with the scene axis (first
  // dim columns, whitened by variance unless whitening = false) applied to every vector
  // added afterwards (setCompress), and the 24 rotateFeature90 images of a feature
  // (addDataRotated24 = the 24 addData calls of pca_models.cpp:109-171)
  void setCompress(const MatrixXf& axis, const std::vector<float>& variance, int dim, bool whitening = true);
  void addDataRotated24(const std::vector<float>& feature);
  void solve(bool regularization_flg = false, float regularization_nolm = 0.0001f);
  void read(const char* filename, bool ascii = false);
  void write(const char* filename, bool ascii = false) const;
  const MatrixXf& getAxis() const { return axis_; }
  const std::vector<float>& getVariance() const { return variance_; }
  const std::vector<float>& getMean() const;
  int dim() const { return axis_.rows; }

 private:
  void flush(bool rotated);
  c3h_pca* handle();
  bool mean_flg_;
  int device_;
  c3h_pca* h_ = nullptr;
  int F_ = -1;
  std::vector<float> rows_[2];  // pending plain / rotated rows
  MatrixXf axis_;
  std::vector<float> variance_, mean_;
};

// pcl::rotateFeature90 (c3_hlac.cpp:49-172) on one host vector (an index gather)
enum RotateMode { R_MODE_1, R_MODE_2, R_MODE_3, R_MODE_4 };
void rotateFeature90(std::vector<float>& output, const std::vector<float>& input, RotateMode mode);

// Param (param.h): the same keys, defaults and -1 error returns.
struct Param {
  static float readVoxelSize(const char* filename = "param/parameters.txt");
  static int readDim(const char* filename = "param/parameters.txt");
  static int readBoxSizeScene(const char* filename = "param/parameters.txt");
  static int readBoxSizeModel(const char* filename = "param/parameters.txt");
  static int readRotateNum(const char* filename = "param/parameters.txt");
  static int readC3HLACFlag(const char* filename = "param/parameters.txt");
  static void readColorThreshold(int& r, int& g, int& b,
                                 const char* filename = "param/color_threshold.txt");
};

enum SearchMode { S_MODE_1, S_MODE_2, S_MODE_3, S_MODE_4, S_MODE_5, S_MODE_6 };

// SearchObj (search.h:53-176): single-model sliding-box search.  The integral table and
// scores live on the device; setC3HLAC extracts and binds the features in one call.
class SearchObj {
 public:
  double search_time = 0.0;
  explicit SearchObj(int hip_device = 0) : ctx_(hip_device) {}
  explicit SearchObj(const Context& ctx) : ctx_(ctx) {}
  virtual ~SearchObj() = default;

  void setRange(int range1, int range2, int range3);
  virtual void setRank(int rank_num);
  void setThreshold(int exist_voxel_num_threshold) { threshold_ = exist_voxel_num_threshold; }
  virtual void readAxis(const char* filename, int dim, int dim_model, bool ascii,
                        bool multiple_similarity);
  void getRange(int& xrange, int& yrange, int& zrange, SearchMode mode) const;
  void search();
  void searchWithoutRotation();
  void writeResult(const char* filename, int box_size);
  virtual void cleanMax();
  void setSceneAxis(const MatrixXf& axis);
  void setSceneAxis(const MatrixXf& axis, const std::vector<float>& var, int dim);
  virtual void cleanData();
  int XYnum() const { return xn_ * yn_; }
  int Znum() const { return zn_; }
  virtual int maxX(int num) const { return det(0, num).x; }
  virtual int maxY(int num) const { return det(0, num).y; }
  virtual int maxZ(int num) const { return det(0, num).z; }
  virtual SearchMode maxMode(int num) const { return (SearchMode)det(0, num).mode; }
  virtual double maxDot(int num) const { return det(0, num).score; }
  virtual int maxXrange(int num) const { return xRange(maxMode(num)); }
  virtual int maxYrange(int num) const { return yRange(maxMode(num)); }
  virtual int maxZrange(int num) const { return zRange(maxMode(num)); }
  void setNormalizeVal(const char* filename);
  // readData (search.cpp:169-210): the legacy integral tables of an already compressed scene
  // (dim values per subdivision, and the exist counts).  They are differenced back to
  // per-subdivision values (double) and searched without a scene axis (D = dim), the box
  // sums formed directly instead of clipValue's inclusion-exclusion.
  void readData(const char* filenameF, const char* filenameN, int dim, bool ascii);

  // setData (search.cpp:539-658) on features already extracted into this context
  void setDataFromContext(const Vector3i& subdiv_b);
  const Context& context() const { return ctx_; }
  // all M x rank detections of the last search (model-major)
  const std::vector<c3h_det>& detections() const { return dets_; }

 protected:
  Context ctx_;
  int range_[3] = {1, 1, 1};
  int rank_ = 0, threshold_ = 0, model_num_ = 1;
  int xn_ = 0, yn_ = 0, zn_ = 0;
  int model_dim_ = 0;                 // r
  std::vector<MatrixXf> axis_q_;      // per model r x D
  MatrixXf axis_p_;                   // D x F (already whitened when var given)
  bool compress_ = false, setup_dirty_ = true;
  std::vector<float> feature_max_;
  std::vector<c3h_det> dets_;
  int xRange(SearchMode m) const;
  int yRange(SearchMode m) const;
  int zRange(SearchMode m) const;
  const c3h_det& det(int m, int num) const;
  void ensureSetup(int F);
  void run(bool rotate, bool remove_overlap);
};

// SearchObjMulti (search.h:181-270): M models scored per position, one list per model.
class SearchObjMulti : public SearchObj {
 public:
  using SearchObj::SearchObj;
  void setModelNum(int model_num) { model_num_ = model_num; }
  void setRank(int rank_num) override;
  void readAxis(char** filename, int dim, int dim_model, bool ascii, bool multiple_similarity);
  int maxX(int m, int num) const { return det(m, num).x; }
  int maxY(int m, int num) const { return det(m, num).y; }
  int maxZ(int m, int num) const { return det(m, num).z; }
  SearchMode maxMode(int m, int num) const { return (SearchMode)det(m, num).mode; }
  double maxDot(int m, int num) const { return det(m, num).score; }
  int maxXrange(int m, int num) const { return xRange(maxMode(m, num)); }
  int maxYrange(int m, int num) const { return yRange(maxMode(m, num)); }
  int maxZrange(int m, int num) const { return zRange(maxMode(m, num)); }
  void removeOverlap();
  void cleanData() override;
};

// SearchC3HLAC{,Multi}::setC3HLAC (search_c3_hlac.h:53-88): C3-HLAC-981 of the grid,
// exist counts and setData, all on the device.  `cloud_downsampled` is not needed: the
// packed grid carries each voxel's colour.
class SearchC3HLAC : public SearchObj {
 public:
  using SearchObj::SearchObj;
  void setC3HLAC(int dim, int color_threshold_r, int color_threshold_g, int color_threshold_b,
                 const VoxelGrid& grid, double voxel_size, int subdivision_size);
};
class SearchC3HLACMulti : public SearchObjMulti {
 public:
  using SearchObjMulti::SearchObjMulti;
  void setC3HLAC(int dim, int color_threshold_r, int color_threshold_g, int color_threshold_b,
                 const VoxelGrid& grid, double voxel_size, int subdivision_size);
};
// SearchVOSCH{,Multi}::setVOSCH and SearchGRSD::setGRSD
// (color_voxel_recognition_2/include/color_voxel_recognition_2/search_new.h:34-76, 106-126):
// the features of extractVOSCH / extractGRSDSignature21 on the device, their exist rule,
// setData.  The grid must come from getVoxelGrid (it holds the cloud).
class SearchVOSCH : public SearchObj {
 public:
  using SearchObj::SearchObj;
  void setVOSCH(int dim, int color_threshold_r, int color_threshold_g, int color_threshold_b, VoxelGrid& grid,
                double voxel_size, int subdivision_size);
};
class SearchVOSCHMulti : public SearchObjMulti {
 public:
  using SearchObjMulti::SearchObjMulti;
  void setVOSCH(int dim, int color_threshold_r, int color_threshold_g, int color_threshold_b, VoxelGrid& grid,
                double voxel_size, int subdivision_size);
};
class SearchGRSD : public SearchObj {
 public:
  using SearchObj::SearchObj;
  void setGRSD(int dim, VoxelGrid& grid, double voxel_size, int subdivision_size);
};

}  // namespace c3hlac

#endif  // C3HLAC_HOST_H_
