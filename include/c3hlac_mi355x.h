/*
 * c3hlac_mi355x.h -- C-ABI of the MI355X (gfx950) colour-voxel C3-HLAC recognition path.
 *
 * This is the drop-in boundary: plain pointers and sizes, no PCL/Eigen/torch types.
 * Each entry point names the reference interface it replaces (paths relative to the
 * reference root).  The C++ facade in mapping-private_amd/host/ re-exposes the
 * reference's own names (getVoxelGrid, extractC3HLACSignature981/117, SearchObj,
 * SearchObjMulti, SearchC3HLAC, PCA, Param) on top of these functions.
 *
 * Conventions:
 *   - every function returns C3H_OK (0) or a negative C3H_ERR_* code; nothing calls exit();
 *     c3h_last_error() describes the last failure of a context;
 *   - output buffers are caller-owned; `on_device` selects whether a pointer is a HIP
 *     device pointer (1) or host memory (0);
 *   - one context = one device + one HIP stream; thread-compatible, not thread-safe
 *     (the reference's SearchObj model).
 */
#ifndef C3HLAC_MI355X_H_
#define C3HLAC_MI355X_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define C3H_OK 0
#define C3H_ERR_ARG -1       /* bad argument (null pointer, negative size, bad variant) */
#define C3H_ERR_HIP -2       /* HIP runtime error (message in c3h_last_error) */
#define C3H_ERR_STATE -3     /* call order: e.g. extract before voxelize */
#define C3H_ERR_NOMEM -4     /* device allocation failed */
#define C3H_ERR_RANGE -5     /* grid too large for int32 voxel indices */
#define C3H_ERR_NOTFOUND -6  /* file could not be opened (PCA / param readers) */
#define C3H_ERR_FORMAT -7    /* malformed file */

#define C3H_VARIANT_981 981  /* C3HLAC981Estimation (rotation-variant) */
#define C3H_VARIANT_117 117  /* C3HLAC117Estimation (rotation-invariant) */

/* setColor of the estimator (c3h_extract_params.color_mode): the six colour channels a
 * voxel contributes (r, r_, g, g_, b, b_).  C3HLAC{,_RI}Estimation (color_chlac/include/
 * color_chlac/color_chlac.hpp:155-179; c3_hlac_core's twin): r = 255 sin(v theta),
 * r_ = 255 cos(v theta), theta = float(M_PI / 510), with sin / cos in double (the 2011
 * build's ::sin(double); v = 255 -> (254, 0)) or float (std::sin(float); -> (255, 0)).
 * ColorCHLAC{,_RI}Estimation (color_chlac.hpp:148-153): r_ = 255 - r.  Bins and
 * normalisation constants are shared (color_chlac.h:38-53). */
#define C3H_COLOR_C3_FLOAT 0
#define C3H_COLOR_C3_DOUBLE 1  /* the default */
#define C3H_COLOR_CHLAC 2

/* SearchMode (color_voxel_recognition/include/color_voxel_recognition/search.h:48) */
enum { C3H_S_MODE_1 = 0, C3H_S_MODE_2, C3H_S_MODE_3, C3H_S_MODE_4, C3H_S_MODE_5, C3H_S_MODE_6 };

typedef struct c3h_ctx c3h_ctx;

/* pcl::VoxelGrid state after filter(): getNrDivisions / getMinBoxCoordinates /
 * getMaxBoxCoordinates, plus the sizes of limitPoint's output and of the
 * downsampled cloud. */
typedef struct {
  int32_t div_b[3];
  int32_t min_b[3];
  int32_t max_b[3];
  int64_t n_valid;
  int64_t n_occ;
  float leaf;
  float inv_leaf;
} c3h_grid_info;

/* extractC3HLACSignature981/117 arguments (c3_hlac/include/c3_hlac/c3_hlac_tools.h:75-86). */
typedef struct {
  int32_t variant;    /* 981 or 117 */
  int32_t thr[3];     /* setColorThreshold r,g,b (c3_hlac.h:92) */
  int32_t subdiv;     /* subdivision_size (0 = one vector for the whole grid) */
  int32_t offset[3];  /* offset_x/y/z */
  int32_t color_mode; /* C3H_COLOR_*: setColor's channels (C3H_COLOR_C3_DOUBLE by default) */
} c3h_extract_params;

/* one ranked detection: maxDot/maxX/maxY/maxZ/maxMode (search.h:99-126) */
typedef struct {
  double score;
  int32_t x, y, z, mode;
} c3h_det;

int c3h_version(void);
/* build provenance (no reference counterpart): "src=<sha256 of the library's sources,
 * concatenated in sorted path order> arch=<gfx> host=<build host> built=<UTC time>" */
const char* c3h_build_info(void);

/* context (one device, one stream) */
int c3h_create(int hip_device, c3h_ctx** out);
void c3h_destroy(c3h_ctx* ctx);
int c3h_set_stream(c3h_ctx* ctx, void* hip_stream); /* NULL = the context's own stream */
int c3h_synchronize(c3h_ctx* ctx);
const char* c3h_last_error(const c3h_ctx* ctx);

/* getVoxelGrid (c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:124-130) preceded by
 * limitPoint (color_voxel_recognition/test/detect_object.cpp:68-87): points with a
 * non-finite coordinate or z >= z_limit are dropped (pass INFINITY for no limit).
 * xyzrgb: n x 4 floats (x, y, z, rgb packed in the float bits as in PCL); at most
 * 16,777,215 points per call and cell coordinates within +-2^20 (C3H_ERR_RANGE).
 * The grid (indices, occupancy, colour means) is deterministic and exact.  Voxel
 * centroids are the fp32 sums of the voxel's points in input order divided by the count
 * (c3h_get_downsampled); where a centroid rounds across its cell boundary, the next
 * c3h_extract takes that voxel's subdivision and neighbour base from the centroid, as
 * c3_hlac.cpp:349-377 does.  With on_device = 1, c3h_get_downsampled reads the points
 * again: keep the buffer alive until then.  Any extent whose voxel count fits int32 is
 * accepted (PCL's check; more: C3H_ERR_RANGE): frames wider than the context's accumulator
 * budget (2^26 cells, 1.6 GB) are voxelised by a sorted pass with the same results.  An
 * internal inconsistency of the accumulators (device-side bound checks) fails with
 * C3H_ERR_HIP without touching memory outside the frame, and the next call starts clean. */
int c3h_voxelize(c3h_ctx* ctx, const float* xyzrgb, int64_t n, int on_device, float leaf,
                 float z_limit, c3h_grid_info* info);
/* sensor_msgs/PointCloud2 ingestion: pcl::fromROSMsg(*msg, cloud) into PointXYZRGB
 * (color_voxel_recognition/test/detect_object.cpp:142) followed by c3h_voxelize.  data =
 * the message's data[] (host, or device with on_device = 1), height x width points,
 * point_step / row_step / is_bigendian as in the message; offsets = the byte offsets of
 * the FLOAT32 fields x, y, z and rgb (rgb < 0: absent, read as 0), i.e. the `offset` of
 * the PointField named "x", "y", "z", "rgb" (or "rgba").  Every point is converted (NaN
 * ones too, limitPoint drops them) on the device.  c3h_get_downsampled stays valid until
 * the next ingestion. */
int c3h_voxelize_pointcloud2(c3h_ctx* ctx, const void* data, uint32_t height, uint32_t width,
                             uint32_t point_step, uint32_t row_step, const int32_t offsets[4],
                             int32_t is_bigendian, int on_device, float leaf, float z_limit,
                             c3h_grid_info* info);
/* the conversion alone, device to device on a HIP stream: d_out = height*width x 4 floats */
int c3h_pointcloud2_to_xyzrgb(const void* d_data, uint32_t height, uint32_t width, uint32_t point_step,
                              uint32_t row_step, const int32_t offsets[4], int32_t is_bigendian,
                              float* d_out, void* hip_stream);
/* VoxelGrid::getLeafLayout (setSaveLeafLayout(true)): div_b product int32, -1 = empty. */
int c3h_get_leaf_layout(c3h_ctx* ctx, int32_t* out, int on_device);
/* the downsampled cloud of getVoxelGrid: n_occ x 4 floats in ascending voxel index. */
int c3h_get_downsampled(c3h_ctx* ctx, float* out_xyzrgb, int on_device);
/* packed colour/occupancy grid, div_b product uint32: 0 = empty, else 1<<24 | rgb. */
int c3h_get_grid(c3h_ctx* ctx, uint32_t* out, int on_device);
/* use an externally produced packed grid (same encoding).  on_device=1 binds the
 * pointer without copying; the caller keeps it alive until the next set/voxelize. */
int c3h_set_grid(c3h_ctx* ctx, const uint32_t* words, const int32_t div_b[3],
                 const int32_t min_b[3], float leaf, int on_device);
int c3h_get_grid_info(c3h_ctx* ctx, c3h_grid_info* info);
/* device pointer of the packed grid in use (for zero-copy c3h_set_grid into another
 * context on the same device); valid until the next voxelize / set_grid. */
int c3h_grid_device_ptr(c3h_ctx* ctx, const uint32_t** out);

/* ---- automatic colour threshold (color_voxel_recognition/test/calc_scene_auto_threshold.cpp)
 * c3h_color_histogram replaces the per-voxel loop of calc_scene_auto_threshold.cpp:92-108
 * over the downsampled cloud (one voxel = one count; colours = the grid's centroid colours):
 * hist[c * 256 + v] (c = 0 r, 1 g, 2 b) counts the occupied voxels of the context's current
 * grid with channel c == v.  accumulate != 0 adds to hist (several frames, as the tool's
 * file loop does); 0 overwrites it.  hist is host memory, 768 int64.
 * c3h_auto_threshold is the tool's arithmetic (:111-146): total/cumulative averages and the
 * first j in 1..255 maximising the between-class variance, per channel; thr_out[3];
 * total_ave_out[3] (may be NULL) = the printed "totalAverage".  An empty histogram gives
 * C3H_ERR_ARG (the tool divides by zero). */
int c3h_color_histogram(c3h_ctx* ctx, int64_t* hist, int32_t accumulate);
int c3h_auto_threshold(const int64_t* hist, int32_t thr_out[3], double* total_ave_out);

/* ---- wire formats (host only, no device) ----
 * c3h_pcd_read_xyzrgb: a PCD point cloud as the reference's tools load it
 * (pcl::io::loadPCDFile, e.g. color_voxel_recognition/test/calc_scene_auto_threshold.cpp:89):
 * v0.7 header with FIELDS x y z rgb (any order, other fields skipped; 4-byte scalars),
 * DATA ascii or binary.  Binary data sits right after the header, or at the next 4096-byte
 * page for ROS-era PCL writers (the reference's demo clouds); the file size decides.
 * out: n x 4 floats (x, y, z, rgb bits) -- the c3h_voxelize input layout; out == NULL
 * returns the point count in *n, else *n is the capacity in points on entry.
 * c3h_feature_pcd_read: readFeature (c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:46-71):
 * COUNT = dim, POINTS = rows, "%f " scans; out == NULL returns the sizes, else *rows and
 * *dim are the capacity on entry.
 * c3h_feature_pcd_write: writeFeature (c3_hlac_tools.hpp:83-113): "%f " per value, one row
 * per line, all-zero rows dropped when remove_zero; fields = the FIELDS name (NULL =
 * "descriptor" as there; grsd_colorCHLAC_tools.hpp:32-58 writes "vfh").
 * Errors: C3H_ERR_NOTFOUND (open), C3H_ERR_FORMAT (malformed), C3H_ERR_ARG. */
int c3h_pcd_read_xyzrgb(const char* path, float* out, int64_t* n);
int c3h_feature_pcd_read(const char* path, float* out, int64_t* rows, int32_t* dim);
int c3h_feature_pcd_write(const char* path, const float* feat, int64_t rows, int32_t dim,
                          int32_t remove_zero, const char* fields);

/* C3HLAC{981,117}Estimation::setVoxelFilter + compute (c3_hlac/src/c3_hlac.cpp:204-416),
 * as called by extractC3HLACSignature981/117 (c3_hlac_tools.hpp:134-202).  Writes the
 * subdivision counts (getSubdivNum) and the number of feature vectors (hist_num; 0 for
 * the reference's silent-empty cases: offsets >= grid or a negative threshold). */
int c3h_extract(c3h_ctx* ctx, const c3h_extract_params* p, int32_t subdiv_out[3],
                int64_t* hist_num);
/* the features the context holds (the last extract, or after c3h_run_frames the last
 * frame's): getSubdivNum, hist_num and the dimension (981 / 117; 0 before any extract) */
int c3h_get_feature_info(c3h_ctx* ctx, int32_t subdiv_out[3], int64_t* hist_num, int32_t* dim);
/* ---- VOSCH / GRSD features (color_chlac/include/color_chlac/
 * grsd_colorCHLAC_tools.hpp), on the points and grid of the last c3h_voxelize (the points
 * it kept; a device input buffer must stay alive).
 * c3h_compute_normals: pcl::NormalEstimation with radius search (computeNormal, :63-87;
 * normals_radius_search = 0.02, grsd_colorCHLAC_tools.h:28): covariance of the points
 * within `radius` (float distances, the point included), smallest-eigenvalue eigenvector
 * (double), flipped towards `viewpoint` (NULL = origin), curvature; < 3 neighbours -> NaN.
 * c3h_get_normals: n x 4 floats (nx, ny, nz, curvature) in input order.
 * c3h_extract_grsd: extractGRSDSignature21 (:131-296): per occupied voxel PCL's
 * PrincipalRadiiRSD (computeRSD: nr_subdiv 5, plane radius 0.2) over the points within
 * max(rsd_radius, leaf sqrt(3)/2) of its centroid, get_type (:99-118), and the 6 x 6 type
 * transitions with its 26 neighbour voxels per subdivision (setVoxelFilter's subdivision
 * rules); features = the first 20 upper-triangle bins (x 20/26 with normalize), exist by
 * the setGRSD rule.  c3h_get_rsd: r_min / r_max and the type per occupied voxel (leaf
 * layout order); returns their count.
 * c3h_extract_vosch: extractVOSCH (:832-843): [GRSD-20 | C3-HLAC-117] = 137 floats per
 * subdivision (the C3 part as c3h_extract with variant 117, thr, color_mode), exist by
 * the setVOSCH rule; the next c3h_search uses them (search_setup with F = 137).
 * The PCL algorithms are restated (PCL is not part of the reference tree); radius-search
 * ties are broken by point index. */
typedef struct {
  int32_t subdiv;     /* subdivision_size (0 = one histogram) */
  int32_t offset[3];
  float rsd_radius;   /* rsd_radius_search (0.01 in the reference) */
  int32_t normalize;  /* is_normalize (default false) */
} c3h_grsd_params;
int c3h_compute_normals(c3h_ctx* ctx, float radius, const float viewpoint[3]);
int c3h_get_normals(c3h_ctx* ctx, float* out, int on_device);
int c3h_extract_grsd(c3h_ctx* ctx, const c3h_grsd_params* p, int32_t subdiv_out[3], int64_t* hist_num);
int c3h_get_rsd(c3h_ctx* ctx, float* radii, int32_t* types, int on_device);
int c3h_extract_vosch(c3h_ctx* ctx, const c3h_grsd_params* p, const int32_t thr[3], int32_t color_mode,
                      int32_t subdiv_out[3], int64_t* hist_num);
/* SearchObj::setData(subdiv_b, feature) (search.cpp:539-658) with features computed
 * elsewhere (VOSCH / ConVOSCH / GRSD extractors, search_new.h:34-76, or stored C3-HLAC
 * rows): subdiv_b[0]*[1]*[2] rows of dim floats, row h = x + y*xn + z*xn*yn.  exist =
 * the rows' exist_voxel_num, or NULL to derive it by exist_rule with the reference's
 * arithmetic: C3H_EXIST_C3HLAC (int)((f0+f1)*2+0.001) (setC3HLAC), C3H_EXIST_VOSCH
 * (int)((f20+f21)*2+0.001) (setVOSCH / setConVOSCH), C3H_EXIST_GRSD an int summing
 * f0..f19, then / 26 (setGRSD).  The next c3h_search / c3h_search_async uses them
 * (dim must equal the F of c3h_search_setup). */
#define C3H_EXIST_C3HLAC 0
#define C3H_EXIST_VOSCH 1
#define C3H_EXIST_GRSD 2
int c3h_set_features(c3h_ctx* ctx, const float* feat, const int32_t subdiv_b[3], int32_t dim,
                     const int32_t* exist, int32_t exist_rule, int on_device);
/* hist_num x variant floats of the last extract.  After an extract at fp16 search precision
 * on a large dense 981 grid (c3h_set_search_precision below) the rows are the f16 ones the
 * C3 kernel wrote, widened: each value is the exact integer-derived feature rounded to f16. */
int c3h_get_features(c3h_ctx* ctx, float* out, int on_device);
/* exist_voxel_num of SearchC3HLAC::setC3HLAC
 * (color_voxel_recognition/include/color_voxel_recognition/search_c3_hlac.h:60-61) */
int c3h_get_exist(c3h_ctx* ctx, int32_t* out, int on_device);

/* SearchObj configuration.
 *   axis_p: D x F row-major projection (setSceneAxis, search.cpp:694-712); when var is
 *           non-NULL row i is whitened by 1/sqrt(var[i]) exactly as setSceneAxis does.
 *           NULL disables compression (compress_flg=false; then D must equal F).
 *   axis_q: M x r x D model subspaces as readAxis leaves them (search.cpp:153-165,
 *           819-837: transposed, MULTIPLE_SIMILARITY scaling already applied).
 *   feature_max: setNormalizeVal values (search.cpp:742-748), NULL/0 = none.
 * Any D >= 1: a D <= 160 that is not a multiple of 4 is run on zero axes appended up to the
 * next multiple (their compressed values are 0, so the scores are the caller's D's bit for
 * bit), which keeps such searches on the sparse list path and the pipeline;
 * c3h_get_compressed returns the caller's D columns. */
int c3h_search_setup(c3h_ctx* ctx, const float* axis_p, const float* var, int32_t D,
                     int32_t F, const float* axis_q, int32_t M, int32_t r,
                     const float* feature_max, int32_t feature_max_len);
/* Search precision of the matrix-core stages.  fp16 = 1: the compress of grids of >= 65,536
 * subdivisions (e.g. BASELINE config 5; D <= 128) rounds the normalised features and the
 * whitened axis to f16, and the matrix-core projection (c3h_set_score_engine) rounds each
 * position's box row -- scaled by a power of two, |Q f|/|f| is scale-free -- and the model
 * basis to f16; both accumulate in f32 on v_mfma_f32_32x32x16_f16.  Scores then agree with
 * the float64 oracle within 2e-3 relative (fp16 = 0, the default: fp32, 1e-5).  The VALU
 * kernels and the pipelined c3h_run_frames path always run in fp32.
 * The setting also applies to c3h_extract: at fp16 a large dense C3-HLAC-981 extract (the
 * matrix-core C3 kernel) writes its feature rows as f16 only.  Setting fp16 = 0 afterwards
 * searches those rounded rows (widened to f32) until the next extract, so the 1e-5 bound of
 * fp32 precision holds only for features extracted at fp16 = 0: re-extract after switching. */
int c3h_set_search_precision(c3h_ctx* ctx, int32_t fp16);
/* Engine of the single-frame search's projection step (SearchObjMulti::searchPart's
 * M x r x D products, search.cpp:915-968): 0 = automatic (default: the matrix cores for
 * grids of >= 65,536 subdivisions and for models with r > 64, the VALU list kernel
 * otherwise), 1 = VALU (score_list_kernel for r <= 64; the generic kernel beyond),
 * 2 = matrix cores (score_mfma_kernel, v_mfma_f32_32x32x2_f32; D <= 160).
 * Both engines form every product as the same k-ordered fp32 fma chain, so the scores are
 * bit-identical.  Batched / pipelined searches (c3h_run_frames) always use the VALU kernel. */
int c3h_set_score_engine(c3h_ctx* ctx, int32_t engine);
/* SearchObj::setRank / SearchObjMulti::setRank (search.cpp:130-143, 778-815):
 * (re)allocates the per-model lists; modes start at S_MODE_1. */
int c3h_set_rank(c3h_ctx* ctx, int32_t rank);
/* cleanMax / cleanData list reset (search.cpp:683-690, 716-732): scores and x,y,z to 0,
 * modes kept (the reference never resets them). */
int c3h_clean_max(c3h_ctx* ctx);
/* setData + search() (rotate=1) or searchWithoutRotation() (rotate=0)
 * (search.cpp:384-480, 539-658, 915-968) on the features of the last extract; the
 * lists continue from their current state.  Writes M x rank detections to `out` (host)
 * and, when remove_overlap != 0, applies SearchObjMulti::removeOverlap
 * (search.cpp:972-992) first.  Returns the number of scheduled modes (>0) or an error. */
int c3h_search(c3h_ctx* ctx, const int32_t range[3], int32_t exist_threshold,
               int32_t rotate, int32_t remove_overlap, c3h_det* out);
/* Asynchronous variant for device-resident pipelines: no host sync; copies the M x rank
 * lists into the device buffer d_out after the search (no removeOverlap). */
int c3h_search_async(c3h_ctx* ctx, const int32_t range[3], int32_t exist_threshold,
                     int32_t rotate, c3h_det* d_out);
/* Batch driver for device-resident frames (configs 3-5): every frame i is bound from
 * d_grids[i] (same dims/min_b/leaf), extracted with *p and searched (async) into
 * d_out + i * M * rank, each frame starting from fresh lists (setRank state: scores 0,
 * S_MODE_1).  Frames go c3h_set_batch at a time through one set of launches and are
 * spread over c3h_set_lanes lanes; afterwards the context holds the last frame's state.
 * One host call, no host synchronisation. */
int c3h_run_frames(c3h_ctx* ctx, const uint32_t* const* d_grids, int32_t nframes,
                   const int32_t div_b[3], const int32_t min_b[3], float leaf,
                   const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                   int32_t rotate, c3h_det* d_out);
/* Frames in flight in c3h_run_frames (default 4): frame lanes are child contexts with
 * their own streams, so the latency-bound search of one frame overlaps the HBM stream of
 * the next.  Lane 0 (this context) takes the last frame.  1 = strictly sequential. */
int c3h_set_lanes(c3h_ctx* ctx, int32_t lanes);
/* Streaming form of c3h_run_frames for a continuous frame source (the ROS callback loop
 * of color_voxel_recognition/test/detect_object.cpp:139-215, one frame after another):
 * same arguments and per-frame results, but the software pipeline stays filled between
 * calls.  Each call enqueues its frames as ceil(nframes / batch) batches, one pipeline
 * tick each, and returns without draining: a batch's detections are complete in d_out
 * once three more batches have been pushed, or after c3h_stream_flush.  The grids and
 * d_out must stay valid until then.  A call with a different geometry / parameter set,
 * and every other entry point that touches this context's buffers, drains the open
 * stream first.  Configurations the pipeline does not cover (rank > 1, ...) complete
 * synchronously as in c3h_run_frames.  Returns the number of searched modes. */
int c3h_stream_frames(c3h_ctx* ctx, const uint32_t* const* d_grids, int32_t nframes,
                      const int32_t div_b[3], const int32_t min_b[3], float leaf,
                      const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                      int32_t rotate, c3h_det* d_out);
/* Runs the remaining ticks of an open stream (no host synchronisation). */
int c3h_stream_flush(c3h_ctx* ctx);

/* Points-in batch driver (BASELINE configs[3]: independent RGB-D frames): the per-callback
 * work of color_voxel_recognition/test/detect_object.cpp:139-186 -- limitPoint + getVoxelGrid
 * (c3h_voxelize), extractC3HLACSignature981/117 (c3h_extract) and SearchObj(Multi)::search
 * from fresh lists (setRank state) -- for nframes point clouds, frame i = pts[i] (n[i] x 4
 * floats as c3h_voxelize takes them; device pointers with on_device = 1, else host memory,
 * copied by the library: pin it for full PCIe rate).  Frames are voxelised on the device in
 * batches (c3h_set_batch) with no per-frame host round trip, each into a canvas grid of
 * canvas[0] x canvas[1] x canvas[2] voxels placed at the frame's own min_b, and go through
 * the software-pipelined tick of c3h_run_frames; a box position passes only inside the
 * frame's own subdivisions, so every frame's results are those of its own grid.  Frame i's
 * M x rank detections land in d_out + i * M * rank (device).  Voxels whose centroid may
 * round across a cell face are summed exactly in the batch (their points in input order),
 * and those whose centroid cell is another cell take it as subdivision and neighbour base
 * (c3_hlac.cpp:349-377): their subdivisions are recomputed after the batch's C3 stage
 * (n_moved in info).  Frames the canvas path cannot reproduce -- extent beyond the canvas,
 * more than 4,096 such voxels (65,536 of their points) or 256 moved ones, a centroid cell
 * past the last subdivision, one subdivision where the canvas has several (computeC3HLAC's
 * hist_num == 1 rule), no valid point -- are recomputed on the single-frame path after the
 * batches (status 1).  info (host, nframes records, may be
 * NULL): the frame's VoxelGrid geometry, getSubdivNum, point and voxel counts and status
 * (0 batched, 1 single-frame path, < 0 the C3H_ERR_* that frame failed with; its lists are
 * the fresh setRank state).  One host synchronisation per call (the frames' records).
 * Rank 1 on the fast search path (else every frame takes the single-frame path).
 * Returns the number of searched modes or an error. */
typedef struct {
  int32_t div_b[3], min_b[3], subdiv_b[3];
  int32_t status;
  int32_t n_moved;  /* voxels whose centroid lies in another cell, corrected in the batch */
  int32_t pad;
  int64_t n_valid, n_occ;
} c3h_frame_info;
int c3h_run_point_frames(c3h_ctx* ctx, const float* const* pts, const int64_t* n, int32_t nframes,
                         int on_device, float leaf, float z_limit, const int32_t canvas[3],
                         const c3h_extract_params* p, const int32_t range[3], int32_t exist_threshold,
                         int32_t rotate, c3h_det* d_out, c3h_frame_info* info);
/* Frames per pipeline batch / launch in c3h_run_frames and c3h_stream_frames
 * (1..64, default 32; the fast search path only). */
int c3h_set_batch(c3h_ctx* ctx, int32_t frames);
/* c3h_run_frames scheduling (default 1): 1 = software pipeline on the context stream, one
 * fused launch per tick running occupancy (batch t) | tile (t-1) | compress+gate (t-2) |
 * score + rank-1 argmax (t-3); applies to rank 1 on the fast search path without split
 * subdivisions, other configurations use the lanes.  0 = lanes only. */
int c3h_set_pipeline(c3h_ctx* ctx, int32_t enable);
/* compressed features (setData before the summed-volume table): hist_num x D floats */
int c3h_get_compressed(c3h_ctx* ctx, float* out, int on_device);
/* per-position similarity of the last search, modes x M x P doubles (-1 = gated out).
 * n_out receives the element count; pass out=NULL to query it. */
int c3h_get_scores(c3h_ctx* ctx, double* out, int64_t* n_out, int on_device);
/* SearchObjMulti::removeOverlap on host lists (pure host function, no context). */
int c3h_remove_overlap(int32_t M, int32_t rank, const int32_t range[3], c3h_det* lists);
/* SearchObj(Multi)::searchPart's sequential rank update (search.cpp:464-474 with checkOverlap
 * :327-356) replayed on host score arrays in c3h_get_scores' layout: per mode of search()'s
 * schedule for range / rotate (modes without a position skipped), M x P doubles in (z, y, x)
 * scan order over subdiv_b, -1 = gated out.  lists (M x rank, host) continue from their
 * state, as search() does.  Pure host function: merges the score arrays of the z-slabs of
 * one scene (c3hlac/dist.py) into the whole scene's ranked lists.  Returns the number of
 * searched modes. */
int c3h_replay_scores(int32_t M, int32_t rank, const int32_t range[3], int32_t rotate, const int32_t subdiv_b[3],
                      const double* scores, c3h_det* lists);
/* c3h_replay_scores that also records every row's entry floor: row_floor[(m * ze + z) * ye
 * + y] (per searched mode, in the scores' mode order) = model m's rank-th score before the
 * row's first position.  A position at or below it cannot change the lists (searchPart
 * updates only above lists[rank-1], which never decreases), so the z-slab merge
 * (c3hlac/dist.py) can leave such positions out and verify that it did so safely. */
int c3h_replay_scores_floor(int32_t M, int32_t rank, const int32_t range[3], int32_t rotate,
                            const int32_t subdiv_b[3], const double* scores, c3h_det* lists, double* row_floor);

/* PCA::read (color_voxel_recognition/src/pca.cpp:119-185): axis column-major dim x dim
 * (eigenvector i contiguous), variances, optional mean.  Returns dim or an error.
 * axis = var = NULL queries the dimension (header only; max_dim ignored). */
int c3h_pca_read(const char* path, int32_t ascii, float* axis, float* var, float* mean,
                 int32_t* has_mean, int32_t max_dim);
/* PCA::write (pca.cpp:190-240): the same layout c3h_pca_read reads; mean may be NULL
 * (mean_flg false).  Host arrays. */
int c3h_pca_write(const char* path, int32_t ascii, int32_t dim, const float* axis, const float* var,
                  const float* mean);

/* ---- PCA training on the GPU --------------------------------------
 * class PCA (color_voxel_recognition/include/color_voxel_recognition/pca.h:45-81) as
 * used by pca_scene.cpp (scene compress axis) and pca_models.cpp (model subspaces: every
 * feature compressed by the scene axis, plus its 23 rotateFeature90 images).  The
 * correlation accumulates in f64 on the device; solve runs rocSOLVER dsyevd (loaded at
 * the first solve) and sortVecAndVal's stable descending order.  Differences from the
 * reference: sums are f64 (the reference accumulates in f32), and solve leaves the
 * accumulated sums untouched (it can be called again after more addData). */
typedef struct c3h_pca c3h_pca;
/* PCA::PCA(bool _mean_flg = true) (pca.cpp:40-44) on a HIP device */
int c3h_pca_create(int hip_device, int32_t mean_flg, c3h_pca** out);
void c3h_pca_destroy(c3h_pca* pca);
const char* c3h_pca_last_error(c3h_pca* pca);
int c3h_pca_set_stream(c3h_pca* pca, void* hip_stream); /* NULL = the object's own stream */
/* compressFeature (pca_models.cpp:48-63) applied to every added vector: axis = the first
 * D eigenvectors of the scene PCA, F x D column-major (PCA::getAxis().block(0,0,F,D));
 * var = its variances (WHITENING, FILE_MODE) or NULL.  Host arrays; before any addData. */
int c3h_pca_set_compress(c3h_pca* pca, const float* axis, const float* var, int32_t F, int32_t D);
/* PCA::addData (pca.cpp:48-69) for n rows of F floats (row stride ld).  rotate24 = 1
 * adds, per row, the 24 vectors of pca_models.cpp:109-171 (the row and its 23
 * rotateFeature90 compositions; F = 981, 495 or 486).  A differing F is an error
 * (pca.cpp:54-57).  Rows on the device (on_device = 1) or the host. */
int c3h_pca_add_data(c3h_pca* pca, const float* rows, int64_t n, int64_t ld, int32_t F, int32_t rotate24,
                     int on_device);
/* PCA::solve(regularization_flg, regularization_nolm) (pca.cpp:73-105) + sortVecAndVal */
int c3h_pca_solve(c3h_pca* pca, int32_t regularization_flg, float regularization_nolm);
/* getAxis / getVariance / getMean after solve: axis dim x dim column-major (eigenvector i
 * contiguous, by descending variance), var dim, mean dim (error without mean_flg, as
 * pca.cpp:110-113); any pointer may be NULL.  Returns dim (D if compressing, else F). */
int c3h_pca_get(c3h_pca* pca, float* axis, float* var, float* mean, int64_t* nsample, int on_device);
/* the normalised correlation matrix solve decomposed (dim x dim doubles, host) */
int c3h_pca_get_correlation(c3h_pca* pca, double* corr);
/* pcl::rotateFeature90 (c3_hlac/src/c3_hlac.cpp:49-172) on n device rows (stride ld) on a
 * HIP stream; dim 981 / 495 / 486, mode 0..3 = R_MODE_1..4; in != out. */
int c3h_rotate_feature90(const float* in, float* out, int64_t n, int64_t ld, int32_t dim, int32_t mode,
                         void* hip_stream);
/* the same rotation as a gather map: map_out[o] = input index of output o (host). */
int c3h_rotate_map(int32_t dim, int32_t mode, int32_t* map_out);

/* Multi-GPU: one process per GPU, frames sharded across them with no
 * data-path collective; the one exchange is this gather of every rank's detection records
 * (rank-major into d_all = world x n_local records) with RCCL ncclAllGather on the
 * context's stream, after the context's queued work (an open c3h_stream_frames stream is
 * flushed first).  nccl_comm = the caller's ncclComm_t (ncclCommInitRank); asynchronous:
 * d_all is complete after c3h_synchronize.  librccl is loaded at the first call. */
int c3h_allgather_detections(c3h_ctx* ctx, void* nccl_comm, const c3h_det* d_local, int64_t n_local,
                             c3h_det* d_all);

/* per-kernel device time (ms) accumulated since the last reset with HIP events on the
 * context stream; slots: 0 voxelize, 1 C3-HLAC, 2 compress, 3 score, 4 rank replay,
 * 5 pipeline tick (c3h_run_frames' fused launches: every stage of four batches).
 * counts_out receives the number of frames the timed launches processed per slot (a
 * batched launch of B frames counts B).  Enabling adds event records.
 * enable: 0 = off, 1 = every slot, otherwise a mask of C3H_TIMING_* bits (the slots
 * bracketed by events; fewer events = less perturbation of back-to-back launches). */
#define C3H_NTIMERS 6
#define C3H_TIMING_VOXELIZE 0x2
#define C3H_TIMING_C3HLAC 0x4
#define C3H_TIMING_COMPRESS 0x8
#define C3H_TIMING_SCORE 0x10
#define C3H_TIMING_REPLAY 0x20
#define C3H_TIMING_PIPELINE 0x40
#define C3H_TIMING_ALL 0x7e
int c3h_timing(c3h_ctx* ctx, int32_t enable);
int c3h_kernel_times(c3h_ctx* ctx, float* ms_out, int32_t* counts_out, int32_t reset);

#ifdef __cplusplus
}
#endif
#endif
