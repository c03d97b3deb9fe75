/*
 * c3hlac_oracle.h -- CPU restatement of the reference's colour-voxel C3-HLAC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker / the timed CPU baseline.  The product path is the HIP
 * library in mapping-private_amd/ and fails loudly when that is missing.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - C3-HLAC arithmetic: the reference's kernel ships binary-only
 *     (c3_hlac_core/Makefile:1-11 downloads libc3_hlac_core.so); this restates its
 *     open twin color_chlac/include/color_chlac/color_chlac.hpp (C3HLACEstimation /
 *     C3HLAC_RI_Estimation).  The 981/117 bin map is pinned against a table
 *     extracted mechanically from color_chlac.hpp (tests/golden/binmap_*.json).
 *   - PCL VoxelGrid (external, unpinned version) restated per SURVEY.md App. B.
 *   - PCA reader pinned against the reference's own binary PCA fixtures.
 *   The reference itself cannot be compiled here (rosbuild + PCL + Eigen + a
 *   downloaded .so), so no oracle/_ref build exists.
 */
#ifndef C3HLAC_ORACLE_H_
#define C3HLAC_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t div_b[3];
  int32_t min_b[3];
  int32_t max_b[3];
  int64_t n_valid;   /* points kept by limitPoint + finite filter */
  int64_t n_occ;     /* occupied voxels (= downsampled cloud size) */
  float leaf;
  float inv_leaf;
} orc_grid;

/* Colour channels of setColor.  ORC_COLOR_C3_DOUBLE / _FLOAT: C3HLAC (color_chlac.hpp:
 * 155-179): lut[2v] = 255*sin(v*theta), lut[2v+1] = 255*cos(v*theta), theta =
 * float(M_PI/510), sin/cos in double (v=255 -> (254,0)) or float (v=255 -> (255,0)).
 * ORC_COLOR_CHLAC: ColorCHLAC{,_RI}Estimation (color_chlac.hpp:148-153): (v, 255 - v). */
#define ORC_COLOR_C3_FLOAT 0
#define ORC_COLOR_C3_DOUBLE 1
#define ORC_COLOR_CHLAC 2
void orc_lut(int color_mode, int32_t* lut /* 512 */);
/* 1 (default): the voxel-grid arithmetic of the reference's PCL 1.0 / Eigen 3.0 (centroid
 * = sum * (1/n), neighbour base floor(c / leaf)); 0: later PCL (see c3hlac_oracle.c). */
void orc_set_voxel_semantics(int pcl_era);

/* Bounds pass of PCL VoxelGrid::applyFilter (+ detect_object.cpp:68-87 limitPoint). */
int orc_voxel_bounds(const float* pts /* n*4: x,y,z,rgb-bits */, int64_t n, float leaf,
                     float z_limit, orc_grid* g);
/* Fill pass: leaf_layout (div product ints, -1 = empty), downsampled cloud (n_occ*4,
 * ascending linear index, xyz = fp32 sum in input order times 1/n, rgb = per-channel
 * fp32 sums times 1/n, truncated). */
int orc_voxel_fill(const float* pts, int64_t n, float z_limit, orc_grid* g,
                   int32_t* leaf_layout, float* cloud_out);

/* extractC3HLACSignature981/117 (c3_hlac_tools.hpp:134-202 -> c3_hlac.cpp:204-416).
 * exact=0: fp32 accumulation in the reference's order; exact=1: int64 accumulation,
 * converted to float once (what the GPU does).  Returns hist_num (>=0) or <0 on error;
 * feat_out must hold hist_num*variant floats (query with feat_out=NULL first). */
int64_t orc_c3hlac(const orc_grid* g, const int32_t* leaf_layout, const float* cloud,
                   int variant, int thr_r, int thr_g, int thr_b, float voxel_size,
                   int subdiv, int ox, int oy, int oz, int color_mode, int exact,
                   float* feat_out, int32_t subdiv_out[3]);

/* exist_voxel_num of SearchC3HLAC::setC3HLAC (search_c3_hlac.h:60-61). */
void orc_exist(const float* feat, int64_t hist_num, int F, int32_t* exist_out);

/* Sliding-box search: SearchObj / SearchObjMulti setData + search/searchWithoutRotation
 * (search.cpp:384-658, 915-968).  dbl=0: fp32 in the reference's order (summed-volume
 * table); dbl=1: float64 everywhere.  axis_p: D x F row-major (already whitened) or NULL
 * (no compression, D=F).  axis_q: M x r x D.  fmax: optional setNormalizeVal values.
 * State arrays (M*rank each) are in/out: callers pass the persistent list (cleanData
 * zeroes x,y,z,score but not mode: search.cpp:716-732). */
int orc_search(int xn, int yn, int zn, const float* feat, int F, const int32_t* exist,
               const float* axis_p, int D, const float* fmax, int fmax_len,
               const float* axis_q, int M, int r, int range1, int range2, int range3,
               int rank, int thr, int rotate, int dbl,
               double* st_score, int32_t* st_x, int32_t* st_y, int32_t* st_z,
               int32_t* st_mode, double* scores_out /* optional modes*M*P */);

/* SearchObjMulti::removeOverlap (search.cpp:972-992) on the per-model lists. */
void orc_remove_overlap(int M, int rank, int range1, int range2, int range3,
                        double* st_score, int32_t* st_x, int32_t* st_y, int32_t* st_z,
                        int32_t* st_mode);

/* PCA::read (pca.cpp:119-185).  Returns dim (>0) or <0.  axis is column-major
 * dim*dim (eigenvector i contiguous), i.e. axis[i*dim + j] = axis(j, i). */
int orc_pca_read(const char* path, int ascii, float* axis, float* var, float* mean,
                 int* has_mean, int max_dim);

#ifdef __cplusplus
}
#endif
#endif
