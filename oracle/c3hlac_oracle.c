/*
 * c3hlac_oracle.c -- CPU restatement of the C3-HLAC colour-voxel recognition path.
 *
 * TEST INFRASTRUCTURE ONLY (see c3hlac_oracle.h).  Single-threaded, -O2,
 * -ffp-contract=off, written to follow the reference's loop and accumulation order
 * so its fp32 results are the reference's up to the documented unpinned parts
 * (Eigen's GEMV/dot reduction order; the PCL version's colour averaging).
 *
 * Reference files followed (paths relative to the reference root):
 *   voxel grid      c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:124-130 (PCL VoxelGrid,
 *                   semantics in SURVEY.md App. B), color_voxel_recognition/test/
 *                   detect_object.cpp:68-87 (limitPoint)
 *   C3-HLAC         c3_hlac/src/c3_hlac.cpp:177-416 (driver, constants :38-45),
 *                   color_chlac/include/color_chlac/color_chlac.hpp:168-179 (setColor),
 *                   :213-1469 (981 bins), :1565-1743 (117 bins)
 *   exist gate      color_voxel_recognition/include/color_voxel_recognition/
 *                   search_c3_hlac.h:60-61
 *   search          color_voxel_recognition/src/search.cpp:122-149 (setters),
 *                   :218-317 (ranges), :327-376 (checkOverlap/maxCpy/maxAssign),
 *                   :384-480 (search/searchPart), :484-535 (clipValue),
 *                   :539-658 (setData), :915-968 (multi searchPart),
 *                   :972-992 (removeOverlap)
 *   PCA reader      color_voxel_recognition/src/pca.cpp:119-185
 */
#include "c3hlac_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* c3_hlac.cpp:38-45 (float constants) */
static const float NORMALIZE_0 = 1 / 255.0;
static const float NORMALIZE_1 = 1 / 65025.0;
static const float NORMALIZE_0_BIN = 1;
static const float NORMALIZE_1_BIN = 1;
static const float NORMALIZE_117_0 = 1 / 255.0;
static const float NORMALIZE_117_1 = 1 / 845325.0;
static const float NORMALIZE_117_0_BIN = 1;
static const float NORMALIZE_117_1_BIN = 1 / 13.0;

/* relative_coordinates, c3_hlac.cpp:180-201 */
static const int REL[13][3] = {
    {-1, -1, -1}, {-1, 0, -1}, {-1, 1, -1}, {0, -1, -1}, {0, 0, -1}, {0, 1, -1},
    {1, -1, -1},  {1, 0, -1},  {1, 1, -1},  {-1, -1, 0}, {0, -1, 0}, {1, -1, 0},
    {-1, 0, 0}};

/* bin-count pairs of the 981/117 "bin" block (color_chlac.hpp:261-292, 1625-1645):
 * r.g r.g_ r.b r.b_ r_.g r_.g_ r_.b r_.b_ g.b g.b_ g_.b g_.b_ (channel order r,r_,g,g_,b,b_) */
static const int PAIRS[12][2] = {{0, 2}, {0, 3}, {0, 4}, {0, 5}, {1, 2}, {1, 3},
                                 {1, 4}, {1, 5}, {2, 4}, {2, 5}, {3, 4}, {3, 5}};

/* first-order 981 bin of (neighbour k, centre channel c, neighbour channel n):
 * the closed form of color_chlac.hpp:295-800 (pinned by tests/golden/binmap_981.json) */
static int bin981(int k, int c, int n) {
  return k <= 8 ? 6 + 78 * c + 9 * n + k : 60 + 78 * c + 4 * n + (k - 9);
}
/* upper-triangle index of the centre auto-products (color_chlac.hpp:222-242) */
static int tri6(int c, int n) { return 6 * c - c * (c - 1) / 2 + (n - c); }

void orc_lut(int color_mode, int32_t* lut) {
  const float angle_norm = M_PI / 510; /* color_chlac.h:9 */
  for (int v = 0; v < 256; ++v) {
    const float a = v * angle_norm;
    if (color_mode == ORC_COLOR_CHLAC) {
      /* ColorCHLAC{,_RI}Estimation::setColor (color_chlac.hpp:148-153): r_ = 255 - r */
      lut[2 * v] = v;
      lut[2 * v + 1] = 255 - v;
    } else if (color_mode == ORC_COLOR_C3_DOUBLE) {
      lut[2 * v] = (int)(255 * sin((double)a));
      lut[2 * v + 1] = (int)(255 * cos((double)a));
    } else {
      lut[2 * v] = (int)(255 * sinf(a));
      lut[2 * v + 1] = (int)(255 * cosf(a));
    }
  }
}

/* ------------------------------------------------------------------ voxel grid */

/* Voxel-grid arithmetic of the PCL / Eigen the reference was built against (pinned by
 * the reference's own color_chlac/demos/shape_data/<name>_GRSD_CCHLAC.pcd vectors, see
 * tests/test_shape_fixtures.py):
 *   1 (default) PCL 1.0-era VoxelGrid on Eigen 3.0: the centroid (xyz and the r, g, b
 *     channel sums) is `centroid / nr_points`, which Eigen 3.0's scalar_quotient1_op
 *     evaluates as centroid * (1 / n) in float; getNeighborCentroidIndices takes its base
 *     cell as floor(p / leaf_size) (float division).
 *   0 later PCL / Eigen (true division; base floor(p * inverse_leaf_size)): only kept to
 *     show, in the fixture test, which files it fails. */
static int g_pcl_era = 1;
void orc_set_voxel_semantics(int pcl_era) { g_pcl_era = pcl_era ? 1 : 0; }

static int pt_valid(const float* p, float z_limit) {
  return isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]) && p[2] < z_limit;
}

int orc_voxel_bounds(const float* pts, int64_t n, float leaf, float z_limit, orc_grid* g) {
  memset(g, 0, sizeof(*g));
  if (!(leaf > 0)) return -1;
  g->leaf = leaf;
  g->inv_leaf = 1.0f / leaf;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  int64_t nv = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + 4 * i;
    if (!pt_valid(p, z_limit)) continue;
    ++nv;
    for (int a = 0; a < 3; ++a) {
      if (p[a] < mn[a]) mn[a] = p[a];
      if (p[a] > mx[a]) mx[a] = p[a];
    }
  }
  g->n_valid = nv;
  if (nv == 0) return 0;
  int64_t prod = 1;
  for (int a = 0; a < 3; ++a) {
    g->min_b[a] = (int)floorf(mn[a] * g->inv_leaf);
    g->max_b[a] = (int)floorf(mx[a] * g->inv_leaf);
    g->div_b[a] = g->max_b[a] - g->min_b[a] + 1;
    prod *= g->div_b[a];
  }
  if (prod > 2147483647LL) return -2;
  return 0;
}

typedef struct {
  int64_t idx;
  int64_t i;
} key_t_;

static int cmp_key(const void* a, const void* b) {
  const key_t_* x = (const key_t_*)a;
  const key_t_* y = (const key_t_*)b;
  if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
  return x->i < y->i ? -1 : (x->i > y->i);
}

int orc_voxel_fill(const float* pts, int64_t n, float z_limit, orc_grid* g,
                   int32_t* leaf_layout, float* cloud_out) {
  const int64_t nvox = (int64_t)g->div_b[0] * g->div_b[1] * g->div_b[2];
  for (int64_t v = 0; v < nvox; ++v) leaf_layout[v] = -1;
  g->n_occ = 0;
  if (g->n_valid == 0) return 0;
  key_t_* keys = (key_t_*)malloc(sizeof(key_t_) * (size_t)g->n_valid);
  if (!keys) return -3;
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) {
    const float* p = pts + 4 * i;
    if (!pt_valid(p, z_limit)) continue;
    int ijk[3];
    for (int a = 0; a < 3; ++a)
      ijk[a] = (int)(floorf(p[a] * g->inv_leaf) - (float)g->min_b[a]);
    keys[m].idx = ijk[0] + (int64_t)ijk[1] * g->div_b[0] +
                  (int64_t)ijk[2] * g->div_b[0] * g->div_b[1];
    keys[m].i = i;
    ++m;
  }
  qsort(keys, (size_t)m, sizeof(key_t_), cmp_key);
  int64_t out = 0;
  for (int64_t s = 0; s < m;) {
    int64_t e = s;
    float c[3] = {0, 0, 0}, col[3] = {0, 0, 0};
    while (e < m && keys[e].idx == keys[s].idx) {
      const float* p = pts + 4 * keys[e].i;
      c[0] += p[0];
      c[1] += p[1];
      c[2] += p[2];
      uint32_t rgb;
      memcpy(&rgb, &p[3], 4);
      col[0] += (float)((rgb >> 16) & 0xff);
      col[1] += (float)((rgb >> 8) & 0xff);
      col[2] += (float)(rgb & 0xff);
      ++e;
    }
    const float cnt = (float)(e - s);
    float m[6];
    if (g_pcl_era) { /* Eigen 3.0: v / n == v * (1 / n) in float */
      const float rn = 1.0f / cnt;
      for (int a = 0; a < 3; ++a) {
        m[a] = c[a] * rn;
        m[3 + a] = col[a] * rn;
      }
    } else {
      for (int a = 0; a < 3; ++a) {
        m[a] = c[a] / cnt;
        m[3 + a] = col[a] / cnt;
      }
    }
    float* o = cloud_out + 4 * out;
    o[0] = m[0];
    o[1] = m[1];
    o[2] = m[2];
    /* colour rule: float mean per channel, truncated, repacked */
    const uint32_t rgb = ((uint32_t)(int)m[3] << 16) | ((uint32_t)(int)m[4] << 8) | (uint32_t)(int)m[5];
    memcpy(&o[3], &rgb, 4);
    leaf_layout[keys[s].idx] = (int32_t)out;
    ++out;
    s = e;
  }
  free(keys);
  g->n_occ = out;
  return 0;
}

/* ------------------------------------------------------------------ C3-HLAC */

typedef struct {
  float* f;
  int64_t* x;
} hist_t;

static inline void hadd(hist_t* h, int exact, int64_t base, int idx, int val) {
  if (exact)
    h->x[base + idx] += val;
  else
    h->f[base + idx] += val; /* float += int, as in the reference */
}

int64_t orc_c3hlac(const orc_grid* g, const int32_t* leaf_layout, const float* cloud,
                   int variant, int thr_r, int thr_g, int thr_b, float voxel_size,
                   int subdiv, int ox, int oy, int oz, int color_mode, int exact,
                   float* feat_out, int32_t subdiv_out[3]) {
  const int F = variant;
  if (F != 981 && F != 117) return -1;
  /* setVoxelFilter, c3_hlac.cpp:204-231 */
  int64_t hist_num = 1;
  float inv_s = 0;
  int sb[3] = {0, 0, 0}, sbm[3] = {0, 0, 0};
  if (subdiv > 0) {
    inv_s = 1.0 / subdiv;
    if (g->div_b[0] <= ox || g->div_b[1] <= oy || g->div_b[2] <= oz) {
      if (subdiv_out) subdiv_out[0] = subdiv_out[1] = subdiv_out[2] = 0;
      return 0; /* setVoxelFilter returns false: empty feature */
    }
    const int off[3] = {ox, oy, oz};
    for (int a = 0; a < 3; ++a) sb[a] = (int)ceilf((g->div_b[a] - off[a]) * inv_s);
    sbm[0] = 1;
    sbm[1] = sb[0];
    sbm[2] = sb[0] * sb[1];
    hist_num = (int64_t)sb[0] * sb[1] * sb[2];
  } else if (subdiv < 0) {
    return -2;
  }
  if (subdiv_out) {
    subdiv_out[0] = sb[0];
    subdiv_out[1] = sb[1];
    subdiv_out[2] = sb[2];
  }
  /* computeFeature: negative threshold -> silent empty output (c3_hlac.cpp:398-401) */
  if (thr_r < 0 || thr_g < 0 || thr_b < 0) return -3;
  if (!feat_out) return hist_num;

  hist_t h;
  h.f = feat_out;
  h.x = NULL;
  for (int64_t i = 0; i < hist_num * F; ++i) feat_out[i] = 0;
  if (exact) {
    h.x = (int64_t*)calloc((size_t)(hist_num * F), sizeof(int64_t));
    if (!h.x) return -4;
  }
  int32_t lut[512];
  orc_lut(color_mode, lut);
  const int thr[3] = {thr_r, thr_g, thr_b};
  const int off[3] = {ox, oy, oz};
  const int64_t divb_mul[3] = {1, g->div_b[0], (int64_t)g->div_b[0] * g->div_b[1]};

  for (int64_t ci = 0; ci < g->n_occ; ++ci) {
    const float* p = cloud + 4 * ci;
    int64_t hist_idx = 0;
    if (hist_num != 1) {
      int tmp[3];
      for (int a = 0; a < 3; ++a) tmp[a] = (int)(floorf(p[a] / voxel_size) - g->min_b[a] - off[a]);
      if (tmp[0] < 0 || tmp[1] < 0 || tmp[2] < 0) continue;
      int ijk[3];
      for (int a = 0; a < 3; ++a) ijk[a] = (int)floorf(tmp[a] * inv_s);
      hist_idx = ijk[0] * (int64_t)sbm[0] + ijk[1] * (int64_t)sbm[1] + ijk[2] * (int64_t)sbm[2];
      if (ijk[0] >= sb[0] || ijk[1] >= sb[1] || ijk[2] >= sb[2]) {
        if (h.x) free(h.x);
        return -5;
      }
    }
    const int64_t base = hist_idx * F;
    uint32_t color;
    memcpy(&color, &p[3], 4);
    const int cr = (color & 0xff0000) >> 16, cg = (color & 0x00ff00) >> 8, cb = color & 0xff;
    const int cbin[6] = {cr > thr[0], !(cr > thr[0]), cg > thr[1], !(cg > thr[1]),
                         cb > thr[2], !(cb > thr[2])};
    const int ca[6] = {lut[2 * cr], lut[2 * cr + 1], lut[2 * cg],
                       lut[2 * cg + 1], lut[2 * cb], lut[2 * cb + 1]};
    /* addC3HLACcol0Bin */
    const int z0 = (F == 981) ? 495 : 63, pc0 = (F == 981) ? 969 : 105;
    for (int c = 0; c < 6; ++c)
      if (cbin[c]) hadd(&h, exact, base, z0 + c, 1);
    for (int q = 0; q < 12; ++q)
      if (cbin[PAIRS[q][0]] && cbin[PAIRS[q][1]]) hadd(&h, exact, base, pc0 + q, 1);
    /* setColor + addC3HLACcol0 */
    const int auto0 = (F == 981) ? 474 : 42;
    for (int c = 0; c < 6; ++c) hadd(&h, exact, base, c, ca[c]);
    for (int c = 0; c < 6; ++c)
      for (int n = c; n < 6; ++n) hadd(&h, exact, base, auto0 + tri6(c, n), ca[c] * ca[n]);
    /* getNeighborCentroidIndices (PCL): base cell from the centroid, floor(p / leaf_size)
     * in the reference's PCL (floor(p * inverse_leaf_size) later) */
    int ijk[3];
    for (int a = 0; a < 3; ++a)
      ijk[a] = g_pcl_era ? (int)floorf(p[a] / g->leaf) : (int)floorf(p[a] * g->inv_leaf);
    for (int k = 0; k < 13; ++k) {
      int ok = 1;
      int64_t lin = 0;
      for (int a = 0; a < 3; ++a) {
        const int d2min = g->min_b[a] - ijk[a], d2max = g->max_b[a] - ijk[a];
        if (!(d2min <= REL[k][a] && d2max >= REL[k][a])) ok = 0;
        lin += (int64_t)(ijk[a] + REL[k][a] - g->min_b[a]) * divb_mul[a];
      }
      if (!ok) continue;
      const int32_t ni = leaf_layout[lin];
      if (ni == -1) continue;
      uint32_t ncol;
      memcpy(&ncol, &cloud[4 * ni + 3], 4);
      const int r = (ncol & 0xff0000) >> 16, gg = (ncol & 0x00ff00) >> 8, b = ncol & 0xff;
      const int nbin[6] = {r > thr[0], !(r > thr[0]), gg > thr[1], !(gg > thr[1]),
                           b > thr[2], !(b > thr[2])};
      const int na[6] = {lut[2 * r], lut[2 * r + 1], lut[2 * gg],
                         lut[2 * gg + 1], lut[2 * b], lut[2 * b + 1]};
      /* addC3HLACcol1Bin: the active centre row receives all six neighbour bins */
      for (int c = 0; c < 6; ++c) {
        if (!cbin[c]) continue;
        for (int n = 0; n < 6; ++n) {
          const int idx = (F == 981) ? 495 + bin981(k, c, n) : 69 + 6 * c + n;
          hadd(&h, exact, base, idx, nbin[n]);
        }
      }
      /* setColor + addC3HLACcol1 */
      for (int c = 0; c < 6; ++c)
        for (int n = 0; n < 6; ++n) {
          const int idx = (F == 981) ? bin981(k, c, n) : 6 + 6 * c + n;
          hadd(&h, exact, base, idx, ca[c] * na[n]);
        }
    }
  }
  if (exact) {
    for (int64_t i = 0; i < hist_num * F; ++i) feat_out[i] = (float)h.x[i];
    free(h.x);
  }
  /* normalizeC3HLAC, c3_hlac.cpp:233-250 (117) and :329-342 (981) */
  for (int64_t hh = 0; hh < hist_num; ++hh) {
    float* o = feat_out + hh * F;
    if (F == 981) {
      for (int i = 0; i < 6; ++i) o[i] *= NORMALIZE_0;
      for (int i = 6; i < 495; ++i) o[i] *= NORMALIZE_1;
      for (int i = 495; i < 501; ++i) o[i] *= NORMALIZE_0_BIN;
      for (int i = 501; i < 981; ++i) o[i] *= NORMALIZE_1_BIN;
    } else {
      for (int i = 0; i < 6; ++i) o[i] *= NORMALIZE_117_0;
      for (int i = 6; i < 42; ++i) o[i] *= NORMALIZE_117_1;
      for (int i = 42; i < 63; ++i) o[i] *= NORMALIZE_1;
      for (int i = 63; i < 69; ++i) o[i] *= NORMALIZE_117_0_BIN;
      for (int i = 69; i < 105; ++i) o[i] *= NORMALIZE_117_1_BIN;
      for (int i = 105; i < 117; ++i) o[i] *= NORMALIZE_1_BIN;
    }
  }
  return hist_num;
}

void orc_exist(const float* feat, int64_t hist_num, int F, int32_t* exist_out) {
  for (int64_t h = 0; h < hist_num; ++h) {
    const float* f = feat + h * F;
    exist_out[h] = (int32_t)((f[0] + f[1]) * 2 + 0.001);
  }
}

/* ------------------------------------------------------------------ search */

enum { S_MODE_1, S_MODE_2, S_MODE_3, S_MODE_4, S_MODE_5, S_MODE_6 };

typedef struct {
  int r1, r2, r3, rank, M;
  double* sc;
  int32_t *x, *y, *z, *mode;
} lists_t;

static void get_range(const lists_t* L, int mode, int* xr, int* yr, int* zr) {
  switch (mode) { /* search.cpp:218-251 */
    case S_MODE_1: *xr = L->r1; *yr = L->r2; *zr = L->r3; break;
    case S_MODE_2: *xr = L->r1; *yr = L->r3; *zr = L->r2; break;
    case S_MODE_3: *xr = L->r2; *yr = L->r1; *zr = L->r3; break;
    case S_MODE_4: *xr = L->r2; *yr = L->r3; *zr = L->r1; break;
    case S_MODE_5: *xr = L->r3; *yr = L->r1; *zr = L->r2; break;
    default: *xr = L->r3; *yr = L->r2; *zr = L->r1; break;
  }
}
static int x_range(const lists_t* L, int mode) {
  int a, b, c;
  get_range(L, mode, &a, &b, &c);
  return a;
}
static int y_range(const lists_t* L, int mode) {
  int a, b, c;
  get_range(L, mode, &a, &b, &c);
  return b;
}
static int z_range(const lists_t* L, int mode) {
  int a, b, c;
  get_range(L, mode, &a, &b, &c);
  return c;
}

/* checkOverlap, search.cpp:327-356 / :862-891 */
static int check_overlap(const lists_t* L, int m, int x, int y, int z, int mode) {
  int xr, yr, zr, num;
  get_range(L, mode, &xr, &yr, &zr);
  const int o = m * L->rank;
  for (num = 0; num < L->rank - 1; num++) {
    int v1 = L->x[o + num] - x;
    if (v1 < 0) v1 = -v1 - x_range(L, L->mode[o + num]);
    else v1 -= xr;
    int v2 = L->y[o + num] - y;
    if (v2 < 0) v2 = -v2 - y_range(L, L->mode[o + num]);
    else v2 -= yr;
    int v3 = L->z[o + num] - z;
    if (v3 < 0) v3 = -v3 - z_range(L, L->mode[o + num]);
    else v3 -= zr;
    if (v1 <= 0 && v2 <= 0 && v3 <= 0) return num;
  }
  return num;
}
static void max_cpy(lists_t* L, int m, int src, int dst) {
  const int o = m * L->rank;
  L->sc[o + dst] = L->sc[o + src];
  L->x[o + dst] = L->x[o + src];
  L->y[o + dst] = L->y[o + src];
  L->z[o + dst] = L->z[o + src];
  L->mode[o + dst] = L->mode[o + src];
}
/* the rank-update of searchPart, search.cpp:464-474 */
static void rank_update(lists_t* L, int m, double dot, int x, int y, int z, int mode) {
  const int o = m * L->rank;
  for (int i = 0; i < L->rank; i++) {
    if (dot > L->sc[o + i]) {
      const int ov = check_overlap(L, m, x, y, z, mode);
      for (int j = 0; j < ov - i; j++) max_cpy(L, m, ov - 1 - j, ov - j);
      if (i <= ov) {
        L->sc[o + i] = dot;
        L->x[o + i] = x;
        L->y[o + i] = y;
        L->z[o + i] = z;
        L->mode[o + i] = mode;
      }
      break;
    }
  }
}

/* clipValue, search.cpp:484-535, for scalar T (int or double); fp32 vectors below */
#define CLIP_BODY(P)                                                                      \
  if (z == 0) {                                                                           \
    if (y == 0) {                                                                         \
      if (x == 0) r = P(xr - 1, yr - 1, zr - 1);                                          \
      else r = P(x + xr - 1, yr - 1, zr - 1) - P(x - 1, yr - 1, zr - 1);                 \
    } else {                                                                              \
      if (x == 0) r = P(xr - 1, y + yr - 1, zr - 1) - P(xr - 1, y - 1, zr - 1);           \
      else                                                                                \
        r = P(x + xr - 1, y + yr - 1, zr - 1) - P(x - 1, y + yr - 1, zr - 1) -            \
            P(x + xr - 1, y - 1, zr - 1) + P(x - 1, y - 1, zr - 1);                       \
    }                                                                                     \
  } else {                                                                                \
    if (y == 0) {                                                                         \
      if (x == 0) r = P(xr - 1, yr - 1, z + zr - 1) - P(xr - 1, yr - 1, z - 1);           \
      else                                                                                \
        r = P(x + xr - 1, yr - 1, z + zr - 1) - P(x - 1, yr - 1, z + zr - 1) -            \
            P(x + xr - 1, yr - 1, z - 1) + P(x - 1, yr - 1, z - 1);                       \
    } else {                                                                              \
      if (x == 0)                                                                         \
        r = P(xr - 1, y + yr - 1, z + zr - 1) - P(xr - 1, y + yr - 1, z - 1) -            \
            P(xr - 1, y - 1, z + zr - 1) + P(xr - 1, y - 1, z - 1);                       \
      else                                                                                \
        r = P(x + xr - 1, y + yr - 1, z + zr - 1) - P(x - 1, y + yr - 1, z + zr - 1) -    \
            P(x + xr - 1, y - 1, z + zr - 1) - P(x + xr - 1, y + yr - 1, z - 1) +         \
            P(x - 1, y - 1, z + zr - 1) + P(x - 1, y + yr - 1, z - 1) +                   \
            P(x + xr - 1, y - 1, z - 1) - P(x - 1, y - 1, z - 1);                         \
    }                                                                                     \
  }

typedef struct {
  int xn, xyn;
} sat_dims;

static int clip_int(const int32_t* S, sat_dims d, int x, int y, int z, int xr, int yr, int zr) {
  int r;
#define PI_(a, b, c) S[(a) + (b) * d.xn + (c) * d.xyn]
  CLIP_BODY(PI_)
#undef PI_
  return r;
}
static float clip_f(const float* S, int D, int dd, sat_dims d, int x, int y, int z, int xr,
                    int yr, int zr) {
  float r;
#define PF_(a, b, c) S[((a) + (b) * d.xn + (c) * d.xyn) * (int64_t)D + dd]
  CLIP_BODY(PF_)
#undef PF_
  return r;
}
static double clip_d(const double* S, int D, int dd, sat_dims d, int x, int y, int z, int xr,
                     int yr, int zr) {
  double r;
#define PD_(a, b, c) S[((a) + (b) * d.xn + (c) * d.xyn) * (int64_t)D + dd]
  CLIP_BODY(PD_)
#undef PD_
  return r;
}

/* summed-volume recurrence of setData (search.cpp:582-653), elementwise left-assoc */
#define SAT_STEP(A, IDX, X, Y, Z)                                                        \
  do {                                                                                   \
    if ((Z) == 0) {                                                                      \
      if ((Y) == 0) {                                                                    \
        if ((X) != 0) A(IDX) += A(IDX - 1);                                              \
      } else {                                                                           \
        if ((X) == 0) A(IDX) += A(IDX - xn);                                             \
        else A(IDX) += A(IDX - 1) + A(IDX - xn) - A(IDX - 1 - xn);                       \
      }                                                                                  \
    } else {                                                                             \
      if ((Y) == 0) {                                                                    \
        if ((X) == 0) A(IDX) += A(IDX - xyn);                                            \
        else A(IDX) += A(IDX - 1) + A(IDX - xyn) - A(IDX - 1 - xyn);                     \
      } else {                                                                           \
        if ((X) == 0) A(IDX) += A(IDX - xn) + A(IDX - xyn) - A(IDX - xn - xyn);          \
        else                                                                             \
          A(IDX) += A(IDX - 1) + A(IDX - xn) + A(IDX - xyn) - A(IDX - 1 - xn) -          \
                    A(IDX - xn - xyn) - A(IDX - 1 - xyn) + A(IDX - 1 - xn - xyn);        \
      }                                                                                  \
    }                                                                                    \
  } while (0)

static void mode_schedule(int r1, int r2, int r3, int rotate, int* modes, int* nm) {
  /* search.cpp:384-427 */
  if (!rotate) {
    modes[0] = S_MODE_1;
    *nm = 1;
    return;
  }
  if (r1 == r2) {
    if (r2 == r3) {
      modes[0] = S_MODE_1;
      *nm = 1;
    } else {
      modes[0] = S_MODE_1; modes[1] = S_MODE_2; modes[2] = S_MODE_5;
      *nm = 3;
    }
  } else if (r2 == r3) {
    modes[0] = S_MODE_1; modes[1] = S_MODE_5; modes[2] = S_MODE_6;
    *nm = 3;
  } else if (r1 == r3) {
    modes[0] = S_MODE_1; modes[1] = S_MODE_5; modes[2] = S_MODE_3;
    *nm = 3;
  } else {
    for (int i = 0; i < 6; ++i) modes[i] = i;
    *nm = 6;
  }
}

int orc_search(int xn, int yn, int zn, const float* feat, int F, const int32_t* exist,
               const float* axis_p, int D, const float* fmax, int fmax_len,
               const float* axis_q, int M, int r, int range1, int range2, int range3,
               int rank, int thr, int rotate, int dbl, double* st_score, int32_t* st_x,
               int32_t* st_y, int32_t* st_z, int32_t* st_mode, double* scores_out) {
  const int xyn = xn * yn;
  const int64_t H = (int64_t)xyn * zn;
  if (H < 1) return 0; /* setData returns early; search() is skipped by the caller */
  if (!axis_p) D = F;
  lists_t L = {range1, range2, range3, rank, M, st_score, st_x, st_y, st_z, st_mode};
  int32_t* ex = (int32_t*)malloc(sizeof(int32_t) * (size_t)H);
  float* gf = dbl ? NULL : (float*)malloc(sizeof(float) * (size_t)(H * D));
  double* gd = dbl ? (double*)malloc(sizeof(double) * (size_t)(H * D)) : NULL;
  float* fv = (float*)malloc(sizeof(float) * (size_t)F);
  if (!ex || (!gf && !gd) || !fv) return -4;
  memcpy(ex, exist, sizeof(int32_t) * (size_t)H);

  /* setData: normalise, compress, summed-volume table (search.cpp:539-658) */
  int64_t idx = 0;
  for (int z = 0; z < zn; z++)
    for (int y = 0; y < yn; y++)
      for (int x = 0; x < xn; x++, idx++) {
        memcpy(fv, feat + idx * F, sizeof(float) * (size_t)F);
        for (int t = 0; t < fmax_len && t < F; t++) {
          if (fmax[t] == 0) fv[t] = 0;
          else if (fv[t] == fmax[t]) fv[t] = 1;
          else fv[t] = 1 * fv[t] / fmax[t];
        }
        for (int d = 0; d < D; d++) {
          if (dbl) {
            double s = 0;
            if (axis_p)
              for (int j = 0; j < F; j++) s += (double)axis_p[(int64_t)d * F + j] * fv[j];
            else
              s = fv[d];
            gd[idx * D + d] = s;
          } else {
            float s = 0;
            if (axis_p)
              for (int j = 0; j < F; j++) s += axis_p[(int64_t)d * F + j] * fv[j];
            else
              s = fv[d];
            gf[idx * D + d] = s;
          }
        }
#define AE_(i) ex[i]
        SAT_STEP(AE_, idx, x, y, z);
#undef AE_
        for (int d = 0; d < D; d++) {
          if (dbl) {
#define AD_(i) gd[(i) * (int64_t)D + d]
            SAT_STEP(AD_, idx, x, y, z);
#undef AD_
          } else {
#define AF_(i) gf[(i) * (int64_t)D + d]
            SAT_STEP(AF_, idx, x, y, z);
#undef AF_
          }
        }
      }

  /* search()/searchWithoutRotation() -> searchPart(mode) for each scheduled mode */
  int modes[6], nm;
  mode_schedule(range1, range2, range3, rotate, modes, &nm);
  sat_dims sd = {xn, xyn};
  float* ff = (float*)malloc(sizeof(float) * (size_t)D);
  double* fd = (double*)malloc(sizeof(double) * (size_t)D);
  int64_t sofs = 0;
  for (int mi = 0; mi < nm; ++mi) {
    const int mode = modes[mi];
    int xr, yr, zr;
    get_range(&L, mode, &xr, &yr, &zr);
    const int xe = xn - xr + 1, ye = yn - yr + 1, ze = zn - zr + 1;
    if (!(xe > 0 && ye > 0 && ze > 0)) continue;
    const int64_t P = (int64_t)xe * ye * ze;
    int64_t p = 0;
    for (int z = 0; z < ze; z++)
      for (int y = 0; y < ye; y++)
        for (int x = 0; x < xe; x++, p++) {
          const int en = clip_int(ex, sd, x, y, z, xr, yr, zr);
          if (!(en > thr)) {
            if (scores_out)
              for (int m = 0; m < M; ++m) scores_out[sofs + m * P + p] = -1.0;
            continue;
          }
          double sum;
          if (dbl) {
            double s = 0;
            for (int d = 0; d < D; d++) {
              fd[d] = clip_d(gd, D, d, sd, x, y, z, xr, yr, zr);
              s += fd[d] * fd[d];
            }
            sum = s;
          } else {
            float s = 0;
            for (int d = 0; d < D; d++) {
              ff[d] = clip_f(gf, D, d, sd, x, y, z, xr, yr, zr);
              s += ff[d] * ff[d];
            }
            sum = s;
          }
          sum = sqrt(sum);
          for (int m = 0; m < M; ++m) {
            double dot;
            const float* Q = axis_q + (int64_t)m * r * D;
            if (dbl) {
              double q2 = 0;
              for (int i = 0; i < r; i++) {
                double t = 0;
                for (int d = 0; d < D; d++) t += (double)Q[(int64_t)i * D + d] * fd[d];
                q2 += t * t;
              }
              dot = q2;
            } else {
              float q2 = 0;
              for (int i = 0; i < r; i++) {
                float t = 0;
                for (int d = 0; d < D; d++) t += Q[(int64_t)i * D + d] * ff[d];
                q2 += t * t;
              }
              dot = q2;
            }
            dot = sqrt(dot);
            dot /= sum;
            if (scores_out) scores_out[sofs + m * P + p] = dot;
            rank_update(&L, m, dot, x, y, z, mode);
          }
        }
    sofs += P * M;
  }
  free(ff);
  free(fd);
  free(ex);
  free(gf);
  free(gd);
  free(fv);
  return nm;
}

void orc_remove_overlap(int M, int rank, int range1, int range2, int range3,
                        double* st_score, int32_t* st_x, int32_t* st_y, int32_t* st_z,
                        int32_t* st_mode) {
  lists_t L = {range1, range2, range3, rank, M, st_score, st_x, st_y, st_z, st_mode};
  for (int m = 0; m < M; m++) {
    for (int i = 0; i < 1; i++) {
      for (int m2 = 0; m2 < M; m2++) {
        if (m2 == m) continue;
        const int o = m * rank;
        const int ov = check_overlap(&L, m2, st_x[o + i], st_y[o + i], st_z[o + i], st_mode[o + i]);
        if (st_score[o + i] > st_score[m2 * rank + ov])
          for (int j = ov; j < rank - 1; j++) max_cpy(&L, m2, j + 1, j);
        else
          for (int j = i; j < rank - 1; j++) max_cpy(&L, m, j + 1, j);
      }
    }
  }
}

/* ------------------------------------------------------------------ PCA reader */

int orc_pca_read(const char* path, int ascii, float* axis, float* var, float* mean,
                 int* has_mean, int max_dim) {
  FILE* fp = fopen(path, ascii ? "r" : "rb");
  if (!fp) return -1;
  int dim = -1;
  if (ascii) {
    if (fscanf(fp, "%d\n", &dim) != 1) dim = -1;
  } else {
    if (fread(&dim, sizeof(int), 1, fp) != 1) dim = -1;
  }
  if (dim <= 0 || dim > max_dim) {
    fclose(fp);
    return -2;
  }
  int ok = 1;
  for (int i = 0; i < dim && ok; i++)
    for (int j = 0; j < dim && ok; j++) {
      float* dst = &axis[(int64_t)i * dim + j]; /* axis(j, i): column i contiguous */
      ok = ascii ? fscanf(fp, "%f ", dst) == 1 : fread(dst, sizeof(float), 1, fp) == 1;
    }
  for (int i = 0; i < dim && ok; i++)
    ok = ascii ? fscanf(fp, "%f\n", &var[i]) == 1 : fread(&var[i], sizeof(float), 1, fp) == 1;
  if (!ok) {
    fclose(fp);
    return -3;
  }
  float t;
  const int got = ascii ? fscanf(fp, "%f\n", &t) == 1 : fread(&t, sizeof(float), 1, fp) == 1;
  *has_mean = 0;
  if (got) {
    *has_mean = 1;
    if (mean) mean[0] = t;
    for (int i = 1; i < dim; i++) {
      float v = 0;
      if (ascii ? fscanf(fp, "%f\n", &v) != 1 : fread(&v, sizeof(float), 1, fp) != 1) break;
      if (mean) mean[i] = v;
    }
  }
  fclose(fp);
  return dim;
}
