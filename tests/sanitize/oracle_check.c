/* ASan/UBSan run of the oracle's C restatement (sanitizers on the
 * CPU build).  Synthetic cloud -> voxel bounds/fill -> C3-HLAC 981 and 117 (fp32 and exact
 * modes, several subdivisions/offsets) -> exist -> search (rotate, multi-model, rank 2)
 * -> removeOverlap, plus PCA::read on the files given on the command line.  Exit 0 = no
 * sanitizer report (they abort). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/c3hlac_oracle.h"

static uint32_t lcg(uint32_t* s) { return *s = *s * 1664525u + 1013904223u; }

int main(int argc, char** argv) {
  const int64_t n = 20000;
  float* pts = malloc(n * 4 * sizeof(float));
  uint32_t s = 7;
  for (int64_t i = 0; i < n; ++i) {
    pts[4 * i + 0] = (lcg(&s) >> 8) * (1.0f / 16777216.0f) * 0.6f;
    pts[4 * i + 1] = (lcg(&s) >> 8) * (1.0f / 16777216.0f) * 0.5f;
    pts[4 * i + 2] = 0.5f + (lcg(&s) >> 8) * (1.0f / 16777216.0f) * 0.4f;
    uint32_t rgb = lcg(&s) & 0xffffffu;
    memcpy(&pts[4 * i + 3], &rgb, 4);
  }
  pts[4 * 5 + 0] = NAN; /* limitPoint drops non-finite points */
  orc_grid g;
  if (orc_voxel_bounds(pts, n, 0.02f, 1.2f, &g) != 0) return 10;
  const int64_t nv = (int64_t)g.div_b[0] * g.div_b[1] * g.div_b[2];
  int32_t* layout = malloc(nv * sizeof(int32_t));
  float* cloud = malloc((g.n_valid + 1) * 4 * sizeof(float));
  if (orc_voxel_fill(pts, n, 1.2f, &g, layout, cloud) != 0) return 11;
  const int variants[2] = {981, 117};
  const int subdivs[3] = {0, 4, 7};
  for (int v = 0; v < 2; ++v)
    for (int sdi = 0; sdi < 3; ++sdi)
      for (int exact = 0; exact < 2; ++exact) {
        int32_t sb[3];
        const int F = variants[v];
        int64_t H = orc_c3hlac(&g, layout, cloud, F, 147, 146, 148, 0.02f, subdivs[sdi], 1, 0, 2, 1, exact, NULL, sb);
        if (H < 0) return 12;
        float* feat = malloc((H + 1) * F * sizeof(float));
        if (orc_c3hlac(&g, layout, cloud, F, 147, 146, 148, 0.02f, subdivs[sdi], 1, 0, 2, 1, exact, feat, sb) != H)
          return 13;
        int32_t* ex = malloc((H + 1) * sizeof(int32_t));
        orc_exist(feat, H, F, ex);
        if (subdivs[sdi] > 0) {
          const int D = 12, M = 3, r = 4, rank = 2;
          float* ap = malloc((size_t)D * F * sizeof(float));
          float* aq = malloc((size_t)M * r * D * sizeof(float));
          for (int i = 0; i < D * F; ++i) ap[i] = ((int)(lcg(&s) >> 16) - 32768) / 32768.0f;
          for (int i = 0; i < M * r * D; ++i) aq[i] = ((int)(lcg(&s) >> 16) - 32768) / 32768.0f;
          double sc[M * rank];
          int32_t x[M * rank], y[M * rank], z[M * rank], mode[M * rank];
          memset(sc, 0, sizeof(sc));
          memset(x, 0, sizeof(x));
          memset(y, 0, sizeof(y));
          memset(z, 0, sizeof(z));
          memset(mode, 0, sizeof(mode));
          for (int dbl = 0; dbl < 2; ++dbl)
            if (orc_search(sb[0], sb[1], sb[2], feat, F, ex, ap, D, NULL, 0, aq, M, r, 2, 2, 1, rank, 1, 1, dbl, sc, x,
                           y, z, mode, NULL) < 0)
              return 14;
          orc_remove_overlap(M, rank, 2, 2, 1, sc, x, y, z, mode);
          free(ap);
          free(aq);
        }
        free(feat);
        free(ex);
      }
  for (int i = 1; i < argc; ++i) {
    int hm = 0, dim = 0;
    FILE* fp = fopen(argv[i], "rb");
    if (!fp || fread(&dim, sizeof(int), 1, fp) != 1 || dim <= 0 || dim > 4096) return 15;
    fclose(fp);
    float* a = malloc((size_t)dim * dim * sizeof(float));
    float* var = malloc(dim * sizeof(float));
    float* m = malloc(dim * sizeof(float));
    if (orc_pca_read(argv[i], 0, a, var, m, &hm, dim) != dim) return 16;
    free(a);
    free(var);
    free(m);
  }
  free(pts);
  free(layout);
  free(cloud);
  printf("oracle_check ok\n");
  return 0;
}
