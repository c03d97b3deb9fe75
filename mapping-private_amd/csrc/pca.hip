// pca.hip -- PCA training on the GPU: the model / scene subspace
// learning of pca_models.cpp and pca_scene.cpp behind the C-ABI.
//
//   PCA::addData (color_voxel_recognition/src/pca.cpp:48-69) is a SYRK over the added
//   rows.  It runs on the f64 matrix cores (v_mfma_f64_16x16x4_f64) from f32 rows
//   widened on the LDS store: f32 x f32 products are exact in f64 and the sums are f64,
//   so the correlation is the exact sum rounded a few times in f64 (the reference sums in
//   f32, one sample at a time).  Row chunks write per-chunk partial tiles that a reduce
//   kernel adds in a fixed order: the result does not depend on scheduling.  A constant-1
//   column F appended to the rows gives the mean sums (column F) and the count for free.
//
//   The 24-rotation augmentation of pca_models.cpp:109-171 adds, per row f, the vectors
//   compress(P_k f) for the 24 rotateFeature90 compositions P_k (c3_hlac.cpp:49-172,
//   pure index permutations).  Their correlation is  W A^T (sum_k P_k C P_k^T) A W  with
//   C = sum f f^T over the raw rows, so the rows are never expanded 24 x nor compressed
//   one by one: the rotated rows accumulate into their own raw F x F correlation, and
//   the solve gathers the 24 permuted copies of it and projects once (two f64 GEMMs).
//
//   PCA::solve (pca.cpp:73-105): 1 / nsample, mean subtraction, regularisation, then the
//   symmetric eigensolve on rocSOLVER's dsyevd (loaded at the first solve: the library
//   is large and only training needs it) and sortVecAndVal's stable descending order
//   (pca.cpp:244-271), written out as the float axis / variance / mean PCA::write stores.
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <rocsolver/rocsolver.h>  // types and prototypes only; the library is dlopen'ed

#include "c3h_internal.h"

using c3h::DevBuf;

namespace {

constexpr int kPT = 128;     // correlation tile edge
constexpr int kPK = 16;      // rows per LDS stage
constexpr int kPS = 144;     // LDS row stride in doubles (k and k + 1 rows 32 banks apart)
constexpr int kPTile = kPT * kPT;
constexpr int kMaxSyrkBlocks = 4096;
constexpr int kRot = 24;

typedef double pca_f64x4 __attribute__((ext_vector_type(4)));

// ---- rotateFeature90 as index maps ---------------------------------------------------
// One 495- / 486-dim half: indices 0..5 and 474.. are copied; the first-order block of
// colour pair (i centre, j neighbour) holds offset slots 6..14 (stride 9 in i) and
// 60..63 (stride 4 in i), 78 apart in j.  A rotation moves each slot to another and, for
// the offsets it reverses, swaps the pair (i, j).  Per mode: input slot s -> output slot
// and the swap flag (c3_hlac.cpp:77-160).
const int kSlot[13] = {6, 7, 8, 9, 10, 11, 12, 13, 14, 60, 61, 62, 63};
const int kRotSlot[4][13][2] = {
    {{8, 0}, {11, 0}, {14, 0}, {7, 0}, {10, 0}, {13, 0}, {6, 0}, {9, 0}, {12, 0}, {62, 0}, {63, 1}, {60, 1}, {61, 0}},
    {{8, 0}, {62, 0}, {12, 1}, {11, 0}, {63, 1}, {9, 1}, {14, 0}, {60, 1}, {6, 1}, {7, 0}, {61, 0}, {13, 1}, {10, 0}},
    {{12, 0}, {13, 0}, {14, 0}, {62, 1}, {61, 1}, {60, 1}, {8, 1}, {7, 1}, {6, 1}, {9, 0}, {10, 0}, {11, 0}, {63, 0}},
    {{12, 0}, {9, 0}, {6, 0}, {13, 0}, {10, 0}, {7, 0}, {14, 0}, {11, 0}, {8, 0}, {62, 1}, {63, 0}, {60, 0}, {61, 1}},
};

bool rot_dim_ok(int dim) { return dim == 981 || dim == 495 || dim == 486; }

// map[o] = input index of output o for one mode over a whole vector
std::vector<int32_t> rot_map(int dim, int mode) {
  std::vector<int32_t> m(dim);
  for (int o = 0; o < dim; ++o) m[o] = o;
  auto half = [&](int base) {
    for (int s = 0; s < 13; ++s) {
      const int is = kSlot[s], os = kRotSlot[mode][s][0], sw = kRotSlot[mode][s][1];
      const int istr = is < 60 ? 9 : 4, ostr = os < 60 ? 9 : 4;
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
          const int a = sw ? j : i, b = sw ? i : j;
          m[base + os + a * ostr + b * 78] = base + is + i * istr + j * 78;
        }
    }
  };
  half(0);
  if (dim == 981) half(495);
  return m;
}

// the 24 compositions pca_models.cpp:109-171 adds, in its order: I, R2, R2^2, R2^3,
// then R3, R3^2, R3^3, R1, R4 each followed by R2, R2^2, R2^3 applied on top
std::vector<int32_t> rot24_maps(int dim) {
  const std::vector<int32_t> m1 = rot_map(dim, 0), m2 = rot_map(dim, 1), m3 = rot_map(dim, 2), m4 = rot_map(dim, 3);
  std::vector<int32_t> I(dim);
  for (int o = 0; o < dim; ++o) I[o] = o;
  // applying rotation r on top of composite c: out[o] = c_in[r[o]] -> map c[r[o]]
  auto then = [&](const std::vector<int32_t>& c, const std::vector<int32_t>& r) {
    std::vector<int32_t> out(dim);
    for (int o = 0; o < dim; ++o) out[o] = c[r[o]];
    return out;
  };
  std::vector<int32_t> all;
  auto add_with_r2 = [&](std::vector<int32_t> c) {
    all.insert(all.end(), c.begin(), c.end());
    for (int t = 0; t < 3; ++t) {
      c = then(c, m2);
      all.insert(all.end(), c.begin(), c.end());
    }
  };
  const std::vector<int32_t> r3 = then(I, m3), r33 = then(r3, m3), r333 = then(r33, m3);
  add_with_r2(I);
  add_with_r2(r3);
  add_with_r2(r33);
  add_with_r2(r333);
  add_with_r2(then(I, m1));
  add_with_r2(then(I, m4));
  return all;
}

// ---- kernels ------------------------------------------------------------------------
__global__ void rotate_kernel(const float* __restrict__ in, float* __restrict__ out, int64_t n, int64_t ld,
                              int dim, const int32_t* __restrict__ map) {
  const int64_t total = n * dim;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / dim;
    const int o = (int)(e - r * dim);
    out[r * ld + o] = in[r * ld + map[o]];
  }
}

__device__ __forceinline__ void tile_pair(int t, int nb, int& bi, int& bj) {
  bi = 0;
  while (t >= nb - bi) {
    t -= nb - bi;
    ++bi;
  }
  bj = bi + t;
}

__device__ __forceinline__ float row_val(const float* __restrict__ X, int64_t ld, int64_t h, int64_t r1, int col, int F) {
  if (h >= r1) return 0.f;
  if (col < F) return X[h * ld + col];
  return col == F ? 1.f : 0.f;
}

// SYRK partials: block (s, t) sums rows [s rows_per, (s + 1) rows_per) of tile pair t
// (bi <= bj) of the (F + 1)-column rows into part[s][t] (128 x 128 doubles, row-major).
// 4 waves, each a 64 x 64 quadrant of 4 x 4 f64 MFMA tiles.
__global__ __launch_bounds__(256) void pca_syrk_kernel(const float* __restrict__ X, int64_t ld, int64_t n, int F,
                                                       int nb, int T, int64_t rows_per, double* __restrict__ part) {
  __shared__ double sa[kPK * kPS], sb[kPK * kPS];
  const int t = blockIdx.x % T, s = blockIdx.x / T;
  int bi, bj;
  tile_pair(t, nb, bi, bj);
  const bool diag = bi == bj;
  const int64_t r0 = (int64_t)s * rows_per, r1 = min(n, r0 + rows_per);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wi = w >> 1, wj = w & 1;
  const int c = tid & 127, rr0 = tid >> 7;
  const int ca = bi * kPT + c, cb = bj * kPT + c;
  pca_f64x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = pca_f64x4{0, 0, 0, 0};
  float va[8], vb[8];
  auto load = [&](int64_t h0) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int64_t h = h0 + rr0 + 2 * m;
      va[m] = row_val(X, ld, h, r1, ca, F);
      vb[m] = diag ? 0.f : row_val(X, ld, h, r1, cb, F);
    }
  };
  if (r0 < r1) load(r0);
  for (int64_t h0 = r0; h0 < r1; h0 += kPK) {
    __syncthreads();  // the previous stage's LDS reads are done
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      sa[(rr0 + 2 * m) * kPS + c] = (double)va[m];
      if (!diag) sb[(rr0 + 2 * m) * kPS + c] = (double)vb[m];
    }
    __syncthreads();
    if (h0 + kPK < r1) load(h0 + kPK);  // next stage's rows in flight during the MFMAs
    const double* pb = diag ? sa : sb;
#pragma unroll
    for (int kk = 0; kk < kPK / 4; ++kk) {
      const int k = 4 * kk + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = sa[k * kPS + wi * 64 + i * 16 + (lane & 15)];
        b[i] = pb[k * kPS + wj * 64 + i * 16 + (lane & 15)];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // C/D map of the f64 16x16 tile: column lane & 15, row (lane >> 4) + 4 r
  double* out = part + ((int64_t)s * T + t) * kPTile;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wi * 64 + i * 16 + (lane >> 4) + 4 * r, col = wj * 64 + j * 16 + (lane & 15);
        out[row * kPT + col] = acc[i][j][r];
      }
}

// acc[e] += sum over s (in order) of part[s][e]
__global__ void pca_reduce_kernel(const double* __restrict__ part, int S, int64_t len, double* __restrict__ acc) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < len; e += (int64_t)gridDim.x * blockDim.x) {
    double v = 0;
    for (int s = 0; s < S; ++s) v += part[(int64_t)s * len + e];
    acc[e] += v;
  }
}

__device__ __forceinline__ double tile_get(const double* __restrict__ acc, int nb, int i, int j) {
  if (i > j) {
    const int t = i;
    i = j;
    j = t;
  }
  const int bi = i >> 7, bj = j >> 7;
  const int t = bi * nb - bi * (bi - 1) / 2 + (bj - bi);
  return acc[(int64_t)t * kPTile + (i & 127) * kPT + (j & 127)];
}

// full F x F correlation sums (+ the column-F mean sums) of the plain rows plus the 24
// permuted copies of the rotated rows' correlation
__global__ void pca_unpack_kernel(const double* __restrict__ plain, const double* __restrict__ rot,
                                  const int32_t* __restrict__ maps, int F, int nb, double* __restrict__ C,
                                  double* __restrict__ msum) {
  const int64_t total = (int64_t)F * (F + 1);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int o1 = (int)(e / (F + 1)), o2 = (int)(e - (int64_t)o1 * (F + 1));  // o2 == F: sums
    double v = plain ? tile_get(plain, nb, o1, o2) : 0.0;
    if (rot)
      for (int k = 0; k < kRot; ++k) {
        const int32_t* m = maps + (int64_t)k * F;
        v += tile_get(rot, nb, m[o1], o2 < F ? m[o2] : F);
      }
    if (o2 < F)
      C[(int64_t)o1 * F + o2] = v;
    else
      msum[o1] = v;
  }
}

// C[m][n] = sum_k A(m, k) B(k, n) in f64, A / B / C addressed by element strides
__global__ __launch_bounds__(256) void gemm_f64_kernel(const double* __restrict__ A, int64_t am, int64_t ak,
                                                       const double* __restrict__ B, int64_t bk, int64_t bn,
                                                       double* __restrict__ Cm, int64_t cm, int64_t cn, int M, int N,
                                                       int K) {
  __shared__ double sA[16][17], sB[16][17];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  const int m = blockIdx.y * 16 + ty, nn = blockIdx.x * 16 + tx;
  double v = 0;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const int ma = blockIdx.y * 16 + ty, ka = k0 + tx;
    sA[ty][tx] = ma < M && ka < K ? A[ma * am + ka * ak] : 0.0;
    const int kb = k0 + ty, nb2 = blockIdx.x * 16 + tx;
    sB[ty][tx] = kb < K && nb2 < N ? B[kb * bk + nb2 * bn] : 0.0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; ++k) v = fma(sA[ty][k], sB[k][tx], v);
    __syncthreads();
  }
  if (m < M && nn < N) Cm[m * cm + nn * cn] = v;
}

// pca.cpp:80-98 on the d x d matrix (symmetric, so the lower-triangle copy is implicit)
__global__ void pca_finalize_kernel(double* __restrict__ G, double* __restrict__ mean, int d, double inv_n,
                                    int mean_flg, int reg_flg, double reg) {
  const int64_t total = (int64_t)d * d;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / d), j = (int)(e - (int64_t)i * d);
    double v = G[e] * inv_n;
    if (mean_flg) v -= (mean[i] * inv_n) * (mean[j] * inv_n);
    if (reg_flg && i == j) v += reg;
    G[e] = v;
  }
}

__global__ void pca_scale_kernel(double* __restrict__ v, int d, double s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d) v[i] *= s;
}

// sortVecAndVal (pca.cpp:244-271): the bubble sort swaps only on a strict '<', so it is
// the stable descending order: position of i = #{j : w_j > w_i} + #{j < i : w_j == w_i}
__global__ void pca_sort_kernel(const double* __restrict__ w, const double* __restrict__ V, int d,
                                float* __restrict__ axis, float* __restrict__ var) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < d; i += gridDim.x * blockDim.x) {
    const double wi = w[i];
    int pos = 0;
    for (int j = 0; j < d; ++j) pos += (w[j] > wi) || (j < i && w[j] == wi);
    var[pos] = (float)wi;
    for (int r = 0; r < d; ++r) axis[(int64_t)pos * d + r] = (float)V[(int64_t)i * d + r];
  }
}

// ---- rocSOLVER, loaded at the first solve --------------------------------------------
struct Solver {
  std::once_flag once;
  bool ok = false;
  std::string err;
  decltype(&rocblas_create_handle) create = nullptr;
  decltype(&rocblas_destroy_handle) destroy = nullptr;
  decltype(&rocblas_set_stream) set_stream = nullptr;
  decltype(&rocsolver_dsyevd) dsyevd = nullptr;
};
Solver g_solver;

bool solver_load() {
  std::call_once(g_solver.once, [] {
    void* blas = dlopen("librocblas.so.5", RTLD_NOW | RTLD_GLOBAL);
    if (!blas) blas = dlopen("/opt/rocm/lib/librocblas.so.5", RTLD_NOW | RTLD_GLOBAL);
    void* sol = dlopen("librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!sol) sol = dlopen("/opt/rocm/lib/librocsolver.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!blas || !sol) {
      g_solver.err = std::string("cannot load rocSOLVER: ") + dlerror();
      return;
    }
    g_solver.create = (decltype(g_solver.create))dlsym(blas, "rocblas_create_handle");
    g_solver.destroy = (decltype(g_solver.destroy))dlsym(blas, "rocblas_destroy_handle");
    g_solver.set_stream = (decltype(g_solver.set_stream))dlsym(blas, "rocblas_set_stream");
    g_solver.dsyevd = (decltype(g_solver.dsyevd))dlsym(sol, "rocsolver_dsyevd");
    g_solver.ok = g_solver.create && g_solver.destroy && g_solver.set_stream && g_solver.dsyevd;
    if (!g_solver.ok) g_solver.err = "rocSOLVER symbols missing";
  });
  return g_solver.ok;
}

template <class T>
void release(DevBuf<T>& b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.n = 0;
}

int grid_for(int64_t total) { return (int)std::min<int64_t>((total + 255) / 256, 8192); }

}  // namespace

struct c3h_pca {
  int device = 0;
  hipStream_t stream = nullptr, own_stream = nullptr;
  std::string err;
  bool mean_flg = true;
  int F = -1;                 // raw row dimension (fixed by the first add)
  int nb = 0, T = 0;          // tile blocks per axis, tile pairs
  int D = 0;                  // compressed dimension (0 = no compression)
  bool whiten = false;
  std::vector<double> h_proj;  // F x D row-major: axis / sqrt(var)
  long long nsample = 0;
  DevBuf<double> acc_plain, acc_rot, part, C, msum, tmp, G, W, E, proj;
  DevBuf<int32_t> maps, info;
  DevBuf<float> stage, out_axis, out_var, out_mean;
  bool have_plain = false, have_rot = false;
  bool solved = false;
  int dim_out = 0;
  rocblas_handle blas = nullptr;
};

namespace {

int pfail(c3h_pca* p, int code, const std::string& msg) {
  if (p) p->err = msg;
  return code;
}

#define PHIP(expr)                                                                     \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) return pfail(p, C3H_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

template <class T>
int pensure(c3h_pca* p, DevBuf<T>& b, size_t n) {
  if (n == 0) n = 1;
  if (b.n >= n) return C3H_OK;
  release(b);
  if (hipMalloc(&b.p, n * sizeof(T)) != hipSuccess) {
    b.p = nullptr;
    return pfail(p, C3H_ERR_NOMEM, "hipMalloc failed");
  }
  b.n = n;
  return C3H_OK;
}

#define PENSURE(buf, n)                               \
  do {                                                \
    int rc_ = pensure(p, buf, (size_t)(n));           \
    if (rc_ != C3H_OK) return rc_;                    \
  } while (0)

// SYRK of n device rows into acc (T tile pairs, f64)
int syrk_rows(c3h_pca* p, const float* X, int64_t n, int64_t ld, DevBuf<double>& acc) {
  if (n <= 0) return C3H_OK;
  int64_t S = std::min<int64_t>((n + 255) / 256, std::max(1, kMaxSyrkBlocks / p->T));
  int64_t rows_per = ((n + S - 1) / S + kPK - 1) / kPK * kPK;
  S = (n + rows_per - 1) / rows_per;
  const int64_t len = (int64_t)p->T * kPTile;
  PENSURE(p->part, S * len);
  hipLaunchKernelGGL(pca_syrk_kernel, dim3((unsigned)(S * p->T)), dim3(256), 0, p->stream, X, ld, n, p->F, p->nb,
                     p->T, rows_per, p->part.p);
  PHIP(hipGetLastError());
  hipLaunchKernelGGL(pca_reduce_kernel, dim3(grid_for(len)), dim3(256), 0, p->stream, p->part.p, (int)S, len, acc.p);
  PHIP(hipGetLastError());
  return C3H_OK;
}

}  // namespace

extern "C" {

int c3h_pca_create(int hip_device, int32_t mean_flg, c3h_pca** out) {
  if (!out) return C3H_ERR_ARG;
  *out = nullptr;
  c3h_pca* p = new (std::nothrow) c3h_pca;
  if (!p) return C3H_ERR_NOMEM;
  p->device = hip_device;
  p->mean_flg = mean_flg != 0;
  if (hipSetDevice(hip_device) != hipSuccess ||
      hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete p;
    return C3H_ERR_HIP;
  }
  p->stream = p->own_stream;
  *out = p;
  return C3H_OK;
}

void c3h_pca_destroy(c3h_pca* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  if (p->blas) (void)g_solver.destroy(p->blas);
  release(p->acc_plain);
  release(p->acc_rot);
  release(p->part);
  release(p->C);
  release(p->msum);
  release(p->tmp);
  release(p->G);
  release(p->W);
  release(p->E);
  release(p->proj);
  release(p->maps);
  release(p->info);
  release(p->stage);
  release(p->out_axis);
  release(p->out_var);
  release(p->out_mean);
  if (p->own_stream) (void)hipStreamDestroy(p->own_stream);
  delete p;
}

const char* c3h_pca_last_error(c3h_pca* p) { return p ? p->err.c_str() : "null PCA handle"; }

int c3h_pca_set_stream(c3h_pca* p, void* hip_stream) {
  if (!p) return C3H_ERR_ARG;
  p->stream = hip_stream ? (hipStream_t)hip_stream : p->own_stream;
  return C3H_OK;
}

int c3h_pca_set_compress(c3h_pca* p, const float* axis, const float* var, int32_t F, int32_t D) {
  if (!p || !axis || F <= 0 || D <= 0 || D > F) return pfail(p, C3H_ERR_ARG, "set_compress: bad arguments");
  if (p->have_plain || p->have_rot) return pfail(p, C3H_ERR_STATE, "set_compress: data already added");
  if (p->F != -1 && p->F != F) return pfail(p, C3H_ERR_ARG, "set_compress: dimension differs");
  p->h_proj.assign((size_t)F * D, 0.0);
  for (int d = 0; d < D; ++d) {
    // compressFeature (pca_models.cpp:48-63): vec2(t) / sqrt(variance(t)), float sqrt
    const double s = var ? (double)sqrtf(var[d]) : 1.0;
    if (var && !(s > 0)) return pfail(p, C3H_ERR_ARG, "set_compress: non-positive variance");
    for (int f = 0; f < F; ++f) p->h_proj[(size_t)f * D + d] = (double)axis[(size_t)d * F + f] / s;
  }
  p->D = D;
  p->whiten = var != nullptr;
  p->solved = false;
  return C3H_OK;
}

int c3h_pca_add_data(c3h_pca* p, const float* rows, int64_t n, int64_t ld, int32_t F, int32_t rotate24,
                     int on_device) {
  if (!p || (!rows && n > 0) || n < 0 || F <= 0 || ld < F) return pfail(p, C3H_ERR_ARG, "add_data: bad arguments");
  if (p->F == -1) {
    if (p->D && (int)(p->h_proj.size() / p->D) != F) return pfail(p, C3H_ERR_ARG, "add_data: vector size differs");
    p->F = F;
    p->nb = (F + 1 + kPT - 1) / kPT;  // + the constant-1 column
    p->T = p->nb * (p->nb + 1) / 2;
  } else if (p->F != F) {
    return pfail(p, C3H_ERR_ARG, "add_data: vector size differs");  // pca.cpp:54-57
  }
  if (rotate24 && !rot_dim_ok(F))
    return pfail(p, C3H_ERR_ARG, "add_data: rotateFeature90: improper dimension");  // c3_hlac.cpp:166-170
  PHIP(hipSetDevice(p->device));
  DevBuf<double>& acc = rotate24 ? p->acc_rot : p->acc_plain;
  bool& have = rotate24 ? p->have_rot : p->have_plain;
  const int64_t len = (int64_t)p->T * kPTile;
  if (!have) {
    PENSURE(acc, len);
    PHIP(hipMemsetAsync(acc.p, 0, len * sizeof(double), p->stream));
    have = true;
  }
  if (on_device) {
    int rc = syrk_rows(p, rows, n, ld, acc);
    if (rc) return rc;
  } else {  // host rows: staged through HBM in chunks
    const int64_t chunk = std::max<int64_t>(1, ((int64_t)64 << 20) / ((int64_t)F * 4));
    PENSURE(p->stage, std::min(n, chunk) * F);
    for (int64_t r = 0; r < n; r += chunk) {
      const int64_t m = std::min(chunk, n - r);
      PHIP(hipMemcpy2DAsync(p->stage.p, F * sizeof(float), rows + r * ld, ld * sizeof(float), F * sizeof(float), m,
                            hipMemcpyHostToDevice, p->stream));
      int rc = syrk_rows(p, p->stage.p, m, F, acc);
      if (rc) return rc;
      PHIP(hipStreamSynchronize(p->stream));  // the staging buffer is reused
    }
  }
  p->nsample += n * (rotate24 ? kRot : 1);
  p->solved = false;
  return C3H_OK;
}

int c3h_pca_solve(c3h_pca* p, int32_t regularization_flg, float regularization_nolm) {
  if (!p) return C3H_ERR_ARG;
  if (p->F == -1 || p->nsample == 0) return pfail(p, C3H_ERR_STATE, "solve: there is no data");  // pca.cpp:74-77
  if (!solver_load()) return pfail(p, C3H_ERR_HIP, g_solver.err);
  PHIP(hipSetDevice(p->device));
  const int F = p->F, d = p->D ? p->D : F;
  // 1. raw correlation sums + mean sums (24 permuted copies for the rotated rows)
  PENSURE(p->C, (size_t)F * F);
  PENSURE(p->msum, F);
  if (p->have_rot && !p->maps.p) {
    const std::vector<int32_t> m = rot24_maps(F);
    PENSURE(p->maps, m.size());
    PHIP(hipMemcpy(p->maps.p, m.data(), m.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(pca_unpack_kernel, dim3(grid_for((int64_t)F * (F + 1))), dim3(256), 0, p->stream,
                     p->have_plain ? p->acc_plain.p : nullptr, p->have_rot ? p->acc_rot.p : nullptr, p->maps.p, F,
                     p->nb, p->C.p, p->msum.p);
  PHIP(hipGetLastError());
  // 2. compression: G = P^T C P, mean = P^T m  (P = axis / sqrt(var), F x D)
  double* Gp = p->C.p;
  double* mp = p->msum.p;
  PENSURE(p->G, (size_t)d * d);
  PENSURE(p->W, d + 1);
  PENSURE(p->E, d + 1);
  if (p->D) {
    PENSURE(p->proj, p->h_proj.size());
    PENSURE(p->tmp, (size_t)F * d);
    PHIP(hipMemcpyAsync(p->proj.p, p->h_proj.data(), p->h_proj.size() * sizeof(double), hipMemcpyHostToDevice,
                        p->stream));
    const dim3 b(256);
    hipLaunchKernelGGL(gemm_f64_kernel, dim3((d + 15) / 16, (F + 15) / 16), b, 0, p->stream, p->C.p, (int64_t)F,
                       (int64_t)1, p->proj.p, (int64_t)d, (int64_t)1, p->tmp.p, (int64_t)d, (int64_t)1, F, d, F);
    hipLaunchKernelGGL(gemm_f64_kernel, dim3((d + 15) / 16, (d + 15) / 16), b, 0, p->stream, p->proj.p, (int64_t)1,
                       (int64_t)d, p->tmp.p, (int64_t)d, (int64_t)1, p->G.p, (int64_t)d, (int64_t)1, d, d, F);
    hipLaunchKernelGGL(gemm_f64_kernel, dim3(1, (d + 15) / 16), b, 0, p->stream, p->proj.p, (int64_t)1, (int64_t)d,
                       p->msum.p, (int64_t)1, (int64_t)0, p->W.p, (int64_t)1, (int64_t)0, d, 1, F);
    PHIP(hipGetLastError());
    Gp = p->G.p;
    mp = p->W.p;
  } else {
    PHIP(hipMemcpyAsync(p->G.p, p->C.p, (size_t)F * F * sizeof(double), hipMemcpyDeviceToDevice, p->stream));
    PHIP(hipMemcpyAsync(p->W.p, p->msum.p, F * sizeof(double), hipMemcpyDeviceToDevice, p->stream));
    Gp = p->G.p;
    mp = p->W.p;
  }
  // 3. pca.cpp:80-98
  PENSURE(p->out_mean, d);
  const double inv_n = 1.0 / (double)p->nsample;
  hipLaunchKernelGGL(pca_finalize_kernel, dim3(grid_for((int64_t)d * d)), dim3(256), 0, p->stream, Gp, mp, d, inv_n,
                     (int)p->mean_flg, (int)(regularization_flg != 0), (double)regularization_nolm);
  PHIP(hipGetLastError());
  // the mean vector (kept in W's slot until the eigensolve overwrites W: copy it out first)
  hipLaunchKernelGGL(pca_scale_kernel, dim3((d + 255) / 256), dim3(256), 0, p->stream, mp, d, inv_n);
  PENSURE(p->tmp, std::max<size_t>(p->tmp.n, (size_t)d));
  PHIP(hipMemcpyAsync(p->tmp.p, mp, d * sizeof(double), hipMemcpyDeviceToDevice, p->stream));
  // keep the decomposed matrix for c3h_pca_get_correlation
  PENSURE(p->part, std::max<size_t>(p->part.n, (size_t)d * d));
  PHIP(hipMemcpyAsync(p->part.p, Gp, (size_t)d * d * sizeof(double), hipMemcpyDeviceToDevice, p->stream));
  // 4. eigensolve (ascending eigenvalues, vectors in the columns of Gp; symmetric input)
  if (!p->blas && g_solver.create(&p->blas) != rocblas_status_success) {
    p->blas = nullptr;
    return pfail(p, C3H_ERR_HIP, "rocblas_create_handle failed");
  }
  if (g_solver.set_stream(p->blas, p->stream) != rocblas_status_success)
    return pfail(p, C3H_ERR_HIP, "rocblas_set_stream failed");
  PENSURE(p->info, 1);
  if (g_solver.dsyevd(p->blas, rocblas_evect_original, rocblas_fill_upper, d, Gp, d, p->W.p, p->E.p, p->info.p) !=
      rocblas_status_success)
    return pfail(p, C3H_ERR_HIP, "rocsolver_dsyevd failed");
  // 5. sortVecAndVal + float outputs
  PENSURE(p->out_axis, (size_t)d * d);
  PENSURE(p->out_var, d);
  hipLaunchKernelGGL(pca_sort_kernel, dim3((d + 63) / 64), dim3(64), 0, p->stream, p->W.p, Gp, d, p->out_axis.p,
                     p->out_var.p);
  PHIP(hipGetLastError());
  std::vector<double> hm(d);
  int32_t info = 0;
  PHIP(hipMemcpyAsync(hm.data(), p->tmp.p, d * sizeof(double), hipMemcpyDeviceToHost, p->stream));
  PHIP(hipMemcpyAsync(&info, p->info.p, sizeof(int32_t), hipMemcpyDeviceToHost, p->stream));
  PHIP(hipStreamSynchronize(p->stream));
  if (info != 0) return pfail(p, C3H_ERR_HIP, "rocsolver_dsyevd did not converge");
  std::vector<float> hmf(d);
  for (int i = 0; i < d; ++i) hmf[i] = (float)hm[i];
  PHIP(hipMemcpy(p->out_mean.p, hmf.data(), d * sizeof(float), hipMemcpyHostToDevice));
  p->dim_out = d;
  p->solved = true;
  return C3H_OK;
}

int c3h_pca_get(c3h_pca* p, float* axis, float* var, float* mean, int64_t* nsample, int on_device) {
  if (!p) return C3H_ERR_ARG;
  if (!p->solved) return pfail(p, C3H_ERR_STATE, "get: solve() first");
  if (mean && !p->mean_flg) return pfail(p, C3H_ERR_STATE, "getMean: There is no mean vector (mean_flg=false)");
  const int d = p->dim_out;
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  PHIP(hipSetDevice(p->device));
  if (axis) PHIP(hipMemcpyAsync(axis, p->out_axis.p, (size_t)d * d * sizeof(float), k, p->stream));
  if (var) PHIP(hipMemcpyAsync(var, p->out_var.p, d * sizeof(float), k, p->stream));
  if (mean) PHIP(hipMemcpyAsync(mean, p->out_mean.p, d * sizeof(float), k, p->stream));
  PHIP(hipStreamSynchronize(p->stream));
  if (nsample) *nsample = p->nsample;
  return d;
}

int c3h_pca_get_correlation(c3h_pca* p, double* corr) {
  if (!p || !corr) return C3H_ERR_ARG;
  if (!p->solved) return pfail(p, C3H_ERR_STATE, "get_correlation: solve() first");
  const int d = p->dim_out;
  PHIP(hipSetDevice(p->device));
  PHIP(hipMemcpyAsync(corr, p->part.p, (size_t)d * d * sizeof(double), hipMemcpyDeviceToHost, p->stream));
  PHIP(hipStreamSynchronize(p->stream));
  return d;
}

int c3h_pca_write(const char* path, int32_t ascii, int32_t dim, const float* axis, const float* var,
                  const float* mean) {
  if (!path || dim <= 0 || !axis || !var) return C3H_ERR_ARG;
  FILE* fp = fopen(path, ascii ? "w" : "wb");
  if (!fp) return C3H_ERR_NOTFOUND;
  bool ok = true;
  if (ascii) {  // pca.cpp:200-218
    ok = fprintf(fp, "%d\n", dim) > 0;
    for (int i = 0; i < dim && ok; i++) {
      for (int j = 0; j < dim && ok; j++) ok = fprintf(fp, "%f ", axis[(size_t)i * dim + j]) > 0;
      ok = ok && fprintf(fp, "\n") > 0;
    }
    for (int i = 0; i < dim && ok; i++) ok = fprintf(fp, "%f\n", var[i]) > 0;
    if (mean)
      for (int i = 0; i < dim && ok; i++) ok = fprintf(fp, "%f\n", mean[i]) > 0;
  } else {  // pca.cpp:220-237
    ok = fwrite(&dim, sizeof(int), 1, fp) == 1 && fwrite(axis, sizeof(float), (size_t)dim * dim, fp) == (size_t)dim * dim &&
         fwrite(var, sizeof(float), dim, fp) == (size_t)dim && (!mean || fwrite(mean, sizeof(float), dim, fp) == (size_t)dim);
  }
  ok = (fclose(fp) == 0) && ok;
  return ok ? C3H_OK : C3H_ERR_FORMAT;
}

int c3h_rotate_map(int32_t dim, int32_t mode, int32_t* map_out) {
  if (!map_out || mode < 0 || mode > 3) return C3H_ERR_ARG;
  if (!rot_dim_ok(dim)) return C3H_ERR_ARG;
  const std::vector<int32_t> m = rot_map(dim, mode);
  std::memcpy(map_out, m.data(), m.size() * sizeof(int32_t));
  return C3H_OK;
}

int c3h_rotate_feature90(const float* in, float* out, int64_t n, int64_t ld, int32_t dim, int32_t mode,
                         void* hip_stream) {
  if (!in || !out || in == out || n < 0 || ld < dim || mode < 0 || mode > 3) return C3H_ERR_ARG;
  if (!rot_dim_ok(dim)) return C3H_ERR_ARG;  // c3_hlac.cpp:166-170
  if (n == 0) return C3H_OK;
  // the four maps of this dimension, resident per device (small and immutable)
  static std::mutex mu;
  static std::vector<std::pair<std::pair<int, int>, int32_t*>> cache;  // (device, dim) -> 4 maps
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return C3H_ERR_HIP;
  int32_t* maps = nullptr;
  {
    std::lock_guard<std::mutex> g(mu);
    for (auto& e : cache)
      if (e.first.first == dev && e.first.second == dim) maps = e.second;
    if (!maps) {
      std::vector<int32_t> all;
      for (int m = 0; m < 4; ++m) {
        const std::vector<int32_t> v = rot_map(dim, m);
        all.insert(all.end(), v.begin(), v.end());
      }
      if (hipMalloc(&maps, all.size() * sizeof(int32_t)) != hipSuccess) return C3H_ERR_NOMEM;
      if (hipMemcpy(maps, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess)
        return C3H_ERR_HIP;
      cache.push_back({{dev, dim}, maps});
    }
  }
  hipLaunchKernelGGL(rotate_kernel, dim3(grid_for(n * dim)), dim3(256), 0, (hipStream_t)hip_stream, in, out, n, ld,
                     dim, maps + (int64_t)mode * dim);
  return hipGetLastError() == hipSuccess ? C3H_OK : C3H_ERR_HIP;
}

}  // extern "C"
