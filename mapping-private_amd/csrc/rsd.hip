// rsd.hip -- normals, RSD radii and GRSD transition histograms on the GPU (SURVEY.md
// 8(f)4, the VOSCH / GRSD features of color_chlac/include/color_chlac/
// grsd_colorCHLAC_tools.hpp:63-296, 832-843).
//
// Radius searches run over a dense grid of cells of the normal radius: the points are
// sorted by cell (rocPRIM radix sort of (cell, point) pairs: stable, so a cell lists its
// points in input order) and every cell keeps its [start, end) range.  A query visits
// the cells within ceil(radius / cell) of its own.
//   normals_kernel: one point per thread; double sums of the neighbours within the
//     radius (the point included, squared distances in float as FLANN compares them);
//     covariance -> smallest-eigenvalue eigenvector (Jacobi, double), flipped towards
//     the viewpoint, curvature = lambda_min / trace; < 3 neighbours -> NaN (PCL).
//   rsd_kernel: one downsampled centroid per thread; PCL's computeRSD over the cloud
//     points within max(rsd_radius, leaf sqrt(3) / 2) of it: the nearest one is the
//     reference ("begin"), the others' normal angles are binned by their distance to it.
//   grsd_kernel: one occupied voxel per thread; its type against the 26 neighbour voxels
//     (EMPTY where unoccupied), int atomics into its subdivision's 6 x 6 matrix.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "c3h_internal.h"

namespace c3h {
namespace {

constexpr uint32_t kNoCell = 0xffffffffu;

__device__ __forceinline__ bool pt_finite(const float4& p) {
  return isfinite(p.x) && isfinite(p.y) && isfinite(p.z);
}

__device__ __forceinline__ bool cell_of(const NbrGrid& g, const float4& p, int c[3]) {
  const float v[3] = {p.x, p.y, p.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    const float t = floorf((v[a] - g.origin[a]) * g.inv_cell);
    if (!(t >= 0.0f && t < (float)g.dim[a])) return false;
    c[a] = (int)t;
  }
  return true;
}

__global__ void nbr_keys_kernel(NbrGrid g, uint32_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g.n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = g.pts[i];
    int c[3];
    keys[i] = pt_finite(p) && cell_of(g, p, c) ? (uint32_t)(c[0] + g.dim[0] * (c[1] + g.dim[1] * c[2])) : kNoCell;
    idx[i] = (uint32_t)i;
  }
}

__global__ void nbr_ranges_kernel(const uint32_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ cstart,
                                  uint32_t* __restrict__ cend) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    if (k == kNoCell) continue;
    if (i == 0 || keys[i - 1] != k) cstart[k] = (uint32_t)i;
    if (i == n - 1 || keys[i + 1] != k) cend[k] = (uint32_t)(i + 1);
  }
}

// visit every grid point within sqrt(r2) of q (float squared distance < r2, strict as
// FLANN's radius result set), in cell order then input order
template <class F>
__device__ __forceinline__ void for_neighbours(const NbrGrid& g, const float4& q, float r2, int reach, F&& f) {
  const float v[3] = {q.x, q.y, q.z};
  int c[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) c[a] = (int)floorf((v[a] - g.origin[a]) * g.inv_cell);
  for (int dz = -reach; dz <= reach; ++dz) {
    const int z = c[2] + dz;
    if (z < 0 || z >= g.dim[2]) continue;
    for (int dy = -reach; dy <= reach; ++dy) {
      const int y = c[1] + dy;
      if (y < 0 || y >= g.dim[1]) continue;
      for (int dx = -reach; dx <= reach; ++dx) {
        const int x = c[0] + dx;
        if (x < 0 || x >= g.dim[0]) continue;
        const uint32_t cell = (uint32_t)(x + g.dim[0] * (y + g.dim[1] * z));
        const uint32_t e = g.cend[cell];
        for (uint32_t s = g.cstart[cell]; s < e; ++s) {
          const uint32_t j = g.sorted[s];
          const float4 p = g.pts[j];
          const float ex = p.x - q.x, ey = p.y - q.y, ez = p.z - q.z;
          const float d2 = __fadd_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), __fmul_rn(ez, ez));
          if (d2 < r2) f(j, p, d2);
        }
      }
    }
  }
}

// eigen decomposition of a symmetric 3 x 3 matrix (cyclic Jacobi, double): w ascending,
// V columns the eigenvectors
__device__ void sym3_eigen(double A[3][3], double w[3], double V[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) V[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 32; ++sweep) {
    const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
    if (off == 0.0) break;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        if (A[p][q] == 0.0) continue;
        const double theta = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 3; ++k) {  // A = J^T A J
          const double akp = A[k][p], akq = A[k][q];
          A[k][p] = c * akp - s * akq;
          A[k][q] = s * akp + c * akq;
        }
        for (int k = 0; k < 3; ++k) {
          const double apk = A[p][k], aqk = A[q][k];
          A[p][k] = c * apk - s * aqk;
          A[q][k] = s * apk + c * aqk;
        }
        for (int k = 0; k < 3; ++k) {
          const double vkp = V[k][p], vkq = V[k][q];
          V[k][p] = c * vkp - s * vkq;
          V[k][q] = s * vkp + c * vkq;
        }
      }
  }
  int o[3] = {0, 1, 2};
  for (int i = 0; i < 3; ++i)
    for (int j = i + 1; j < 3; ++j)
      if (A[o[j]][o[j]] < A[o[i]][o[i]]) {
        const int t = o[i];
        o[i] = o[j];
        o[j] = t;
      }
  double W[3][3];
  for (int i = 0; i < 3; ++i) {
    w[i] = A[o[i]][o[i]];
    for (int k = 0; k < 3; ++k) W[k][i] = V[k][o[i]];
  }
  for (int i = 0; i < 3; ++i)
    for (int k = 0; k < 3; ++k) V[k][i] = W[k][i];
}

__global__ void normals_kernel(NbrGrid g, float r2, int reach, float vx, float vy, float vz,
                               float4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g.n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 q = g.pts[i];
    const float nan = __int_as_float(0x7fc00000);
    float4 res = make_float4(nan, nan, nan, nan);
    if (pt_finite(q)) {
      double s[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // n, x, y, z, xx, xy, xz, yy, yz, zz
      for_neighbours(g, q, r2, reach, [&](uint32_t, const float4& p, float) {
        const double x = p.x, y = p.y, z = p.z;
        s[0] += 1;
        s[1] += x;
        s[2] += y;
        s[3] += z;
        s[4] += x * x;
        s[5] += x * y;
        s[6] += x * z;
        s[7] += y * y;
        s[8] += y * z;
        s[9] += z * z;
      });
      if (s[0] >= 3) {
        const double n = s[0], mx = s[1] / n, my = s[2] / n, mz = s[3] / n;
        double A[3][3] = {{s[4] / n - mx * mx, s[5] / n - mx * my, s[6] / n - mx * mz},
                          {0, s[7] / n - my * my, s[8] / n - my * mz},
                          {0, 0, s[9] / n - mz * mz}};
        A[1][0] = A[0][1];
        A[2][0] = A[0][2];
        A[2][1] = A[1][2];
        double w[3], V[3][3];
        sym3_eigen(A, w, V);
        double nx = V[0][0], ny = V[1][0], nz = V[2][0];
        const double nl = sqrt(nx * nx + ny * ny + nz * nz);
        nx /= nl;
        ny /= nl;
        nz /= nl;
        // flipNormalTowardsViewpoint
        if ((vx - (double)q.x) * nx + (vy - (double)q.y) * ny + (vz - (double)q.z) * nz < 0) {
          nx = -nx;
          ny = -ny;
          nz = -nz;
        }
        const double tr = w[0] + w[1] + w[2];
        res = make_float4((float)nx, (float)ny, (float)nz, (float)(tr != 0 ? w[0] / tr : 0.0));
      }
    }
    out[i] = res;
  }
}

// grsd_colorCHLAC_tools.hpp:99-118
__device__ __forceinline__ int grsd_type(float rmin, float rmax) {
  if ((double)rmin > 0.100) return 1;  // PLANE
  if ((double)rmax > 0.175) return 2;  // CYLINDER
  if ((double)rmin < 0.015) return 0;  // NOISE
  if ((double)(rmax - rmin) < 0.050) return 3;  // SPHERE
  return 4;  // EDGE
}

constexpr int kRsdSubdiv = 5;  // RSDEstimation defaults: nr_subdiv 5, plane_radius 0.2

__global__ void rsd_kernel(NbrGrid g, const float4* __restrict__ nrm, const float4* __restrict__ cent,
                           int64_t nc, float max_dist, int reach, float2* __restrict__ radii,
                           int32_t* __restrict__ types) {
  const double kPi = 3.14159265358979323846;
  const float r2 = max_dist * max_dist;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nc; c += (int64_t)gridDim.x * blockDim.x) {
    const float4 q = cent[c];
    // the nearest neighbour (ties: the lower point index) and the neighbour count
    uint32_t best = 0xffffffffu;
    float bd = 0.0f;
    int cnt = 0;
    for_neighbours(g, q, r2, reach, [&](uint32_t j, const float4&, float d2) {
      ++cnt;
      if (best == 0xffffffffu || d2 < bd || (d2 == bd && j < best)) {
        best = j;
        bd = d2;
      }
    });
    float rmin = 0.0f, rmax = 0.0f;
    if (cnt >= 2) {
      double mn[kRsdSubdiv], mx[kRsdSubdiv];
      mn[0] = mx[0] = 0.0;
      for (int d = 1; d < kRsdSubdiv; ++d) {
        mn[d] = 1.7976931348623157e308;
        mx[d] = -1.7976931348623157e308;
      }
      const float4 pb = g.pts[best];
      const float4 nb = nrm[best];
      for_neighbours(g, q, r2, reach, [&](uint32_t j, const float4& p, float) {
        if (j == best) return;
        const float4 ni = nrm[j];
        double cosine = (double)__fadd_rn(__fadd_rn(__fmul_rn(ni.x, nb.x), __fmul_rn(ni.y, nb.y)), __fmul_rn(ni.z, nb.z));
        if (cosine > 1) cosine = 1;
        if (cosine < -1) cosine = -1;
        double angle = acos(cosine);
        if (angle > kPi / 2) angle = kPi - angle;
        const float ex = p.x - pb.x, ey = p.y - pb.y, ez = p.z - pb.z;
        const double dist = sqrt((double)__fadd_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey)), __fmul_rn(ez, ez)));
        if (dist > max_dist) return;
        int bin = (int)floor(kRsdSubdiv * dist / max_dist);
        if (bin > kRsdSubdiv - 1) bin = kRsdSubdiv - 1;
        if (mn[bin] > angle) mn[bin] = angle;
        if (mx[bin] < angle) mx[bin] = angle;
      });
      double aa = 0, ad = 0, xa = 0, xd = 0;
      for (int d = 0; d < kRsdSubdiv; ++d)
        if (mx[d] >= 0) {
          const double f = (d + 0.5) * max_dist / kRsdSubdiv;
          aa += mn[d] * mn[d];
          ad += mn[d] * f;
          xa += mx[d] * mx[d];
          xd += mx[d] * f;
        }
      const double plane = 0.2;
      float a = (float)(aa == 0 ? plane : fmin(ad / aa, plane));
      float b = (float)(xa == 0 ? plane : fmin(xd / xa, plane));
      a = (float)(a * 1.1);
      b = (float)(b * 0.9);
      rmin = a < b ? a : b;
      rmax = a < b ? b : a;
    }
    radii[c] = make_float2(rmin, rmax);
    types[c] = grsd_type(rmin, rmax);
  }
}

__global__ void grsd_kernel(GrsdArgs a) {
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < a.nc; c += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = a.cent[c];
    const float v[3] = {p.x, p.y, p.z};
    int64_t h = 0;
    if (a.hist1 == 0) {  // hist_idx (grsd_colorCHLAC_tools.hpp:245-258)
      int ijk[3];
      bool ok = true;
      for (int ax = 0; ax < 3; ++ax) {
        const int t = (int)floorf(__fdiv_rn(v[ax], a.leaf)) - a.min_b[ax] - a.off[ax];
        ok = ok && t >= 0;
        ijk[ax] = (int)floorf((float)t * a.inv_s);
        ok = ok && ijk[ax] < a.sb[ax];
      }
      if (!ok) continue;
      h = ijk[0] + (int64_t)a.sb[0] * (ijk[1] + (int64_t)a.sb[1] * ijk[2]);
    }
    const int src = a.types[c];
    int base[3];
    for (int ax = 0; ax < 3; ++ax) base[ax] = (int)floorf(v[ax] * a.inv_leaf) - a.min_b[ax];
    int32_t* T = a.trans + h * 36 + src * 6;
    for (int k = 0; k < 26; ++k) {  // relative_coordinates, then their negatives
      const int kk = k % 13, sg = k < 13 ? 1 : -1;
      const int rdx = kk <= 8 ? kk / 3 - 1 : (kk <= 11 ? kk - 10 : -1);
      const int rdy = kk <= 8 ? kk % 3 - 1 : (kk <= 11 ? -1 : 0);
      const int rdz = kk <= 8 ? -1 : 0;
      const int x = base[0] + sg * rdx, y = base[1] + sg * rdy, z = base[2] + sg * rdz;
      int nt = 5;  // EMPTY
      if (x >= 0 && y >= 0 && z >= 0 && x < a.div_b[0] && y < a.div_b[1] && z < a.div_b[2]) {
        const int32_t li = a.layout[x + (int64_t)a.div_b[0] * (y + (int64_t)a.div_b[1] * z)];
        if (li >= 0) nt = a.types[li];
      }
      atomicAdd(&T[nt], 1);
    }
  }
}

// upper-triangle bins (i <= j) of each 6 x 6 matrix, the first 20 (:277-283), times norm
__global__ void grsd_feat_kernel(const int32_t* __restrict__ trans, int64_t H, float norm, float* __restrict__ out,
                                 int stride) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < H * 20; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = e / 20;
    const int b = (int)(e - h * 20);
    int i = 0, j = 0, k = 0;
    for (i = 0; i < 6; ++i) {
      if (b < k + (6 - i)) {
        j = i + (b - k);
        break;
      }
      k += 6 - i;
    }
    out[h * stride + b] = (float)trans[h * 36 + i * 6 + j] * norm;
  }
}

// [grsd (20) | c3 (117)] rows; c3 rows of empty subdivisions may be stale: exist 0 -> zeros
__global__ void vosch_concat_kernel(const float* __restrict__ grsd, const float* __restrict__ c3,
                                    const int32_t* __restrict__ exist, int64_t H, float* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < H * 137; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t h = e / 137;
    const int t = (int)(e - h * 137);
    out[e] = t < 20 ? grsd[h * 20 + t] : (exist[h] ? c3[h * 117 + (t - 20)] : 0.0f);
  }
}

int grid_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192)); }

}  // namespace

hipError_t nbr_build(NbrGrid& g, uint32_t* keys, uint32_t* keys2, uint32_t* idx, uint32_t* idx2, void* tmp,
                     size_t* tmp_bytes, hipStream_t s) {
  if (!tmp) {  // size query
    size_t b = 0;
    const hipError_t e = rocprim::radix_sort_pairs(nullptr, b, keys, keys2, idx, idx2, (size_t)std::max<int64_t>(g.n, 1),
                                                   0, 32, s);
    *tmp_bytes = b;
    return e;
  }
  nbr_keys_kernel<<<grid_blocks(g.n), 256, 0, s>>>(g, keys, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t b = *tmp_bytes;
  e = rocprim::radix_sort_pairs(tmp, b, keys, keys2, idx, idx2, (size_t)g.n, 0, 32, s);
  if (e != hipSuccess) return e;
  const int64_t ncell = (int64_t)g.dim[0] * g.dim[1] * g.dim[2];
  e = hipMemsetAsync(const_cast<uint32_t*>(g.cstart), 0, ncell * 4, s);
  if (e == hipSuccess) e = hipMemsetAsync(const_cast<uint32_t*>(g.cend), 0, ncell * 4, s);
  if (e != hipSuccess) return e;
  nbr_ranges_kernel<<<grid_blocks(g.n), 256, 0, s>>>(keys2, g.n, const_cast<uint32_t*>(g.cstart),
                                                    const_cast<uint32_t*>(g.cend));
  g.sorted = idx2;
  return hipGetLastError();
}

hipError_t launch_normals(const NbrGrid& g, float radius, const float vp[3], float4* out, hipStream_t s) {
  const int reach = std::max(1, (int)ceilf(radius * g.inv_cell));
  normals_kernel<<<grid_blocks(g.n), 256, 0, s>>>(g, radius * radius, reach, vp[0], vp[1], vp[2], out);
  return hipGetLastError();
}

hipError_t launch_rsd(const NbrGrid& g, const float4* nrm, const float4* cent, int64_t nc, float max_dist, float2* radii,
                      int32_t* types, hipStream_t s) {
  if (nc == 0) return hipSuccess;
  const int reach = std::max(1, (int)ceilf(max_dist * g.inv_cell));
  rsd_kernel<<<grid_blocks(nc), 256, 0, s>>>(g, nrm, cent, nc, max_dist, reach, radii, types);
  return hipGetLastError();
}

hipError_t launch_grsd(const GrsdArgs& a, hipStream_t s) {
  if (a.nc > 0) grsd_kernel<<<grid_blocks(a.nc), 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_grsd_feat(const int32_t* trans, int64_t H, float norm, float* out, int stride, hipStream_t s) {
  if (H > 0) grsd_feat_kernel<<<grid_blocks(H * 20), 256, 0, s>>>(trans, H, norm, out, stride);
  return hipGetLastError();
}

hipError_t launch_vosch_concat(const float* grsd, const float* c3, const int32_t* exist, int64_t H, float* out,
                               hipStream_t s) {
  if (H > 0) vosch_concat_kernel<<<grid_blocks(H * 137), 256, 0, s>>>(grsd, c3, exist, H, out);
  return hipGetLastError();
}

}  // namespace c3h
