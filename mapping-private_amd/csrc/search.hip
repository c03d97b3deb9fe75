// search.hip -- sliding-box subspace search on gfx950.
//
// Replaces SearchObj{,Multi}::setData + searchPart (color_voxel_recognition/src/
// search.cpp:431-480, 539-658, 915-968).
//
// compress: G = f' * axis_p^T, an LDS-tiled fp32 GEMM (64 subdivisions x 128 dims per
//   workgroup, 4x8 register tile per thread, fma chain in ascending feature order);
//   setNormalizeVal's max-normalisation (search.cpp:563-570) is applied while loading.
// score: per sliding-box position, the occupied-voxel gate (exact integer box sum of
//   exist_voxel_num, = the reference's int summed-volume table), the box feature as a
//   direct sum of the box's subdivision vectors (no fp32 summed-volume differencing:
//   see DESIGN.md "A12"), then |Q_m f| / |f| per model with the reference's double
//   sqrt/divide.  Scores of gated-out positions are -1.
// replay: the order-dependent rank update with checkOverlap (search.cpp:327-376,
//   464-474) replayed exactly, one wave per model, scanning positions in the
//   reference's (mode, z, y, x) order; only candidates above the current rank-th score
//   (the lists only grow) are visited serially.
#include "c3h_internal.h"

namespace c3h {
namespace {

// ---------------------------------------------------------------- compress (GEMM)
constexpr int kCM = 64, kCN = 128, kCK = 16;

__global__ __launch_bounds__(kBlock) void compress_kernel(
    const float* __restrict__ feat, int64_t H, int F, const float* __restrict__ PT, int D,
    int Dpad, const float* __restrict__ fmax, int fmax_len, float* __restrict__ G) {
  __shared__ float fs[kCK][kCM + 4];
  __shared__ float ps[kCK][kCN];
  const int tid = threadIdx.x;
  const int th = tid & 15, td = tid >> 4;
  const int64_t h0 = blockIdx.x * (int64_t)kCM;
  const int d0 = blockIdx.y * kCN;
  float acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = 0.0f;

  for (int j0 = 0; j0 < F; j0 += kCK) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + kBlock * q, row = e >> 4, col = e & 15;
      const int64_t hh = h0 + row;
      const int jj = j0 + col;
      float v = 0.0f;
      if (hh < H && jj < F) {
        v = feat[hh * F + jj];
        if (jj < fmax_len) {  // SearchObj::setData histogram normalisation
          const float mx = fmax[jj];
          if (mx == 0.0f) v = 0.0f;
          else if (v == mx) v = 1.0f;
          else v = __fdiv_rn(v, mx);
        }
      }
      fs[col][row] = v;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = tid + kBlock * q, row = e >> 7, col = e & 127;
      ps[row][col] = (j0 + row < F && d0 + col < Dpad) ? PT[(int64_t)(j0 + row) * Dpad + d0 + col] : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kCK; ++kk) {
      float av[4], bv[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) av[i] = fs[kk][th * 4 + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = ps[kk][td * 8 + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t hh = h0 + th * 4 + i;
    if (hh >= H) continue;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int d = d0 + td * 8 + j;
      if (d < D) G[hh * D + d] = acc[i][j];
    }
  }
}

// ---------------------------------------------------------------- score
// SP positions per workgroup (64, or 16 when the box vectors are wide: no compression)
template <int SP>
__global__ __launch_bounds__(kBlock) void score_kernel(ScoreLaunch a, int64_t P) {
  extern __shared__ __attribute__((aligned(16))) float ssm[];
  const int DP = a.D + 1;
  float* fbox = ssm;                  // SP x DP
  float* qv = fbox + SP * DP;         // r x SP
  float* ffv = qv + a.r * SP;         // SP
  int* gate = reinterpret_cast<int*>(ffv + SP);  // SP
  const int tid = threadIdx.x;
  const int64_t p0 = blockIdx.x * (int64_t)SP;
  const int xyn = a.xn * a.yn;

  if (tid < SP) {
    const int64_t p = p0 + tid;
    int ok = 0;
    if (p < P) {
      const int x = (int)(p % a.xe), y = (int)((p / a.xe) % a.ye), z = (int)(p / ((int64_t)a.xe * a.ye));
      int e = 0;
      for (int dz = 0; dz < a.zr; ++dz)
        for (int dy = 0; dy < a.yr; ++dy)
          for (int dx = 0; dx < a.xr; ++dx) e += a.exist[(z + dz) * xyn + (y + dy) * a.xn + x + dx];
      ok = e > a.thr;
    }
    gate[tid] = ok;
  }
  __syncthreads();
  for (int idx = tid; idx < SP * a.D; idx += kBlock) {
    const int pp = idx / a.D, d = idx - pp * a.D;
    float s = 0.0f;
    if (gate[pp]) {
      const int64_t p = p0 + pp;
      const int x = (int)(p % a.xe), y = (int)((p / a.xe) % a.ye), z = (int)(p / ((int64_t)a.xe * a.ye));
      for (int dz = 0; dz < a.zr; ++dz)
        for (int dy = 0; dy < a.yr; ++dy)
          for (int dx = 0; dx < a.xr; ++dx)
            s += a.G[(int64_t)((z + dz) * xyn + (y + dy) * a.xn + x + dx) * a.D + d];
    }
    fbox[pp * DP + d] = s;
  }
  __syncthreads();
  if (tid < SP) {
    float s = 0.0f;
    for (int d = 0; d < a.D; ++d) s = __builtin_fmaf(fbox[tid * DP + d], fbox[tid * DP + d], s);
    ffv[tid] = s;
  }
  constexpr int kRowsPerPass = kBlock / SP;
  const int pp = tid & (SP - 1);
  // wave-uniform model row -> the basis is read through the scalar cache
  const int i0 = __builtin_amdgcn_readfirstlane(tid / SP);
  for (int m = 0; m < a.M; ++m) {
    const float* __restrict__ Q = a.axis_q + (int64_t)m * a.r * a.D;
    for (int i = i0; i < a.r; i += kRowsPerPass) {
      float t = 0.0f;
      const float* qrow = Q + (int64_t)i * a.D;
      const float* frow = fbox + pp * DP;
      for (int d = 0; d < a.D; ++d) t = __builtin_fmaf(qrow[d], frow[d], t);
      qv[i * SP + pp] = t;
    }
    __syncthreads();
    if (tid < SP) {
      const int64_t p = p0 + tid;
      if (p < P) {
        double sc = -1.0;
        if (gate[tid]) {
          float q2 = 0.0f;
          for (int i = 0; i < a.r; ++i) q2 = __builtin_fmaf(qv[i * SP + tid], qv[i * SP + tid], q2);
          sc = sqrt((double)q2) / sqrt((double)ffv[tid]);
        }
        a.scores[(int64_t)m * P + p] = sc;
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- rank replay
__device__ __forceinline__ void get_range(int mode, int r1, int r2, int r3, int& xr, int& yr,
                                          int& zr) {
  switch (mode) {  // search.cpp:218-251
    case 0: xr = r1; yr = r2; zr = r3; break;
    case 1: xr = r1; yr = r3; zr = r2; break;
    case 2: xr = r2; yr = r1; zr = r3; break;
    case 3: xr = r2; yr = r3; zr = r1; break;
    case 4: xr = r3; yr = r1; zr = r2; break;
    default: xr = r3; yr = r2; zr = r1; break;
  }
}

__global__ __launch_bounds__(64) void replay_kernel(const double* __restrict__ scores,
                                                    ReplayModes modes, int rank, int r1,
                                                    int r2, int r3,
                                                    c3h_det* __restrict__ lists) {
  extern __shared__ __attribute__((aligned(16))) c3h_det L[];
  const int m = blockIdx.x, lane = threadIdx.x;
  c3h_det* gl = lists + (int64_t)m * rank;
  for (int i = lane; i < rank; i += 64) L[i] = gl[i];
  __syncthreads();
  for (int mi = 0; mi < modes.n; ++mi) {
    const ReplayMode md = modes.m[mi];
    int xr, yr, zr;
    get_range(md.mode, r1, r2, r3, xr, yr, zr);
    const double* sc = scores + md.offset + (int64_t)m * md.P;
    for (int64_t base = 0; base < md.P; base += 64) {
      const int64_t p = base + lane;
      const double s = p < md.P ? sc[p] : -1.0;
      double T = L[rank - 1].score;
      unsigned long long mask = __ballot(s > T);
      while (mask) {
        const int j = __ffsll((long long)mask) - 1;
        const double cs = __shfl(s, j, 64);
        if (lane == 0) {
          const int64_t pc = base + j;
          const int x = (int)(pc % md.xe), y = (int)((pc / md.xe) % md.ye),
                    z = (int)(pc / ((int64_t)md.xe * md.ye));
          for (int i = 0; i < rank; i++) {
            if (cs > L[i].score) {
              // checkOverlap (search.cpp:327-356)
              int num;
              for (num = 0; num < rank - 1; num++) {
                int oxr, oyr, ozr;
                get_range(L[num].mode, r1, r2, r3, oxr, oyr, ozr);
                int v1 = L[num].x - x;
                v1 = v1 < 0 ? -v1 - oxr : v1 - xr;
                int v2 = L[num].y - y;
                v2 = v2 < 0 ? -v2 - oyr : v2 - yr;
                int v3 = L[num].z - z;
                v3 = v3 < 0 ? -v3 - ozr : v3 - zr;
                if (v1 <= 0 && v2 <= 0 && v3 <= 0) break;
              }
              for (int q = 0; q < num - i; q++) L[num - q] = L[num - 1 - q];
              if (i <= num) {
                L[i].score = cs;
                L[i].x = x;
                L[i].y = y;
                L[i].z = z;
                L[i].mode = md.mode;
              }
              break;
            }
          }
        }
        __syncthreads();
        T = L[rank - 1].score;
        const unsigned long long later = j >= 63 ? 0ull : (~0ull << (j + 1));
        mask = __ballot(s > T) & later;
      }
    }
  }
  __syncthreads();
  for (int i = lane; i < rank; i += 64) gl[i] = L[i];
}

// cleanMax on the device copy of the lists: score and x,y,z to 0, modes kept
__global__ void clean_lists_kernel(c3h_det* __restrict__ L, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    L[i].score = 0.0;
    L[i].x = 0;
    L[i].y = 0;
    L[i].z = 0;
  }
}

}  // namespace

hipError_t launch_clean_lists(c3h_det* lists, int n, hipStream_t s) {
  clean_lists_kernel<<<(n + 255) / 256, 256, 0, s>>>(lists, n);
  return hipGetLastError();
}

hipError_t launch_compress(const float* feat, int64_t H, int F, const float* axis_pt, int D,
                           int Dpad, const float* fmax, int fmax_len, float* G, hipStream_t s) {
  dim3 grid((unsigned)((H + kCM - 1) / kCM), (unsigned)((Dpad + kCN - 1) / kCN));
  compress_kernel<<<grid, kBlock, 0, s>>>(feat, H, F, axis_pt, D, Dpad, fmax, fmax_len, G);
  return hipGetLastError();
}

size_t score_lds_bytes(int D, int r, int SP) {
  return sizeof(float) * ((size_t)SP * (D + 1) + (size_t)r * SP + SP) + sizeof(int) * SP;
}

hipError_t launch_score(const ScoreLaunch& a, hipStream_t s) {
  const int64_t P = (int64_t)a.xe * a.ye * a.ze;
  if (P <= 0) return hipSuccess;
  if (a.D <= 256) {
    score_kernel<64><<<(unsigned)((P + 63) / 64), kBlock, score_lds_bytes(a.D, a.r, 64), s>>>(a, P);
  } else {
    score_kernel<16><<<(unsigned)((P + 15) / 16), kBlock, score_lds_bytes(a.D, a.r, 16), s>>>(a, P);
  }
  return hipGetLastError();
}

hipError_t launch_replay(const double* scores, const ReplayModes& modes, int M, int rank,
                         int r1, int r2, int r3, c3h_det* lists, hipStream_t s) {
  replay_kernel<<<M, 64, sizeof(c3h_det) * rank, s>>>(scores, modes, rank, r1, r2, r3, lists);
  return hipGetLastError();
}

}  // namespace c3h
