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
#include "search_dev.h"

namespace c3h {
namespace {

// ---------------------------------------------------------------- compress (GEMM)
// G[h][d] = sum_j f'[h][j] * P[j][d] (P = whitened axis_p transposed, F x Dpad).
// 512-thread block: 64 rows x 128 columns; lane = row (f staged k-major in LDS, read
// conflict-free), wave = 16 columns whose P values are wave-uniform scalar loads.
// fma chain in ascending j (the reference's GEMV order).
constexpr int kCM = 64, kCN = 128, kCK = 128, kCT = 512, kCW = 16;

__global__ __launch_bounds__(kCT) void compress_kernel(
    const float* __restrict__ feat, int64_t H, int F, const float* __restrict__ PT, int D,
    int Dpad, const float* __restrict__ fmax, int fmax_len, float* __restrict__ G,
    const int32_t* __restrict__ rows, const uint32_t* __restrict__ nrows,
    const int32_t* __restrict__ exist) {
  __shared__ float fs[kCK * (kCM + 1)];
  __shared__ int64_t s_row[kCM];
  const int tid = threadIdx.x;
  const int row = tid & (kCM - 1);
  const int cg = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t h0 = blockIdx.x * (int64_t)kCM;
  // sparse mode: this block's rows are rows[h0 .. h0+63] of the non-empty-row list
  // (G rows of empty subdivisions are left untouched; consumers gate them on exist)
  const int64_t nr = rows ? (int64_t)*nrows : H;
  if (h0 >= nr) return;
  if (tid < kCM) s_row[tid] = h0 + tid < nr ? (rows ? (int64_t)rows[h0 + tid] : h0 + tid) : -1;
  __syncthreads();
  const int c0 = blockIdx.y * kCN + cg * kCW;
  const bool active = c0 < D;
  float acc[kCW];
#pragma unroll
  for (int j = 0; j < kCW; ++j) acc[j] = 0.0f;
  for (int j0 = 0; j0 < F; j0 += kCK) {
    const int kn = min(kCK, F - j0);
    int r = tid / kn, c = tid - (tid / kn) * kn;  // e = tid + kCT*i -> (r, c), no division in the loop
    const int sr = kCT / kn, sc = kCT - (kCT / kn) * kn;
    for (int e = tid; e < kCM * kn; e += kCT) {
      const int64_t hh = s_row[r];
      const int jj = j0 + c;
      float v = 0.0f;
      // exist gate (sparse features: rows of empty subdivisions are stale, their true
      // value is 0, which is what an ungated zero row would give)
      if (hh >= 0 && (!exist || exist[hh])) {
        v = feat[hh * F + jj];
        if (jj < fmax_len) {  // SearchObj::setData histogram normalisation (search.cpp:563-570)
          const float mx = fmax[jj];
          if (mx == 0.0f) v = 0.0f;
          else if (v == mx) v = 1.0f;
          else v = __fdiv_rn(v, mx);
        }
      }
      fs[c * (kCM + 1) + r] = v;
      r += sr;
      c += sc;
      if (c >= kn) {
        c -= kn;
        ++r;
      }
    }
    __syncthreads();
    if (active) {
      const float* __restrict__ pk = PT + (int64_t)j0 * Dpad + c0;
      for (int k = 0; k < kn; ++k) {
        const float fv = fs[k * (kCM + 1) + row];
        const float* __restrict__ p = pk + (int64_t)k * Dpad;
#pragma unroll
        for (int j = 0; j < kCW; ++j) acc[j] = __builtin_fmaf(fv, p[j], acc[j]);
      }
    }
    __syncthreads();
  }
  const int64_t hh = s_row[row];
  if (active && hh >= 0) {
#pragma unroll
    for (int j = 0; j < kCW; ++j)
      if (c0 + j < D) G[hh * D + c0 + j] = acc[j];
  }
}

__global__ __launch_bounds__(kBlock) void compress_rows_kernel(CompressRows cr) {
  extern __shared__ __attribute__((aligned(16))) float crk_smem[];
  compress_rows_body(cr, blockIdx.x, gridDim.x, blockIdx.y, crk_smem);
}

// ---------------------------------------------------------------- score
// Generic path (any D, any M*r): SP positions per workgroup, basis through the scalar path.
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

__global__ __launch_bounds__(kBlock) void gate_kernel(SparseSearch b) {
  gate_body(b, blockIdx.x, blockIdx.y);
}

// one launch for two independent stages: gate workgroups first, then the sparse compress
__global__ __launch_bounds__(kBlock) void compress_gate_kernel(CompressRows cr, SparseSearch b, int ngate) {
  extern __shared__ __attribute__((aligned(16))) float cg_smem[];
  if ((int)blockIdx.x < ngate) gate_body(b, blockIdx.x, blockIdx.y);
  else compress_rows_body(cr, blockIdx.x - ngate, gridDim.x - ngate, blockIdx.y, cg_smem);
}

__global__ __launch_bounds__(kBlock, 3) void compress_f32c_kernel(CompressRows cr) {
  extern __shared__ __attribute__((aligned(16))) float cc_smem[];
  compress_f32c_body(cr, blockIdx.x, gridDim.x, blockIdx.y, cc_smem);
}

__global__ __launch_bounds__(kBlock, 3) void compress_f16_kernel(CompressRows cr, const _Float16* PT16, int Fp16) {
  __shared__ __attribute__((aligned(16))) _Float16 cf_smem[kCFLds / 2];
  if (cr.feat16 && *cr.feat16_flag)  // uniform: the extract wrote f16 rows
    compress_f16_body<true>(cr, PT16, Fp16, blockIdx.x, gridDim.x, blockIdx.y, cf_smem);
  else
    compress_f16_body<false>(cr, PT16, Fp16, blockIdx.x, gridDim.x, blockIdx.y, cf_smem);
}

__global__ __launch_bounds__(kBlock) void boxsum_kernel(SparseSearch a) {
  const int64_t n = a.pstart[a.nmodes] * (a.D >> 2);
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kBlock)
    boxsum_body(a, e, blockIdx.y);
}

// ---------------------------------------------------------------- score on the matrix cores
// SearchObjMulti::searchPart's projections (search.cpp:915-968) for the listed positions
// of one frame as a GEMM: Q = B * qt, B = the box-summed G rows (boxsum_kernel, P x D),
// qt = the models' basis rows (D x M*r).  Workgroup = 128 listed positions (32 per wave:
// the wave's A fragment, D/2 k-pairs, lives in registers for the whole column sweep) x the
// columns of one model group [m0*r, m1*r), swept in chunks of 32 columns staged in LDS
// (double-buffered, prefetched one chunk ahead in registers); one
// v_mfma_f32_32x32x2_f32 per k-pair.  The MFMA is bit-for-bit the k-ordered fmaf chain
// (compress_mfma_body), so every q is the VALU kernels' q.  Epilogue per chunk: the 32x32
// tile goes to a per-wave LDS scratch and lane p (< 32) folds its position's row in
// column order into |Q_m f|^2 (the fmaf chain over i = 0..r-1 of score_list_body),
// finishing model m at its last column: sqrt(q2)/sqrt(f.f) in double, as the reference.
constexpr int kSMP = 128;  // listed positions per workgroup
constexpr int kSMC = 32;   // basis columns per chunk
constexpr int kSMES = 33;  // epilogue scratch row stride (conflict-free row reads)

__host__ __device__ constexpr size_t score_mfma_lds_bytes(int KP) {
  return sizeof(float) * (2 * (size_t)(2 * KP) * kSMC + (size_t)(kBlock / 64) * 32 * kSMES) + 3 * 6 * sizeof(int64_t);
}

#ifndef C3H_SMF_WAVES
#define C3H_SMF_WAVES 3  // waves per SIMD the registers must allow (LDS: 3 workgroups per CU)
#endif
#ifndef C3H_SMF_GROUP
#define C3H_SMF_GROUP 16
#endif
constexpr int kSMG = C3H_SMF_GROUP;  // k-pairs whose B fragments are in registers together
template <int KP>  // k-pairs (D <= 2 KP), KP % 4 == 0
__global__ __launch_bounds__(kBlock, C3H_SMF_WAVES) void score_mfma_kernel(SparseSearch a, int ngroups) {
  extern __shared__ __attribute__((aligned(16))) float smf[];
  constexpr int K2 = 2 * KP;
  constexpr int kBE = K2 * kSMC / kBlock;  // B-chunk elements per thread
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hk = lane >> 5, l32 = lane & 31;
  float* se = smf + 2 * K2 * kSMC + wave * 32 * kSMES;
  // the mode table (pstart, score offset, P) in LDS: indexed per lane by the entry's mode
  int64_t* s_mode = reinterpret_cast<int64_t*>(smf + 2 * K2 * kSMC + (kBlock / 64) * 32 * kSMES);
  if (tid < a.nmodes) {
    s_mode[3 * tid] = a.pstart[tid];
    s_mode[3 * tid + 1] = a.md[tid].offset;
    s_mode[3 * tid + 2] = a.md[tid].P;
  }
  __syncthreads();
  const int D = a.D, r = a.r, Qs = a.Opad;
  const int n = (int)a.cnt[a.epoch & 1];
  const int g = blockIdx.y;
  const int m0 = (int)((int64_t)g * a.M / ngroups), m1 = (int)((int64_t)(g + 1) * a.M / ngroups);
  const int cb = m0 * r, ce = m1 * r;
  const int nch = (ce - cb + kSMC - 1) / kSMC;
  for (int pb = blockIdx.x; pb * kSMP < n; pb += gridDim.x) {
    const int e = pb * kSMP + wave * 32 + l32;
    const bool valid = e < n;
    const long long en = valid ? a.list[e] : 0;
    const int mi = (int)(en >> 40);
    const int64_t p = en & ((1ll << 40) - 1);
    // no per-lane masks (they would live in SGPR pairs): entries past the count read row 0
    // and are never stored; k-pairs past D (D even: a wave-uniform test) are zero
    const float* __restrict__ row = a.gbox + (valid ? (s_mode[3 * mi] + p) * D : 0);
    float av[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) av[j] = 2 * j < D ? row[2 * j + hk] : 0.0f;
    // f.f in ascending d (lane p holds the even k of its row, lane p + 32 the odd one)
    float ff = 0.0f;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      const float odd = __shfl(av[j], l32 + 32, 64);
      if (2 * j < D) ff = __builtin_fmaf(av[j], av[j], ff);
      if (2 * j + 1 < D) ff = __builtin_fmaf(odd, odd, ff);
    }
    const int64_t sbase = s_mode[3 * mi + 1] + p, sP = s_mode[3 * mi + 2];
    float bl[kBE];
    auto load_b = [&](int c) {
      const int col0 = cb + c * kSMC;
#pragma unroll
      for (int i = 0; i < kBE; ++i) {
        // clamped, not masked: rows past D meet A = 0, columns past the group are never
        // folded (qt is finite everywhere)
        const int el = tid + i * kBlock, k = min(el / kSMC, D - 1), col = min(col0 + (el % kSMC), Qs - 1);
        bl[i] = a.qt[(int64_t)k * Qs + col];
      }
    };
    load_b(0);
    float q2 = 0.0f;
    int m = m0, ir = 0;  // model and basis row of the next folded column (wave-uniform)
    for (int c = 0; c < nch; ++c) {
      float* sb = smf + (c & 1) * K2 * kSMC;
#pragma unroll
      for (int i = 0; i < kBE; ++i) sb[tid + i * kBlock] = bl[i];
      if (c + 1 < nch) load_b(c + 1);
      __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      mf_f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
      const float* bcol = sb + hk * kSMC + l32;
      // k-pairs in groups of kSMG: the group's B fragments are read (LDS) while the previous
      // group's MFMAs run, and no more than a group's are held in registers
#pragma unroll
      for (int j0 = 0; j0 < KP; j0 += kSMG) {
#pragma unroll
        for (int j = j0; j < j0 + kSMG && j < KP; ++j)
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[j], bcol[2 * j * kSMC], acc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // C/D map: column l32, row (q & 3) + 8 (q >> 2) + 4 hk
#pragma unroll
      for (int q = 0; q < 16; ++q) se[((q & 3) + 8 * (q >> 2) + 4 * hk) * kSMES + l32] = acc[q];
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int ncol = min(kSMC, ce - (cb + c * kSMC));
      if (hk == 0) {
        // the row's 32 reads issued together (one LDS round trip, not 32 dependent ones),
        // then the fold over registers
        const float* qrow = se + l32 * kSMES;
#pragma unroll
        for (int h0 = 0; h0 < kSMC; h0 += 16) {
          float qv[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) qv[j] = qrow[h0 + j];
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            if (h0 + j < ncol) {  // uniform (no break: the loop must unroll, qv stays in registers)
              q2 = __builtin_fmaf(qv[j], qv[j], q2);
              if (++ir == r) {  // model m complete
                if (valid) a.scores[sbase + (int64_t)m * sP] = sqrt((double)q2) / sqrt((double)ff);
                q2 = 0.0f;
                ir = 0;
                ++m;
              }
            }
          }
        }
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // scratch reads before the next tile's writes
    }
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // B buffers reused by the next block
  }
}

template <int KP>
hipError_t launch_score_mfma_kp(const SparseSearch& a, hipStream_t s) {
  static thread_local int slots = 0, dev_c = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const size_t lds = score_mfma_lds_bytes(KP);
  if (dev != dev_c) {
    int n_cu = 256, per_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, score_mfma_kernel<KP>, kBlock, lds) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    slots = per_cu * n_cu;
    dev_c = dev;
  }
  // the list count is on the device: size for every position passing (dense grids), the
  // workgroups past the count exit at once; model groups fill the chip when positions
  // alone would not (whole models per group: |Q_m f|^2 never spans workgroups)
  // Model groups: the launch takes ~ rounds of resident workgroups x a workgroup's time,
  // which is a fixed part (its positions' box rows into registers, f.f: ~3 column chunks of
  // matrix work, measured) plus one unit per 32-column chunk of its group's models
  const int64_t pblocks = (a.pstart[a.nmodes] + kSMP - 1) / kSMP;
  int ng = 1;
  double best = 1e300;
  for (int g = 1; g <= a.M; ++g) {
    const int64_t rounds = (pblocks * g + slots - 1) / slots;
    const int64_t cols = (int64_t)((a.M + g - 1) / g) * a.r;
    const double t = (double)rounds * (3.0 + (double)((cols + kSMC - 1) / kSMC));
    if (t < best) {
      best = t;
      ng = g;
    }
  }
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(pblocks, 65535));
  score_mfma_kernel<KP><<<dim3(gx, (unsigned)ng), kBlock, lds, s>>>(a, ng);
  return hipGetLastError();
}

hipError_t launch_score_mfma(const SparseSearch& a, hipStream_t s) {
  const int kp = (a.D + 1) / 2;
  if (kp <= 16) return launch_score_mfma_kp<16>(a, s);
  if (kp <= 24) return launch_score_mfma_kp<24>(a, s);
  if (kp <= 32) return launch_score_mfma_kp<32>(a, s);
  if (kp <= 40) return launch_score_mfma_kp<40>(a, s);
  if (kp <= 52) return launch_score_mfma_kp<52>(a, s);
  if (kp <= 64) return launch_score_mfma_kp<64>(a, s);
  if (kp <= 72) return launch_score_mfma_kp<72>(a, s);
  if (kp <= 80) return launch_score_mfma_kp<80>(a, s);
  return hipErrorInvalidValue;
}

// fp16 search precision (c3h_set_search_precision(ctx, 1)): the same projection with f16
// operands on v_mfma_f32_32x32x16_f16 (f32 accumulation, 16x the f32 matrix rate).  The
// score |Q f| / |f| is invariant to scaling f, so each position's box row is scaled by a
// power of two that puts its largest element in [0.5, 1) before rounding to f16 (exact
// scaling: no overflow, full f16 precision), and f.f is taken over the same rounded values.
// The basis is f16 too (qt16, [column][16 * Kq16]); each wave reads its B fragments straight
// from L2 (16 B per lane per k step, one tile ahead) -- no LDS staging, no barriers.  Stated
// tolerance with the fp16 compress: 2e-3 relative of the float64 oracle.
template <int KQ>  // 16-wide k steps
__global__ __launch_bounds__(kBlock, 3) void score_mfma_f16_kernel(SparseSearch a, int ngroups) {
  extern __shared__ __attribute__((aligned(16))) float smh[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hk = lane >> 5, l32 = lane & 31;
  float* se = smh + wave * 32 * kSMES;
  int64_t* s_mode = reinterpret_cast<int64_t*>(smh + (kBlock / 64) * 32 * kSMES);
  if (tid < a.nmodes) {
    s_mode[3 * tid] = a.pstart[tid];
    s_mode[3 * tid + 1] = a.md[tid].offset;
    s_mode[3 * tid + 2] = a.md[tid].P;
  }
  __syncthreads();
  constexpr int KH = 16 * KQ;
  const int D = a.D, r = a.r, Qs = a.Opad;
  const int n = (int)a.cnt[a.epoch & 1];
  const int g = blockIdx.y;
  const int m0 = (int)((int64_t)g * a.M / ngroups), m1 = (int)((int64_t)(g + 1) * a.M / ngroups);
  const int cb = m0 * r, ce = m1 * r;
  const int ntile = (ce - cb + 31) / 32;
  for (int pb = blockIdx.x; pb * kSMP < n; pb += gridDim.x) {
    const int e = pb * kSMP + wave * 32 + l32;
    const bool valid = e < n;
    const long long en = valid ? a.list[e] : 0;
    const int mi = (int)(en >> 40);
    const int64_t p = en & ((1ll << 40) - 1);
    const float* __restrict__ row = a.gbox + (valid ? (s_mode[3 * mi] + p) * D : 0);
    float v[KQ][8];
    float mx = 0.0f;
#pragma unroll
    for (int s = 0; s < KQ; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + 8 * hk + j;
        const float x = row[min(k, D - 1)];
        v[s][j] = k < D ? x : 0.0f;
        mx = fmaxf(mx, fabsf(v[s][j]));
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    int ex = 0;
    (void)frexpf(mx, &ex);  // mx = m * 2^ex, m in [0.5, 1) (ex = 0 for a zero row)
    mf_f16x8 av[KQ];
    float ff = 0.0f;
#pragma unroll
    for (int s = 0; s < KQ; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)ldexpf(v[s][j], -ex);
        av[s][j] = h;
        ff = __builtin_fmaf((float)h, (float)h, ff);
      }
    ff += __shfl_xor(ff, 32, 64);  // this lane's k and its partner's (a + b == b + a)
    const int64_t sbase = s_mode[3 * mi + 1] + p, sP = s_mode[3 * mi + 2];
    auto load_b = [&](int t, mf_f16x8 (&dst)[KQ]) {
      const int col = min(cb + 32 * t + l32, Qs - 1);  // clamped: columns past the group are never folded
#pragma unroll
      for (int s = 0; s < KQ; ++s)
        dst[s] = *reinterpret_cast<const mf_f16x8*>(a.qt16 + (int64_t)col * KH + 16 * s + 8 * hk);
    };
    mf_f16x8 bcur[KQ];
    load_b(0, bcur);
    float q2 = 0.0f;
    int m = m0, ir = 0;
    for (int t = 0; t < ntile; ++t) {
      mf_f16x8 bnxt[KQ];
      if (t + 1 < ntile) load_b(t + 1, bnxt);
      mf_f32x16 acc;
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] = 0.0f;
#pragma unroll
      for (int s = 0; s < KQ; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av[s], bcur[s], acc, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < 16; ++q) se[((q & 3) + 8 * (q >> 2) + 4 * hk) * kSMES + l32] = acc[q];
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int ncol = min(32, ce - (cb + 32 * t));
      if (hk == 0) {
        const float* qrow = se + l32 * kSMES;
#pragma unroll
        for (int h0 = 0; h0 < 32; h0 += 16) {
          float qv[16];
#pragma unroll
          for (int j = 0; j < 16; ++j) qv[j] = qrow[h0 + j];
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            if (h0 + j < ncol) {  // uniform
              q2 = __builtin_fmaf(qv[j], qv[j], q2);
              if (++ir == r) {
                if (valid) a.scores[sbase + (int64_t)m * sP] = sqrt((double)q2) / sqrt((double)ff);
                q2 = 0.0f;
                ir = 0;
                ++m;
              }
            }
          }
        }
      }
      __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 1 < ntile) {
#pragma unroll
        for (int s = 0; s < KQ; ++s) bcur[s] = bnxt[s];
      }
    }
  }
}

// fp16 projection for models of r >= 16 (a 32-column tile then meets at most 3 models),
// basis-stationary: a workgroup of 8 waves holds one model group's whole f16 basis in LDS
// (loaded once; the host picks the fewest groups whose columns fit, 63 x r = 70 -> 7 groups
// of 9 models, 145 KB) and streams listed positions through it, 32 per wave at a time
// (their f16 rows in registers, the next set's rows loaded during this set's sweep).  Each
// model's columns are padded to rp = r rounded up to 4 with zero basis rows, so the four
// consecutive columns a lane holds per accumulator quad always belong to one model: the
// epilogue is branch-free per lane (uniform branch on whether a model ends in the tile).
// Per 32-column tile: KQ ds_read_b128 of B fragments (column stride 2 KH + 16 bytes: the
// 16 lanes of a read hit distinct banks) and KQ MFMAs formed transposed (rows = basis
// columns, columns = positions), so lane (l32, hk) holds position l32's products with
// columns (q & 3) + 8 (q >> 2) + 4 hk; their squares accumulate per lane and the two lane
// halves are combined with one exchange when a model completes.  No global traffic in the
// sweep but the score stores, no barrier after the basis load.
// x + the same variable of lane ^ 32 (one v_permlane32_swap: each lane gets its own value
// and its partner's, in either order; a + b == b + a, so both halves hold the same sum)
__device__ __forceinline__ float sum_half_pair(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_half_pair(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
constexpr int kSSW = 8;                 // waves per workgroup
constexpr int kSSP = 32 * kSSW;         // listed positions per workgroup step
constexpr size_t kSSLds = 152 * 1024;   // LDS bytes for a group's basis
__host__ __device__ constexpr int ss_rs(int KQ) { return 2 * 16 * KQ + 16; }  // bytes per basis column
__host__ __device__ constexpr int ss_rp(int r) { return (r + 3) & ~3; }       // padded model columns

template <int KQ>
__global__ __launch_bounds__(64 * kSSW, 1) void score_mfma_f16s_kernel(SparseSearch a, int ngroups) {
  constexpr int KH = 16 * KQ;
  constexpr int RS = ss_rs(KQ);
  extern __shared__ __attribute__((aligned(16))) uint8_t sss[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hk = lane >> 5, l32 = lane & 31;
  const int D = a.D, r = a.r, rp = ss_rp(a.r);
  const int g = blockIdx.y;
  const int m0 = (int)((int64_t)g * a.M / ngroups), m1 = (int)((int64_t)(g + 1) * a.M / ngroups);
  const int ncols = (m1 - m0) * rp, ntile = (ncols + 31) / 32;
  int64_t* s_mode = reinterpret_cast<int64_t*>(sss + (size_t)ntile * 32 * RS);
  if (tid < a.nmodes) {
    s_mode[3 * tid] = a.pstart[tid];
    s_mode[3 * tid + 1] = a.md[tid].offset;
    s_mode[3 * tid + 2] = a.md[tid].P;
  }
  // the group's basis, padded column c (< ntile * 32) at c * RS: 2 KQ 16-byte parts; model
  // m0 + c / rp's basis row c % rp, zero past r and past the group
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  for (int e = tid; e < ntile * 32 * 2 * KQ; e += 64 * kSSW) {
    const int c = e / (2 * KQ), part = e - c * (2 * KQ);
    const int mm = c / rp, ii = c - mm * rp;
    u4 x = {0u, 0u, 0u, 0u};
    if (ii < r && m0 + mm < m1) x = *reinterpret_cast<const u4*>(a.qt16 + (int64_t)((m0 + mm) * r + ii) * KH + 8 * part);
    *reinterpret_cast<u4*>(sss + (size_t)c * RS + 16 * part) = x;
  }
  __syncthreads();
  const int n = (int)a.cnt[a.epoch & 1];
  // this wave's position sets: e0 = pb * kSSP + 32 * wave, pb = blockIdx.x, + gridDim.x, ...
  const int step = gridDim.x * kSSP;
  float v[KQ][8];
  auto load_rows = [&](int e0) {
    const int e = e0 + l32;
    const long long en = e < n ? a.list[e] : 0;
    const int mi = (int)(en >> 40);
    const int64_t p = en & ((1ll << 40) - 1);
    const float4* __restrict__ row = reinterpret_cast<const float4*>(a.gbox + (e < n ? (s_mode[3 * mi] + p) * D : 0));
#pragma unroll
    for (int s = 0; s < KQ; ++s)
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // D % 4 == 0: a 4-float chunk is wholly inside or past the row
        const int k = 16 * s + 8 * hk + 4 * h;
        float4 x = row[min(k, D - 4) >> 2];  // unconditional (no branch per load), then masked
        if (k >= D) x = make_float4(0.f, 0.f, 0.f, 0.f);
        v[s][4 * h] = x.x;
        v[s][4 * h + 1] = x.y;
        v[s][4 * h + 2] = x.z;
        v[s][4 * h + 3] = x.w;
      }
  };
  int e0 = blockIdx.x * kSSP + 32 * wave;
  if (e0 < n) load_rows(e0);
  for (; e0 < n; e0 += step) {
    // this set: scale (the power of two of score_mfma_f16_kernel) and round to f16
    const int e = e0 + l32;
    const bool valid = e < n;
    float mx = 0.0f;
#pragma unroll
    for (int s = 0; s < KQ; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf(v[s][j]));
    mx = max_half_pair(mx);
    int ex = 0;
    (void)frexpf(mx, &ex);
    mf_f16x8 av[KQ];
    float ff = 0.0f;
#pragma unroll
    for (int s = 0; s < KQ; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const _Float16 h = (_Float16)ldexpf(v[s][j], -ex);
        av[s][j] = h;
        ff = __builtin_fmaf((float)h, (float)h, ff);
      }
    ff = sum_half_pair(ff);
    int64_t sbase = 0, sP = 0;
    {
      const long long en = valid ? a.list[e] : 0;
      const int mi = (int)(en >> 40);
      sbase = s_mode[3 * mi + 1] + (en & ((1ll << 40) - 1));
      sP = s_mode[3 * mi + 2];
    }
    if (e0 + step < n) load_rows(e0 + step);  // the next set's rows, in flight during the sweep
    const uint8_t* bl = sss + (size_t)l32 * RS + 16 * hk;
    auto tile_mfma = [&](int t, mf_f32x16& acc) {
      mf_f16x8 bf[KQ];
#pragma unroll
      for (int s = 0; s < KQ; ++s) bf[s] = *reinterpret_cast<const mf_f16x8*>(bl + (size_t)t * 32 * RS + 32 * s);
      // every fragment read is issued before the first MFMA waits on one: one LDS round
      // trip per tile (interleaved read / MFMA pairs exposed it four times)
#pragma unroll
      for (int s = 0; s < KQ; ++s) __asm__ volatile("" : "+v"(bf[s]));
      const mf_f32x16 zero = {};
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf[0], av[0], zero, 0, 0, 0);
#pragma unroll
      for (int s = 1; s < KQ; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(bf[s], av[s], acc, 0, 0, 0);
    };
    const float rf = 1.0f / __fsqrt_rn(ff);  // scores in float: within the fp16 tolerance
    const bool emit = valid && hk == 0;
    float q2 = 0.0f;  // this lane's share of the current model's |Q f|^2
    auto finish = [&](int m, float x) {
      const float tot = sum_half_pair(x);
      if (emit) a.scores[sbase + (int64_t)(m0 + m) * sP] = (double)(__fsqrt_rn(tot) * rf);
    };
    auto epilogue = [&](int t, const mf_f32x16& acc) {
      float sq[4];  // this lane's quad j: columns 32 t + 8 j + 4 hk + 0..3, one model
      typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // packed: register pairs (4j, 4j+1), (4j+2, 4j+3)
        const f2 x = {acc[4 * j], acc[4 * j + 1]}, y = {acc[4 * j + 2], acc[4 * j + 3]};
        const f2 s2 = __builtin_elementwise_fma(y, y, x * x);
        sq[j] = s2.x + s2.y;
      }
      const int c0 = 32 * t, mA = c0 / rp, b1 = (mA + 1) * rp - c0;  // uniform
      if (b1 > 32) {  // no model ends in this tile
        q2 += (sq[0] + sq[1]) + (sq[2] + sq[3]);
        return;
      }
      // quads before b1 close model mA, quads in [b1, b1 + rp) go to mA + 1, the rest to
      // mA + 2 (r >= 16: at most two boundaries in 32 columns; a model may end exactly at
      // the tile's end, the group's last one always ends in the last tile)
      const int t1 = b1 - 4 * hk, t2 = t1 + rp;
      float p0 = 0.0f, p1 = 0.0f, p2 = 0.0f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool in0 = 8 * j < t1, in1 = 8 * j < t2;
        p0 += in0 ? sq[j] : 0.0f;
        p1 += (!in0 && in1) ? sq[j] : 0.0f;
        p2 += in1 ? 0.0f : sq[j];
      }
      if (m0 + mA < m1) finish(mA, q2 + p0);
      q2 = p1;
      if (b1 + rp <= 32) {
        if (m0 + mA + 1 < m1) finish(mA + 1, q2);
        q2 = p2;
      }
    };
    // two accumulators in turn: tile t + 1's fragment reads and MFMAs are issued before tile
    // t's epilogue reads its accumulator (no register copy waits on an MFMA in flight)
    mf_f32x16 accA, accB;
    tile_mfma(0, accA);
    for (int t = 0; t < ntile; t += 2) {
      if (t + 1 < ntile) tile_mfma(t + 1, accB);
      epilogue(t, accA);
      if (t + 1 < ntile) {
        if (t + 2 < ntile) tile_mfma(t + 2, accA);
        epilogue(t + 1, accB);
      }
    }
  }
}

// fewest model groups whose padded columns fit kSSLds (0: none fits)
int ss_groups(int M, int r, int KQ) {
  for (int g = 1; g <= M; ++g) {
    const int cols = (M + g - 1) / g * ss_rp(r);
    if ((size_t)((cols + 31) / 32) * 32 * ss_rs(KQ) + 3 * 6 * sizeof(int64_t) <= kSSLds) return g;
  }
  return 0;
}

template <int KQ>
hipError_t launch_score_mfma_f16s_kq(const SparseSearch& a, int ng, hipStream_t s) {
  static thread_local int n_cu = 0, dev_c = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != dev_c) {
    n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&score_mfma_f16s_kernel<KQ>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)kSSLds);
    dev_c = dev;
  }
  const int cols = (a.M + ng - 1) / ng * ss_rp(a.r);
  const size_t lds = (size_t)((cols + 31) / 32) * 32 * ss_rs(KQ) + 3 * 6 * sizeof(int64_t);
  // one workgroup per CU over all groups (LDS holds one), each sweeping its positions
  const int64_t pblocks = (a.pstart[a.nmodes] + kSSP - 1) / kSSP;
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(pblocks, std::max(1, n_cu / ng)));
  score_mfma_f16s_kernel<KQ><<<dim3(gx, (unsigned)ng), 64 * kSSW, lds, s>>>(a, ng);
  return hipGetLastError();
}

template <int KQ>
hipError_t launch_score_mfma_f16_kq(const SparseSearch& a, hipStream_t s) {
  if (a.r >= 16) {
    const int ng = ss_groups(a.M, a.r, KQ);
    if (ng > 0) return launch_score_mfma_f16s_kq<KQ>(a, ng, s);
  }
  static thread_local int slots = 0, dev_c = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  const size_t lds = sizeof(float) * (kBlock / 64) * 32 * kSMES + 3 * 6 * sizeof(int64_t);
  if (dev != dev_c) {
    int n_cu = 256, per_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, score_mfma_f16_kernel<KQ>, kBlock, lds) !=
            hipSuccess || per_cu < 1)
      per_cu = 1;
    slots = per_cu * n_cu;
    dev_c = dev;
  }
  const int64_t pblocks = (a.pstart[a.nmodes] + kSMP - 1) / kSMP;
  int ng = 1;
  double best = 1e300;
  for (int g = 1; g <= a.M; ++g) {  // the f32 kernel's cost model, in 32-column tiles
    const int64_t rounds = (pblocks * g + slots - 1) / slots;
    const int64_t cols = (int64_t)((a.M + g - 1) / g) * a.r;
    const double t = (double)rounds * (3.0 + (double)((cols + 31) / 32));
    if (t < best) {
      best = t;
      ng = g;
    }
  }
  const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(pblocks, 65535));
  score_mfma_f16_kernel<KQ><<<dim3(gx, (unsigned)ng), kBlock, lds, s>>>(a, ng);
  return hipGetLastError();
}

hipError_t launch_score_mfma_f16(const SparseSearch& a, hipStream_t s) {
  switch (a.Kq16) {
    case 1: return launch_score_mfma_f16_kq<1>(a, s);
    case 2: return launch_score_mfma_f16_kq<2>(a, s);
    case 3: return launch_score_mfma_f16_kq<3>(a, s);
    case 4: return launch_score_mfma_f16_kq<4>(a, s);
    case 5: return launch_score_mfma_f16_kq<5>(a, s);
    case 6: return launch_score_mfma_f16_kq<6>(a, s);
    case 7: return launch_score_mfma_f16_kq<7>(a, s);
    case 8: return launch_score_mfma_f16_kq<8>(a, s);
    case 9: return launch_score_mfma_f16_kq<9>(a, s);
    case 10: return launch_score_mfma_f16_kq<10>(a, s);
    default: return hipErrorInvalidValue;
  }
}

// rank 1 on large grids: block (b, m) reduces model m's scores of global positions
// g = b, b + grid, ... (every mode, scan order) to a (score desc, scan order asc) partial
constexpr int kArgmaxBlocks = 256;
__global__ __launch_bounds__(kBlock) void scores_argmax_kernel(SparseSearch a) {
  const int m = blockIdx.y;
  const int64_t ptot = a.pstart[a.nmodes];
  double best = -2.0;
  long long bo = -1;
  for (int64_t g = blockIdx.x * (int64_t)kBlock + threadIdx.x; g < ptot; g += (int64_t)gridDim.x * kBlock) {
    const int mi = find_mode(a, g);
    const ModeGeom& md = a.md[mi];
    const int64_t p = g - a.pstart[mi];
    const double sc = a.scores[md.offset + (int64_t)m * md.P + p];
    const long long o = a.order_base[mi] + p;
    if (sc >= 0 && (sc > best || (sc == best && o < bo))) {
      best = sc;
      bo = o;
    }
  }
  __shared__ double s_sc[kBlock / 64];
  __shared__ long long s_o[kBlock / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double os = __shfl_xor(best, o, 64);
    const long long oo = __shfl_xor(bo, o, 64);
    if (oo >= 0 && (os > best || (os == best && (bo < 0 || oo < bo)))) {
      best = os;
      bo = oo;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s_sc[w] = best;
    s_o[w] = bo;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kBlock / 64; ++i)
      if (s_o[i] >= 0 && (s_sc[i] > best || (s_sc[i] == best && (bo < 0 || s_o[i] < bo)))) {
        best = s_sc[i];
        bo = s_o[i];
      }
    a.partials[(int64_t)blockIdx.x * a.M + m] = ScorePartial{best, bo};
  }
}

// one wave per model (a model's reduction is a chain of dependent round trips: spread them)
__global__ __launch_bounds__(kBlock) void argmax_finalize_kernel(SparseSearch a, int nparts) {
  argmax_finalize(a, a.partials, a.lists, a.outs[0], nparts, blockIdx.x * (kBlock / 64), gridDim.x * (kBlock / 64));
}
unsigned finalize_blocks(int M) { return (unsigned)std::max(1, (M + kBlock / 64 - 1) / (kBlock / 64)); }

__global__ __launch_bounds__(kBlock) void score_list_kernel(SparseSearch b) {
  extern __shared__ __attribute__((aligned(16))) float sl_smem[];
  score_list_body(b, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y, sl_smem);
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

// rank update of searchPart (search.cpp:464-474) incl. checkOverlap (:327-356)
__device__ void rank_update(c3h_det* L, int rank, double cs, int x, int y, int z, int mode,
                            int xr, int yr, int zr, int r1, int r2, int r3) {
  for (int i = 0; i < rank; i++) {
    if (cs > L[i].score) {
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
        L[i].mode = mode;
      }
      break;
    }
  }
}

// general rank: one wave per model scans the scores in (mode, z, y, x) order, eight
// 64-position chunks per load batch; only candidates above the current rank-th score
// (lists only grow) reach the serial update.
__global__ __launch_bounds__(64) void replay_kernel(const double* __restrict__ scores,
                                                    ReplayModes modes, int rank, int r1,
                                                    int r2, int r3, int clean,
                                                    c3h_det* __restrict__ lists,
                                                    c3h_det* __restrict__ out2) {
  extern __shared__ __attribute__((aligned(16))) c3h_det L[];
  const int m = blockIdx.x, lane = threadIdx.x;
  c3h_det* gl = lists + (int64_t)m * rank;
  for (int i = lane; i < rank; i += 64) {
    c3h_det e = gl[i];
    if (clean) {  // 1: cleanMax (modes kept); 2: setRank state
      e.score = 0.0;
      e.x = e.y = e.z = 0;
      if (clean == 2) e.mode = 0;
    }
    L[i] = e;
  }
  __syncthreads();
  for (int mi = 0; mi < modes.n; ++mi) {
    const ReplayMode md = modes.m[mi];
    int xr, yr, zr;
    get_range(md.mode, r1, r2, r3, xr, yr, zr);
    const double* sc = scores + md.offset + (int64_t)m * md.P;
    for (int64_t b0 = 0; b0 < md.P; b0 += 512) {
      double s[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t p = b0 + 64 * j + lane;
        s[j] = p < md.P ? sc[p] : -1.0;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t base = b0 + 64 * j;
        double T = L[rank - 1].score;
        unsigned long long mask = __ballot(s[j] > T);
        while (mask) {
          const int jl = __ffsll((long long)mask) - 1;
          const double cs = __shfl(s[j], jl, 64);
          if (lane == 0) {
            const int64_t pc = base + jl;
            rank_update(L, rank, cs, (int)(pc % md.xe), (int)((pc / md.xe) % md.ye),
                        (int)(pc / ((int64_t)md.xe * md.ye)), md.mode, xr, yr, zr, r1, r2, r3);
          }
          __syncthreads();
          T = L[rank - 1].score;
          const unsigned long long later = jl >= 63 ? 0ull : (~0ull << (jl + 1));
          mask = __ballot(s[j] > T) & later;
        }
      }
    }
  }
  __syncthreads();
  for (int i = lane; i < rank; i += 64) {
    gl[i] = L[i];
    if (out2) out2[(int64_t)m * rank + i] = L[i];
  }
}

}  // namespace

// subdivision counts from which the stand-alone search compresses on the matrix cores
// (512^3 at S = 10: 140,608; the bench's 256^3 frames, 17,576, keep the fused VALU launch)
// kCompressMfmaRows (c3h_internal.h): the matrix-core compresses from this many rows

bool compress_rows_ok(int F, int Dpad) {
  (void)F;
  return Dpad <= 128;
}

hipError_t launch_compress(const float* feat, int64_t H, int F, const float* axis_pt, int D,
                           int Dpad, const float* fmax, int fmax_len, float* G,
                           const int32_t* rows, const uint32_t* nrows, const int32_t* exist,
                           hipStream_t s) {
  if (rows && compress_rows_ok(F, Dpad)) {  // sparse list
    const size_t lds = compress_rows_lds_bytes(Dpad);
    const CompressRows cr{feat, axis_pt, fmax, G, rows, nrows, F, D, Dpad, fmax_len, 0, 0, 0, 0};
    compress_rows_kernel<<<(unsigned)((H + kRR - 1) / kRR), kBlock, lds, s>>>(cr);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((H + kCM - 1) / kCM), (unsigned)((Dpad + kCN - 1) / kCN));
  compress_kernel<<<grid, kCT, 0, s>>>(feat, H, F, axis_pt, D, Dpad, fmax, fmax_len, G, rows, nrows, exist);
  return hipGetLastError();
}

// dst[h][:] = exist[h] ? src[h][:] : 0 (readback of sparse feature / G buffers)
__global__ __launch_bounds__(kBlock) void masked_rows_kernel(const float* __restrict__ src,
                                                             const int32_t* __restrict__ exist,
                                                             int64_t H, int W, float* __restrict__ dst) {
  const int64_t n = H * W;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int64_t h = i / W;
    dst[i] = exist[h] ? src[i] : 0.0f;
  }
}

hipError_t launch_masked_rows(const float* src, const int32_t* exist, int64_t H, int W, float* dst,
                              hipStream_t s) {
  const int64_t n = H * W;
  if (n <= 0) return hipSuccess;
  const unsigned g = (unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 4096);
  masked_rows_kernel<<<g, kBlock, 0, s>>>(src, exist, H, W, dst);
  return hipGetLastError();
}

size_t score_lds_bytes(int D, int r, int SP) {
  return sizeof(float) * ((size_t)SP * (D + 1) + (size_t)r * SP + SP) + sizeof(int) * SP;
}

bool score_fast_ok(int D, int r) { return D <= 160 && (D & 3) == 0 && r <= kOC; }
bool score_mfma_ok(int D) { return D >= 4 && D <= 160 && (D & 3) == 0; }

int64_t score_blocks(const ScoreLaunch& a) {
  const int64_t P = (int64_t)a.xe * a.ye * a.ze;
  if (score_fast_ok(a.D, a.r)) return (P + kFP - 1) / kFP;
  return a.D <= 256 ? (P + 63) / 64 : (P + 15) / 16;
}

hipError_t launch_score(const ScoreLaunch& a, hipStream_t s) {
  const int64_t P = (int64_t)a.xe * a.ye * a.ze;
  if (P <= 0) return hipSuccess;
  if (score_fast_ok(a.D, a.r)) {
    return hipErrorInvalidValue;  // the fast path is the sparse search (launch_sparse_search)
  } else if (a.D <= 256) {
    score_kernel<64><<<(unsigned)((P + 63) / 64), kBlock, score_lds_bytes(a.D, a.r, 64), s>>>(a, P);
  } else {
    score_kernel<16><<<(unsigned)((P + 15) / 16), kBlock, score_lds_bytes(a.D, a.r, 16), s>>>(a, P);
  }
  return hipGetLastError();
}

int64_t sparse_score_blocks(const SparseSearch& a) { return (a.pstart[a.nmodes] + kFP - 1) / kFP; }

hipError_t launch_sparse_search(const SparseSearch& a, const SparseCompress* sc, hipStream_t s) {
  const int64_t ptot = a.pstart[a.nmodes];
  if (ptot <= 0) return hipSuccess;
  const unsigned ngate = (unsigned)((ptot + kBlock - 1) / kBlock);
  const unsigned nf = (unsigned)a.nframes;
  if (sc) {  // compress (non-empty rows) and gate in one launch
    const CompressRows cr{sc->feat, sc->PT, sc->fmax, sc->G, sc->rows, sc->nrows, sc->F, sc->D, sc->Dpad,
                          sc->fmax_len, sc->s_feat, sc->s_G, sc->s_rows, sc->s_nrows, sc->H,
                          sc->PT16 ? sc->feat16 : nullptr, sc->feat16_flag, sc->f16s};
    if (sc->H >= kCompressMfmaRows) {  // large grids: the f32 matrix-core compress, then the gate
      // persistent: every workgroup resident (row blocks b, b + grid, ...), so no partial
      // last round of workgroups
      if (sc->PT16) {  // fp16 search precision
        const int64_t rblocks = (sc->H + kMR - 1) / kMR;
        unsigned ncomp = (unsigned)std::min<int64_t>(rblocks, 2048);
#ifndef C3H_CF16_BALANCED
#define C3H_CF16_BALANCED 0  // diagnostics: persistent workgroups in balanced rounds (3 per CU)
#endif
        if (C3H_CF16_BALANCED) {
          int dev = 0, n_cu = 256;
          (void)hipGetDevice(&dev);
          (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
          const int64_t slots = std::max<int64_t>(1, 3 * (int64_t)n_cu / std::max(1u, nf));
          const int64_t rounds = (rblocks + slots - 1) / slots;
          ncomp = (unsigned)std::min<int64_t>(rblocks, (rblocks + rounds - 1) / rounds);
        }
        compress_f16_kernel<<<dim3(ncomp, nf), kBlock, 0, s>>>(cr, sc->PT16, sc->Fp16);
        gate_kernel<<<dim3(ngate, nf), kBlock, 0, s>>>(a);
        goto score;
      }
      {  // f32: row-coalesced LDS staging (3 workgroups per CU at 49 KB)
        static thread_local int c_slots = 0, c_dev = -1;
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev != c_dev) {
          int n_cu = 256, per_cu = 0;
          (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
          (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&compress_f32c_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCLds);
          if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, compress_f32c_kernel, kBlock, kCLds) != hipSuccess ||
              per_cu < 1)
            per_cu = 1;
          c_slots = per_cu * n_cu;
          c_dev = dev;
        }
        // persistent: every workgroup resident (row blocks b, b + grid, ...), balanced rounds
        const int64_t rblocks = (sc->H + kCR - 1) / kCR;
        const int64_t slots = std::max<int64_t>(1, c_slots / std::max(1u, nf));
        const int64_t rounds = (rblocks + slots - 1) / slots;
        const unsigned ncomp = (unsigned)std::min<int64_t>(rblocks, (rblocks + rounds - 1) / rounds);
        compress_f32c_kernel<<<dim3(ncomp, nf), kBlock, kCLds, s>>>(cr);
        gate_kernel<<<dim3(ngate, nf), kBlock, 0, s>>>(a);
      }
    } else {
      const size_t lds = compress_rows_lds_bytes(sc->Dpad);
      // compress workgroups: surface frames have ~700 non-empty rows (~44 row blocks)
      const unsigned ncomp = (unsigned)std::min<int64_t>((sc->H + kRR - 1) / kRR, kCompressGridCap);
      compress_gate_kernel<<<dim3(ngate + ncomp, nf), kBlock, lds, s>>>(cr, a, (int)ngate);
    }
  } else {
    gate_kernel<<<dim3(ngate, nf), kBlock, 0, s>>>(a);
  }
score:
  if (a.gbox) {
    const int64_t n = ptot * (a.D >> 2);
    boxsum_kernel<<<dim3((unsigned)std::min<int64_t>((n + kBlock - 1) / kBlock, 16384), nf), kBlock, 0, s>>>(a);
  }
  if (a.score_mfma) {  // single frame, box sums above: the matrix-core projection
    if (!a.gbox || nf != 1 || !score_mfma_ok(a.D)) return hipErrorInvalidValue;
    const hipError_t e = a.qt16 ? launch_score_mfma_f16(a, s) : launch_score_mfma(a, s);
    if (e != hipSuccess) return e;
    if (a.lists) {  // rank 1: parallel argmax over the written scores + finalize
      scores_argmax_kernel<<<dim3(kArgmaxBlocks, a.M), kBlock, 0, s>>>(a);
      argmax_finalize_kernel<<<finalize_blocks(a.M), kBlock, 0, s>>>(a, kArgmaxBlocks);
    }
    return hipGetLastError();
  }
  const size_t lds = score_list_lds_bytes(a.D, a.mpg);
  const unsigned groups = (unsigned)((a.M + a.mpg - 1) / a.mpg);
  // workgroups per (group, frame): list chunks beyond the cap loop (dense scenes only);
  // surface frames pass ~1k positions (~30 chunks), so few workgroups exit unused
  // (large grids with precomputed box sums: enough workgroups to fill the chip)
  const unsigned gx = (unsigned)std::min<int64_t>(sparse_score_blocks(a), a.gbox ? 2048 : kScoreGridCap);
  if (a.gbox && a.lists) {  // large grid, rank 1: scores, then a parallel argmax + finalize
    SparseSearch b = a;
    b.partials = nullptr;
    b.lists = nullptr;
    score_list_kernel<<<dim3(gx, groups, nf), kBlock, lds, s>>>(b);
    scores_argmax_kernel<<<dim3(kArgmaxBlocks, a.M), kBlock, 0, s>>>(a);
    argmax_finalize_kernel<<<finalize_blocks(a.M), kBlock, 0, s>>>(a, kArgmaxBlocks);
    return hipGetLastError();
  }
  score_list_kernel<<<dim3(gx, groups, nf), kBlock, lds, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_replay(const double* scores, const ReplayModes& modes, int M, int rank,
                         int r1, int r2, int r3, int clean, c3h_det* lists, c3h_det* out2,
                         hipStream_t s) {
  replay_kernel<<<M, 64, sizeof(c3h_det) * rank, s>>>(scores, modes, rank, r1, r2, r3, clean,
                                                      lists, out2);
  return hipGetLastError();
}


}  // namespace c3h
