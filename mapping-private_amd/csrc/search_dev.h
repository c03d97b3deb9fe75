// search_dev.h -- device bodies of the sparse search stages (sparse compress, exist
// gate, list scoring with the fused rank-1 argmax), shared by the stand-alone kernels
// (search.hip) and the pipelined tick kernel (pipeline.hip).  Bodies take their block
// coordinates and LDS base explicitly.  See search.hip for the method.
#pragma once
#include "c3h_internal.h"

namespace c3h {

// Sparse compress (row list from the extract): 16 listed rows per workgroup x all
// columns (Dpad <= 128).  Per 32-feature chunk, the 16 rows' feature slice (max-
// normalised) and the 32 x Dpad slice of P are staged in LDS, both prefetched one chunk
// ahead into registers so only the first load's latency is exposed; LDS use does not
// depend on F (981 fits the tick).  Thread = (row, 8 columns); the fma chain per output
// runs in ascending j exactly like compress_kernel, so both paths give identical G rows.
constexpr int kRR = 16, kRK = 32;
constexpr int kRS = kRK + 1;  // feature slice row stride (4 rows per wave: no bank conflict)
constexpr int kCompressGridCap = 128;  // row-block workgroups per frame of the fused launch
__host__ __device__ inline size_t compress_rows_lds_bytes(int Dpad) {
  return sizeof(float) * ((size_t)kRK * Dpad + (size_t)kRR * kRS);
}

struct CompressRows {
  const float* feat;
  const float* PT;
  const float* fmax;
  float* G;
  const int32_t* rows;
  const uint32_t* nrows;
  int F, D, Dpad, fmax_len;
  int64_t s_feat, s_G, s_rows, s_nrows;  // per-frame strides (frame = launch y / z index)
  int64_t H = 0;  // subdivisions per frame: a list of all H rows is read as rows 0..H-1 in order
  const _Float16* feat16 = nullptr;  // f16 rows (stride f16s) instead of feat when *feat16_flag
  const uint32_t* feat16_flag = nullptr;
  int f16s = 0;
};

__device__ __forceinline__ void compress_rows_body(const CompressRows& cr, int bid, int nblk, int64_t f,
                                                   float* csm) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, Dpad = cr.Dpad, fmax_len = cr.fmax_len;
  float* pc = csm;                 // kRK x Dpad
  float* fs = csm + kRK * Dpad;    // kRR x kRS (one 32-feature slice of the 16 rows)
  const int tid = threadIdx.x;
  const int nq4 = kRK * Dpad / 4, tot4 = F * Dpad / 4;
  const float4* P4 = reinterpret_cast<const float4*>(cr.PT);
  float4 pre[4];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = tid + j * kBlock, g = c * nq4 + e;
      pre[j] = (e < nq4 && g < tot4) ? P4[g] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // feature slice: element e = tid + i * kBlock -> row e / kRK, feature c * kRK + e % kRK
  float fpre[kRR * kRK / kBlock];
  int64_t rbase[kRR * kRK / kBlock];
  auto load_feat = [&](int c) {
#pragma unroll
    for (int i = 0; i < kRR * kRK / kBlock; ++i) {
      const int e = tid + i * kBlock, j = c * kRK + (e & (kRK - 1));
      float v = 0.0f;
      if (rbase[i] >= 0 && j < F) {
        v = feat[rbase[i] + j];
        if (j < fmax_len) {  // setData max-normalisation (search.cpp:563-570)
          const float mx = fmax[j];
          if (mx == 0.0f) v = 0.0f;
          else if (v == mx) v = 1.0f;
          else v = __fdiv_rn(v, mx);
        }
      }
      fpre[i] = v;
    }
  };
  // P's first chunk is independent of the row count: in flight before the count arrives
  load_chunk(0);
  const int n = (int)cr.nrows[f * cr.s_nrows];
  const int row = tid >> 4, cg = tid & 15;
  const bool active = 8 * cg < Dpad;
  const int nch = (F + kRK - 1) / kRK;
  // row blocks bid, bid + nblk, ... (the launch holds few workgroups; dense scenes loop)
  for (int r0 = bid * kRR; r0 < n; r0 += nblk * kRR) {
    if (r0 != bid * kRR) load_chunk(0);
#pragma unroll
    for (int i = 0; i < kRR * kRK / kBlock; ++i) {
      const int r = (tid + i * kBlock) / kRK;
      rbase[i] = r0 + r < n ? (int64_t)rows[r0 + r] * F : -1;
    }
    load_feat(0);
    float acc[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[q] = 0.0f;
    for (int c = 0; c < nch; ++c) {
      lds_barrier();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + j * kBlock;
        if (e < nq4) reinterpret_cast<float4*>(pc)[e] = pre[j];
      }
#pragma unroll
      for (int i = 0; i < kRR * kRK / kBlock; ++i) {
        const int e = tid + i * kBlock;
        fs[(e / kRK) * kRS + (e & (kRK - 1))] = fpre[i];
      }
      if (c + 1 < nch) {
        load_chunk(c + 1);
        load_feat(c + 1);
      }
      lds_barrier();
      if (active) {
        const int kn = min(kRK, F - c * kRK);
        const float* fr = fs + row * kRS;
        for (int k = 0; k < kn; ++k) {
          const float fv = fr[k];
          const float4 p0 = *reinterpret_cast<const float4*>(&pc[k * Dpad + 8 * cg]);
          const float4 p1 = *reinterpret_cast<const float4*>(&pc[k * Dpad + 8 * cg + 4]);
          acc[0] = __builtin_fmaf(fv, p0.x, acc[0]);
          acc[1] = __builtin_fmaf(fv, p0.y, acc[1]);
          acc[2] = __builtin_fmaf(fv, p0.z, acc[2]);
          acc[3] = __builtin_fmaf(fv, p0.w, acc[3]);
          acc[4] = __builtin_fmaf(fv, p1.x, acc[4]);
          acc[5] = __builtin_fmaf(fv, p1.y, acc[5]);
          acc[6] = __builtin_fmaf(fv, p1.z, acc[6]);
          acc[7] = __builtin_fmaf(fv, p1.w, acc[7]);
        }
      }
    }
    if (active && r0 + row < n) {
      const int64_t h = rows[r0 + row];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (8 * cg + q < D) G[h * D + 8 * cg + q] = acc[q];
    }
    lds_barrier();  // fs / pc are rewritten by the next row block
  }
}

// Dense frames (tens of thousands of listed rows): the same G = f' * P on the matrix cores.
// v_mfma_f32_32x32x2_f32 is bit-for-bit a k-ordered fmaf chain
// (D = fma(a_k1, b_k1, fma(a_k0, b_k0, C))), so feeding k in ascending order gives the VALU
// body's G exactly (zero products pad F to the chunk size: fma(0, 0, x) = x).
constexpr int kMR = 128;  // rows per workgroup of the fp16 compress
typedef float mf_f32x16 __attribute__((ext_vector_type(16)));

// f32 matrix-core compress, row-coalesced (round 3; replaced an LDS-DMA ring whose 64-lane
// loads touched four rows in 64-B pieces: 0.57 -> 0.41 ms at 512^3): ascending k pairs on
// v_mfma_f32_32x32x2_f32 (G bit-identical to the VALU body), with
// k in chunks of 64 staged in LDS from registers: every wave-wide feature load reads 64
// consecutive floats of ONE row (256 B) instead of 16-float pieces of four rows, and the
// next chunk's loads (the block's 64 rows, a 64 x 128 slice of P) are in flight in
// registers while this chunk's MFMAs run.  64 rows per workgroup, wave (rw, cw) = 32 rows x
// 2 column tiles: 32 accumulator registers per lane, so 3 waves per SIMD and 3 workgroups
// per CU (49 KB of LDS each), and 2,197 row blocks of a 512^3 frame fill 768 slots in 2.9
// rounds where 128-row blocks took 3 rounds of twice the work (1,099 over 512 slots).
// Normalises by feature_max on the LDS store.
constexpr int kCK = 64;                 // k per chunk
constexpr int kCR = 64;                 // rows per workgroup
constexpr int kCAS = kCK + 1;           // A row stride in floats (odd: conflict-free column reads)
constexpr size_t kCLds = sizeof(float) * ((size_t)kCR * kCAS + (size_t)kCK * 128);

__device__ __forceinline__ void compress_f32c_body(const CompressRows& cr, int bid, int nblk, int64_t f,
                                                   float* smem) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, Dpad = cr.Dpad, fmax_len = cr.fmax_len;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rw = wave & 1, cw = wave >> 1;
  const int n = (int)cr.nrows[f * cr.s_nrows];
  const int nch = (F + kCK - 1) / kCK;
  float* As = smem;               // [kCR rows][kCAS]
  float* Bs = smem + kCR * kCAS;  // [kCK][128]
  const bool ident = n == cr.H;
  for (int r0 = bid * kCR; r0 < n; r0 += nblk * kCR) {
    // every subdivision listed (dense frame): rows in memory order (contiguous feature rows)
    const int myrow = r0 + wave * 16 + (lane & 15);
    const int hrow = myrow < n ? (ident ? myrow : rows[myrow]) : -1;  // lane j < 16: this wave's load row j
    float areg[16];
    float4 breg[8];
    auto fetch = [&](int c) {
      const int k = c * kCK + lane;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int h = __builtin_amdgcn_readlane(hrow, j);
        areg[j] = (h >= 0 && k < F) ? __builtin_nontemporal_load(feat + (int64_t)h * F + k) : 0.0f;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pc = tid + kBlock * i, kk = c * kCK + (pc >> 5), col = 4 * (pc & 31);
        breg[i] = (kk < F && col < Dpad) ? *reinterpret_cast<const float4*>(cr.PT + (int64_t)kk * Dpad + col)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto stage = [&](int c) {
      const int k = c * kCK + lane;
      float mx = 1.0f;
      const bool norm = k < fmax_len;  // setData max-normalisation (search.cpp:563-570)
      if (norm) mx = fmax[k];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        float v = areg[j];
        if (norm) v = mx == 0.0f ? 0.0f : (v == mx ? 1.0f : __fdiv_rn(v, mx));
        As[(wave * 16 + j) * kCAS + lane] = v;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int pc = tid + kBlock * i;
        *reinterpret_cast<float4*>(Bs + (pc >> 5) * 128 + 4 * (pc & 31)) = breg[i];
      }
    };
    mf_f32x16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.0f;
    fetch(0);
    const float* arow = As + (rw * 32 + (lane & 31)) * kCAS + (lane >> 5);
    const float* bcol = Bs + (lane >> 5) * 128 + 64 * cw + (lane & 31);
    for (int c = 0; c < nch; ++c) {
      __syncthreads();  // every wave is done reading chunk c - 1
      stage(c);
      __syncthreads();
      if (c + 1 < nch) fetch(c + 1);  // in flight while the matrix cores run
#pragma unroll 8
      for (int k = 0; k < kCK; k += 2) {
        const float av = arow[k];
        const float b0 = bcol[k * 128], b1 = bcol[k * 128 + 32];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b1, acc[1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rr = r0 + rw * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
      if (rr >= n) continue;
      const int64_t hh = ident ? rr : rows[rr];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int col = 64 * cw + 32 * t + (lane & 31);
        if (col < D) G[hh * D + col] = acc[t][q];
      }
    }
  }
}

// The tick's compress role on the matrix cores (round 6): compress_f32c_body's GEMM with k
// in chunks of 32 (24.8 KB of LDS instead of 49: inside the tick's per-workgroup budget, so
// the tick keeps its workgroups per CU), rows from the frame's non-empty row list.  The VALU
// body (compress_rows_body) reads 3 LDS words per 8 FMAs and is LDS-bound; here a wave reads
// 768 B per 4,096 FMAs.  k pairs run in ascending order on v_mfma_f32_32x32x2_f32: G is
// bit-identical to the VALU body's (the same k-ordered fmaf chain per output).
constexpr int kTK = 32;
constexpr int kTAS = kTK + 1;
constexpr size_t kTLds = sizeof(float) * ((size_t)kCR * kTAS + (size_t)kTK * 128);

__device__ __forceinline__ void compress_f32t_body(const CompressRows& cr, int bid, int nblk, int64_t f,
                                                   float* smem) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, Dpad = cr.Dpad, fmax_len = cr.fmax_len;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rw = wave & 1, cw = wave >> 1;
  const int half = lane >> 5, kl = lane & 31;
  const int n = (int)cr.nrows[f * cr.s_nrows];
  const int nch = (F + kTK - 1) / kTK;
  float* As = smem;               // [kCR rows][kTAS]
  float* Bs = smem + kCR * kTAS;  // [kTK][128]
  for (int r0 = bid * kCR; r0 < n; r0 += nblk * kCR) {
    const int myrow = r0 + wave * 16 + (lane & 15);
    const int hrow = myrow < n ? rows[myrow] : -1;  // lane j < 16: this wave's load row j
    float areg[8];
    float4 breg[4];
    auto fetch = [&](int c) {
      const int k = c * kTK + kl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // rows 2 j (lanes 0-31) and 2 j + 1 (lanes 32-63)
        const int h = __shfl(hrow, 2 * j + half, 64);
        areg[j] = (h >= 0 && k < F) ? __builtin_nontemporal_load(feat + (int64_t)h * F + k) : 0.0f;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pc = tid + kBlock * i, kk = c * kTK + (pc >> 5), col = 4 * (pc & 31);
        breg[i] = (kk < F && col < Dpad) ? *reinterpret_cast<const float4*>(cr.PT + (int64_t)kk * Dpad + col)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    auto stage = [&](int c) {
      const int k = c * kTK + kl;
      float mx = 1.0f;
      const bool norm = k < fmax_len;  // setData max-normalisation (search.cpp:563-570)
      if (norm) mx = fmax[k];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = areg[j];
        if (norm) v = mx == 0.0f ? 0.0f : (v == mx ? 1.0f : __fdiv_rn(v, mx));
        As[(wave * 16 + 2 * j + half) * kTAS + kl] = v;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pc = tid + kBlock * i;
        *reinterpret_cast<float4*>(Bs + (pc >> 5) * 128 + 4 * (pc & 31)) = breg[i];
      }
    };
    mf_f32x16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.0f;
    fetch(0);
    const float* arow = As + (rw * 32 + kl) * kTAS + half;
    const float* bcol = Bs + half * 128 + 64 * cw + kl;
    for (int c = 0; c < nch; ++c) {
      __syncthreads();  // every wave is done reading chunk c - 1
      stage(c);
      __syncthreads();
      if (c + 1 < nch) fetch(c + 1);  // in flight while the matrix cores run
#pragma unroll
      for (int k = 0; k < kTK; k += 2) {
        const float av = arow[k];
        const float b0 = bcol[k * 128], b1 = bcol[k * 128 + 32];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b0, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b1, acc[1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rr = r0 + rw * 32 + (q & 3) + 8 * (q >> 2) + 4 * half;
      if (rr >= n) continue;
      const int64_t hh = rows[rr];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int col = 64 * cw + 32 * t + kl;
        if (col < D) G[hh * D + col] = acc[t][q];
      }
    }
    __syncthreads();  // As / Bs are restaged by the next row block
  }
}

// fp16 variant of the matrix-core compress (c3h_set_search_precision): the normalised
// features are rounded to f16, the whitened axis is kept as f16 (PT16: 128 columns x
// Fp16 = F rounded up to 16, column-major), products accumulate in f32 on
// v_mfma_f32_32x32x16_f16.  Workgroup = 128 rows; k runs in chunks of 64 staged through
// LDS: each wave-wide load reads 64 consecutive floats of ONE row (256 coalesced bytes,
// not 64 rows' scattered dwords), the next chunk's loads are in flight in registers while
// the matrix cores consume the current one.  Stated tolerance: scores within 2e-3
// relative of the float64 oracle (tests/test_gpu_parity.py::test_config5_dense_512_periodic).
typedef _Float16 mf_f16x8 __attribute__((ext_vector_type(8)));
constexpr int kCFK = 64;             // k per LDS chunk
constexpr int kCFS = kCFK + 8;       // LDS row stride in halves (144 B: conflict-free b128 reads)
constexpr int kCFRows = kMR / 4;     // rows of one wave's loads (= the wave's 32 A rows)
constexpr int kCFLds = 2 * 128 * kCFS * 2;  // A (128 rows) + B (128 columns), bytes

typedef unsigned mf_u32x4 __attribute__((ext_vector_type(4)));
// kF16In: the rows are the C3 epilogue's f16 rows (c3h_set_search_precision before the
// extract): a lane loads 16 B = 8 halves of a row, so one wave-wide load covers 8 rows'
// 128-B chunk slices (2-B loads per lane ran the compress at 0.54 ms instead of 0.17)
template <bool kF16In>
__device__ __forceinline__ void compress_f16_body(const CompressRows& cr, const _Float16* __restrict__ PT16,
                                                  int Fp16, int bid, int nblk, int64_t f, _Float16* smem) {
  const float* __restrict__ feat = cr.feat + f * cr.s_feat;
  const float* __restrict__ fmax = cr.fmax;
  float* __restrict__ G = cr.G + f * cr.s_G;
  const int32_t* __restrict__ rows = cr.rows + f * cr.s_rows;
  const int F = cr.F, D = cr.D, fmax_len = cr.fmax_len;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = (int)cr.nrows[f * cr.s_nrows];
  const int nch = (Fp16 + kCFK - 1) / kCFK;
  _Float16* As = smem;               // [128 rows][kCFS]
  _Float16* Bs = smem + 128 * kCFS;  // [128 columns][kCFS]
  const bool ident = n == cr.H;
  const _Float16* __restrict__ f16 = cr.feat16;
  const int f16s = cr.f16s;  // a multiple of 8 halves (16-B aligned rows, zero padding)
  for (int r0 = bid * kMR; r0 < n; r0 += nblk * kMR) {
    // every subdivision listed (dense frame): the list is a permutation of 0..H-1, so row
    // block r0 covers subdivisions r0.. in memory order instead (contiguous feature rows)
    const int myrow = r0 + wave * 32 + (lane & 31);
    const int hrow = myrow < n ? (ident ? myrow : rows[myrow]) : -1;  // lane j: the wave's row j
    float areg[kF16In ? 1 : kCFRows];
    mf_u32x4 a16[kF16In ? kCFRows / 8 : 1];
    uint4 breg[4];
    auto fetch = [&](int c) {
      if (kF16In) {
        const int kq = c * kCFK + (lane & 7) * 8;
#pragma unroll
        for (int j = 0; j < kCFRows / 8; ++j) {
          const int h = __shfl(hrow, j * 8 + (lane >> 3), 64);
          a16[j] = (h >= 0 && kq < f16s)
                       ? __builtin_nontemporal_load(reinterpret_cast<const mf_u32x4*>(f16 + (int64_t)h * f16s + kq))
                       : mf_u32x4{0u, 0u, 0u, 0u};
        }
      } else {
        const int k = c * kCFK + lane;
#pragma unroll
        for (int j = 0; j < kCFRows; ++j) {
          const int h = __builtin_amdgcn_readlane(hrow, j);
          areg[j] = (h >= 0 && k < F) ? __builtin_nontemporal_load(feat + (int64_t)h * F + k) : 0.0f;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pc = tid + kBlock * i, col = pc >> 3, kk = c * kCFK + (pc & 7) * 8;
        breg[i] = kk < Fp16 ? *reinterpret_cast<const uint4*>(PT16 + (int64_t)col * Fp16 + kk) : make_uint4(0, 0, 0, 0);
      }
    };
    auto stage = [&](int c) {
      if (kF16In) {
        const int kq = c * kCFK + (lane & 7) * 8;
        float mx[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) mx[e] = kq + e < fmax_len ? fmax[kq + e] : -1.0f;  // -1: not normalised
#pragma unroll
        for (int j = 0; j < kCFRows / 8; ++j) {
          mf_u32x4 o;
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const uint32_t w = a16[j][e2];
            float v[2] = {(float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu)),
                          (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16))};
#pragma unroll
            for (int u = 0; u < 2; ++u) {  // setData max-normalisation (search.cpp:563-570)
              const float m = mx[2 * e2 + u];
              if (m >= 0.0f) v[u] = m == 0.0f ? 0.0f : (v[u] == m ? 1.0f : __fdiv_rn(v[u], m));
            }
            o[e2] = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v[0]) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, (_Float16)v[1]) << 16);
          }
          *reinterpret_cast<mf_u32x4*>(As + (wave * 32 + j * 8 + (lane >> 3)) * kCFS + (lane & 7) * 8) = o;
        }
      } else {
        const int k = c * kCFK + lane;
        float mx = 1.0f;
        const bool norm = k < fmax_len;  // setData max-normalisation (search.cpp:563-570)
        if (norm) mx = fmax[k];
#pragma unroll
        for (int j = 0; j < kCFRows; ++j) {
          float v = areg[j];
          if (norm) v = mx == 0.0f ? 0.0f : (v == mx ? 1.0f : __fdiv_rn(v, mx));
          As[(wave * 32 + j) * kCFS + lane] = (_Float16)v;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pc = tid + kBlock * i;
        *reinterpret_cast<uint4*>(Bs + (pc >> 3) * kCFS + (pc & 7) * 8) = breg[i];
      }
    };
    mf_f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[t][q] = 0.0f;
    fetch(0);
    const _Float16* arow = As + (wave * 32 + (lane & 31)) * kCFS + 8 * (lane >> 5);
    const _Float16* bcol = Bs + (lane & 31) * kCFS + 8 * (lane >> 5);
    for (int c = 0; c < nch; ++c) {
      __syncthreads();  // every wave is done reading chunk c - 1
      stage(c);
      __syncthreads();
      if (c + 1 < nch) fetch(c + 1);  // in flight while the matrix cores run
#pragma unroll
      for (int s = 0; s < kCFK / 16; ++s) {
        const mf_f16x8 av = *reinterpret_cast<const mf_f16x8*>(arow + 16 * s);
        mf_f16x8 bv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[t] = *reinterpret_cast<const mf_f16x8*>(bcol + 32 * t * kCFS + 16 * s);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv[t], acc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int rr = r0 + wave * 32 + (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
      if (rr >= n) continue;
      const int64_t hh = ident ? rr : rows[rr];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int col = 32 * t + (lane & 31);
        if (col < D) G[hh * D + col] = acc[t][q];
      }
    }
  }
}

// Fast path (D <= 256, D % 4 == 0, M*r <= 256) = the sparse search below: 32 list
// entries per workgroup.  Box features are summed with float4 loads and staged k-major in
// LDS (lanes = positions: conflict-free); the projection onto all M*r basis rows is a
// 32 x Opad x D fp32 GEMM with a 2-position x 16-row register tile per thread (one
// ds_read_b64 of box features + four ds_read_b128 of basis rows feed 32 FMAs), the basis
// streamed through LDS in 16-row chunks prefetched one chunk ahead into registers;
// |Q_m f|^2 is summed per (position, model) in a fixed order.  The block also emits its
// per-model best (score, scan order) so rank-1 searches need no second pass.
constexpr int kFP = 32;
#ifndef C3H_SCORE_CB
#define C3H_SCORE_CB 2
#endif
constexpr int kOC = 64;  // basis rows per workgroup (whole models)
constexpr int kScoreGridCap = 128;  // workgroups per (model group, frame) of the score launch

// ---------------------------------------------------------------- sparse search
// The exist gate passes few positions on surface scenes (a depth camera sees a 2-D
// manifold), so the gate runs first over every position of every mode and compacts the
// passing ones into a list; the projection then runs over the list only.  Entries are
// (mode index << 40) | position; list order is irrelevant: scores are per position and
// the per-block partials break ties on the scan order explicitly.
__device__ __forceinline__ int find_mode(const SparseSearch& a, int64_t g) {
  int mi = 0;
  while (mi + 1 < a.nmodes && g >= a.pstart[mi + 1]) ++mi;
  return mi;
}

// frame f of a batched search: per-frame pointers at base + f * stride (no struct copy:
// a by-value SparseSearch with its dynamically indexed mode table would live in scratch)
__device__ __forceinline__ void gate_body(const SparseSearch& a, int bid, int64_t f) {
  const int tid = threadIdx.x, lane = tid & 63;
  uint32_t* __restrict__ fcnt = a.cnt + f * a.s_cnt;
  uint32_t* __restrict__ fdone = a.done + f * a.s_cnt;
  const int32_t* __restrict__ fexist = a.exist + f * a.s_exist;
  double* __restrict__ fscores = a.scores + f * a.s_scores;
  long long* __restrict__ flist = a.list + f * a.s_list;
  if (bid == 0 && tid == 0) {  // the next search's counters
    fcnt[(a.epoch + 1) & 1] = 0;
    fdone[(a.epoch + 1) & 1] = 0;
  }
  const int64_t g = bid * (int64_t)kBlock + tid;
  bool pass = false;
  int64_t entry = 0;
  if (g < a.pstart[a.nmodes]) {
    const int mi = find_mode(a, g);
    const ModeGeom& md = a.md[mi];
    const int64_t p = g - a.pstart[mi];
    const int64_t xye = (int64_t)md.xe * md.ye;
    const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
    const int xyn = a.xn * a.yn;
    const int h = z * xyn + y * a.xn + x;
    // model 0's score of the previous search of this layout (issued with the exist loads)
    const double prev = a.sparse_scores ? fscores[md.offset + p] : 0.0;
    int e = 0;  // SearchObj::clipValue<int> on exist_voxel_num (search.cpp:484-535), exact
    for (int dz = 0; dz < md.zr; ++dz)
      for (int dy = 0; dy < md.yr; ++dy)
        for (int dx = 0; dx < md.xr; ++dx) e += fexist[h + dz * xyn + dy * a.xn + dx];
    pass = e > a.thr;
    if (a.lim) {  // a canvas frame: the position must lie inside the frame's own subdivisions
      const int32_t* L = a.lim + 4 * f;
      pass = pass && x + md.xr <= L[0] && y + md.yr <= L[1] && z + md.zr <= L[2];
    }
    entry = ((int64_t)mi << 40) | p;
    if (!pass && prev != -1.0)  // (a dense fill without sparse_scores: prev is 0)
      for (int m = 0; m < a.M; ++m) fscores[md.offset + (int64_t)m * md.P + p] = -1.0;
  }
  const unsigned long long m = __ballot(pass);
  if (m) {
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&fcnt[a.epoch & 1], (uint32_t)__popcll(m));
    base = __shfl(base, 0, 64);
    if (pass) flist[base + __popcll(m & ((1ull << lane) - 1))] = entry;
  }
}

// box sums of G for every position of every mode (large grids): thread = (position, d4);
// the cells in the score body's (dz, dy, dx) order, rows of empty subdivisions skipped,
// so each sum is the one the score body would form
__device__ __forceinline__ void boxsum_body(const SparseSearch& a, int64_t e, int64_t f) {
  const int D4 = a.D >> 2;
  const int64_t g = e / D4;
  const int d4 = (int)(e - g * D4);
  if (g >= a.pstart[a.nmodes]) return;
  const int mi = find_mode(a, g);
  const ModeGeom& md = a.md[mi];
  const int64_t p = g - a.pstart[mi];
  const int64_t xye = (int64_t)md.xe * md.ye;
  const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
  const int xyn = a.xn * a.yn;
  const int h = z * xyn + y * a.xn + x;
  const int32_t* __restrict__ fexist = a.exist + f * a.s_exist;
  const float4* G4 = reinterpret_cast<const float4*>(a.G + f * a.s_G);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int dz = 0; dz < md.zr; ++dz)
    for (int dy = 0; dy < md.yr; ++dy)
      for (int dx = 0; dx < md.xr; ++dx) {
        const int hh = h + dz * xyn + dy * a.xn + dx;
        if (!a.skip_empty || fexist[hh] != 0) {
          const float4 v = G4[(int64_t)hh * D4 + d4];
          s.x += v.x;
          s.y += v.y;
          s.z += v.z;
          s.w += v.w;
        }
      }
  reinterpret_cast<float4*>(a.gbox + f * a.s_gbox)[g * D4 + d4] = s;
}

// Rank-1 replay fused into the score launch (search.cpp:464-474 with rank_num == 1:
// checkOverlap returns slot 0, so the update is "first strictly greater maximum in scan
// order").  One wave per model reduces the partials with (score desc, scan order asc);
// partials of other workgroups are read with device-scope atomic loads.
// Models w, w + stride, ... of wave w (the standalone kernel spreads the models over
// workgroups: model_base = blockIdx.x * 4, stride = gridDim.x * 4).
__device__ void argmax_finalize(const SparseSearch& a, const ScorePartial* partials, c3h_det* lists,
                                c3h_det* out, int nparts, int model_base = 0, int model_stride = kBlock / 64) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int m = model_base + w; m < a.M; m += model_stride) {
    double best = -2.0;
    long long bo = -1;
    for (int i = lane; i < nparts; i += 64) {
      const ScorePartial* q = partials + (int64_t)i * a.M + m;
      const long long qo = __hip_atomic_load(&q->order, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const double qs = __hip_atomic_load(&q->score, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (qo >= 0 && (qs > best || (qs == best && qo < bo))) {
        best = qs;
        bo = qo;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double os = __shfl_xor(best, o, 64);
      const long long oo = __shfl_xor(bo, o, 64);
      if (oo >= 0 && (os > best || (os == best && (bo < 0 || oo < bo)))) {
        best = os;
        bo = oo;
      }
    }
    if (lane == 0) {
      c3h_det e = lists[m];
      if (a.clean) {  // 1: cleanMax (modes kept, search.cpp:683-690); 2: setRank state
        e.score = 0.0;
        e.x = e.y = e.z = 0;
        if (a.clean == 2) e.mode = 0;
      }
      if (bo >= 0 && best > e.score) {
        const int mi = (int)(bo >> 40);
        const int64_t p = bo & ((1ll << 40) - 1);
        const ModeGeom& md = a.md[mi];
        e.score = best;
        e.x = (int)(p % md.xe);
        e.y = (int)((p / md.xe) % md.ye);
        e.z = (int)(p / ((int64_t)md.xe * md.ye));
        e.mode = md.mode;
      }
      lists[m] = e;
      if (out) out[m] = e;
    }
  }
}

// Fast-path projection over the gate list:
// kFP entries per workgroup; box rows of empty subdivisions are skipped (their G rows
// may be stale: the sparse compress only writes non-empty rows; an all-zero row adds
// nothing to a sum that starts at +0).
// LDS bytes of the score body: feature/projection region, basis window, per-position
// scratch, per-block best scores, the last-workgroup flag
__host__ __device__ inline size_t score_list_lds_bytes(int D, int mpg) {
  const size_t region = ((size_t)D * kFP > (size_t)kFP * (kOC + 1) ? (size_t)D * kFP : (size_t)kFP * (kOC + 1)) +
                        (size_t)D * kOC;
  return sizeof(float) * (region + kFP) + sizeof(int) * 4 * kFP + sizeof(long long) * kFP +
         sizeof(double) * kFP * mpg + 16 + 16;
}

// block (bx, by, fz) of a (gdx, gdy, frames) launch; smem: score_list_lds_bytes(D, mpg)
__device__ __forceinline__ void score_list_body(const SparseSearch& b, int bx, int by, int fz_, int gdx, int gdy,
                                                float* ssm) {
  const SparseSearch& a = b;  // frame-independent fields; per-frame pointers below
  const int64_t fz = fz_;
  const float* __restrict__ fG = b.G + fz * b.s_G;
  const int32_t* __restrict__ fexist = b.exist + fz * b.s_exist;
  double* __restrict__ fscores = b.scores + fz * b.s_scores;
  const long long* __restrict__ flist = b.list + fz * b.s_list;
  const uint32_t* fcnt = b.cnt + fz * b.s_cnt;
  uint32_t* fdone = b.done + fz * b.s_cnt;
  ScorePartial* fpart = b.partials ? b.partials + fz * b.s_partials : nullptr;
  c3h_det* flists = b.lists ? b.lists + fz * b.s_lists : nullptr;
  c3h_det* fout = b.outs[fz];
  long long* fprof = fz ? nullptr : b.prof;
  const int D = a.D, D4 = a.D >> 2, Qs = a.Opad;  // qt row stride
#define C3H_SPROF(k) \
  if (fprof && threadIdx.x == 0 && by == 0) fprof[bx * 8 + (k)] = (long long)wall_clock64()
  C3H_SPROF(0);
  const int tid = threadIdx.x;
  // issued together: the list count, this workgroup's first list chunk (speculative: the
  // list buffer holds P_total entries, entries past the count are ignored) and the
  // group's basis window, so the count costs no extra round trip
  const int64_t ptot = a.pstart[a.nmodes];
  long long en_first = -1;
  if (tid < kFP) en_first = flist[min((int64_t)bx * kFP + tid, ptot - 1)];
  // model group(s) of this workgroup: group by (models [by*mpg, ...)), or with group_loop
  // every group in turn over the same box sums (one workgroup per list chunk: the box-sum
  // gathers run once instead of once per group)
  const int ngl = a.group_loop ? (a.M + a.mpg - 1) / a.mpg : 1;
  const int fts = max(D * kFP, kFP * (kOC + 1));
  // the group's basis window goes straight to LDS (global_load_lds: no VGPR staging, the
  // score role would otherwise spill in the tick kernel); element e = j*kBlock + tid lands
  // at qw[e] (wave-uniform base + lane*4); retired by a vmcnt(0) before the GEMM barrier
  auto issue_window = [&](int grp) {
    constexpr int kQW = 160 * kOC / kBlock;  // window floats per lane at the largest D
    const int g0 = grp * a.mpg, g1 = min(a.M, g0 + a.mpg);
    const int row0 = g0 * a.r, oc = ((g1 - g0) * a.r + 15) & ~15;  // <= kOC
    float* qwl = ssm + fts;
    const int wave = tid >> 6;
#pragma unroll 4
    for (int j = 0; j < kQW; ++j) {
      const int e = j * kBlock + tid, d = e / oc, o = e - d * oc;
      if (j * kBlock >= D * oc) break;  // uniform
      if (e < D * oc)
        __builtin_amdgcn_global_load_lds(a.qt + (int64_t)d * Qs + row0 + o, qwl + j * kBlock + wave * 64, 4, 0, 0);
    }
  };
  issue_window(by);
  const int n = (int)fcnt[a.epoch & 1];
  const int nch = (n + kFP - 1) / kFP;  // list chunks; chunk c -> workgroups c mod gdx
  if (bx >= nch) {
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
    if (n == 0 && flists && bx == 0 && by == 0) argmax_finalize(a, fpart, flists, fout, 0);  // clean / copy out
    return;
  }
  float* fT = ssm;                    // D x kFP (k-major box features)
  float* qw = ssm + fts;              // D x oc: this group's whole basis window
  // kFP x (kOC+1) projections after the GEMM: over fT, or with group_loop (fT serves every
  // group) over the window (the host checks D * kOC >= kFP * (kOC + 1))
  float* qv = a.group_loop ? qw : ssm;
  float* ffv = qw + D * kOC;
  int* gate = reinterpret_cast<int*>(ffv + kFP);
  int* hrow = gate + kFP;
  int* rng = hrow + kFP;                       // packed xr | yr << 10 | zr << 20
  long long* ent = reinterpret_cast<long long*>(rng + kFP + (kFP & 1));
  double* bsc = reinterpret_cast<double*>(ent + kFP);  // kFP * mpg
  const int xyn = a.xn * a.yn;
  for (int ch = bx; ch < nch; ch += gdx) {
    const int64_t e0 = (int64_t)ch * kFP;
    if (tid < kFP) {
      const int64_t e = e0 + tid;
      int ok = 0, h = 0, rr = 0;
      long long en = -1;
      if (e < n) {
        en = ch == bx ? en_first : flist[e];
        const int mi = (int)(en >> 40);
        const int64_t p = en & ((1ll << 40) - 1);
        const ModeGeom& md = a.md[mi];
        const int64_t xye = (int64_t)md.xe * md.ye;
        const int x = (int)(p % md.xe), y = (int)((p / md.xe) % md.ye), z = (int)(p / xye);
        h = z * xyn + y * a.xn + x;
        rr = md.xr | (md.yr << 10) | (md.zr << 20);
        ok = 1;
      }
      gate[tid] = ok;
      hrow[tid] = h;
      rng[tid] = rr;
      ent[tid] = en;
    }
    lds_barrier();
    C3H_SPROF(1);
    if (b.gbox) {  // precomputed box sums (boxsum_kernel): one row per position
      const float4* B4 = reinterpret_cast<const float4*>(b.gbox + fz * b.s_gbox);
      for (int e = tid; e < kFP * D4; e += kBlock) {
        const int pp = e & (kFP - 1), d4 = e / kFP;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gate[pp]) {
          const long long en = ent[pp];
          v = B4[(a.pstart[(int)(en >> 40)] + (en & ((1ll << 40) - 1))) * D4 + d4];
        }
        fT[(4 * d4 + 0) * kFP + pp] = v.x;
        fT[(4 * d4 + 1) * kFP + pp] = v.y;
        fT[(4 * d4 + 2) * kFP + pp] = v.z;
        fT[(4 * d4 + 3) * kFP + pp] = v.w;
      }
    } else {  // box sums in the fixed (dz, dy, dx) order over non-empty rows; lane = position.
       // Cells go in batches of 4 x (this thread's d4 slots): every load of a batch is in
       // flight together.  Rows of empty subdivisions read as 0 (their G rows may be stale;
       // +0 added to a sum that starts at +0 changes nothing) -- for C3 extracts, where
       // exist 0 means empty (skip_empty); other features add every row.
      const int pp = tid & (kFP - 1), dg = tid / kFP;
      constexpr int kDG = kBlock / kFP;  // d4 stride
      const bool ok = gate[pp];
      const int h = hrow[pp], rr = rng[pp];
      const int xr = rr & 1023, yr = (rr >> 10) & 1023, zr = rr >> 20;
      const int ncell = ok ? xr * yr * zr : 0;
      const float4* G4 = reinterpret_cast<const float4*>(fG);
      constexpr int kSlots = 4;  // d4 values per thread handled together (D4 <= 64)
      constexpr int kCB = C3H_SCORE_CB;  // box cells whose loads are in flight together
      float4 s[kSlots];
#pragma unroll
      for (int q = 0; q < kSlots; ++q) s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int d4b = 0; d4b < D4; d4b += kSlots * kDG) {
        for (int c0 = 0; c0 < ncell; c0 += kCB) {
          float4 g[kCB][kSlots];
          bool lv[kCB];
#pragma unroll
          for (int k = 0; k < kCB; ++k) {
            const int c = c0 + k;
            const int dx = c % xr, dy = (c / xr) % yr, dz = c / (xr * yr);
            const int hh = h + dz * xyn + dy * a.xn + dx;
            lv[k] = c < ncell && (!a.skip_empty || fexist[c < ncell ? hh : h] != 0);
#pragma unroll
            for (int q = 0; q < kSlots; ++q) {
              const int d4 = d4b + dg + q * kDG;
              g[k][q] = (c < ncell && d4 < D4) ? G4[(int64_t)hh * D4 + d4] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
          }
#pragma unroll
          for (int k = 0; k < kCB; ++k)
#pragma unroll
            for (int q = 0; q < kSlots; ++q)
              if (lv[k]) {
                s[q].x += g[k][q].x;
                s[q].y += g[k][q].y;
                s[q].z += g[k][q].z;
                s[q].w += g[k][q].w;
              }
        }
#pragma unroll
        for (int q = 0; q < kSlots; ++q) {
          const int d4 = d4b + dg + q * kDG;
          if (d4 < D4) {
            fT[(4 * d4 + 0) * kFP + pp] = s[q].x;
            fT[(4 * d4 + 1) * kFP + pp] = s[q].y;
            fT[(4 * d4 + 2) * kFP + pp] = s[q].z;
            fT[(4 * d4 + 3) * kFP + pp] = s[q].w;
          }
          s[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the basis window's LDS-DMA (first chunk)
    lds_barrier();
    C3H_SPROF(2);
    if (tid < kFP) {
      float s = 0.0f;
      for (int d = 0; d < D; ++d) s = __builtin_fmaf(fT[d * kFP + tid], fT[d * kFP + tid], s);
      ffv[tid] = s;
    }
    for (int gi = 0; gi < ngl; ++gi) {
      const int grp = by + gi;  // by == 0 with group_loop
      const int m0 = grp * a.mpg, m1 = min(a.M, m0 + a.mpg);
      const int oc = ((m1 - m0) * a.r + 15) & ~15;  // <= kOC
      if (a.group_loop && (gi > 0 || ch != bx)) {  // this group's window is not in LDS yet
        lds_barrier();  // the previous group's projections (aliasing the window) are read
        issue_window(grp);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
      }
      // GEMM: thread (tp, to): positions 2*tp, 2*tp+1; basis rows 4*to .. 4*to+3 of the group
      const int tp = tid & 15, to = tid >> 4;
      const bool active = 4 * to < oc;
      float acc[2][4];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = 0.0f;
      if (active) {
#pragma unroll 4
        for (int d = 0; d < D; ++d) {
          const float2 f = *reinterpret_cast<const float2*>(&fT[d * kFP + 2 * tp]);
          const float4 q = *reinterpret_cast<const float4*>(&qw[d * oc + 4 * to]);
          acc[0][0] = __builtin_fmaf(f.x, q.x, acc[0][0]);
          acc[0][1] = __builtin_fmaf(f.x, q.y, acc[0][1]);
          acc[0][2] = __builtin_fmaf(f.x, q.z, acc[0][2]);
          acc[0][3] = __builtin_fmaf(f.x, q.w, acc[0][3]);
          acc[1][0] = __builtin_fmaf(f.y, q.x, acc[1][0]);
          acc[1][1] = __builtin_fmaf(f.y, q.y, acc[1][1]);
          acc[1][2] = __builtin_fmaf(f.y, q.z, acc[1][2]);
          acc[1][3] = __builtin_fmaf(f.y, q.w, acc[1][3]);
        }
      }
      lds_barrier();  // qv aliases fT (or the window, with group_loop)
      C3H_SPROF(3);
      if (active) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) qv[(2 * tp + i) * (kOC + 1) + 4 * to + q] = acc[i][q];
      }
      lds_barrier();
      const int nm = m1 - m0;
      for (int e = tid; e < kFP * nm; e += kBlock) {
        const int mm = e / kFP, pp = e - mm * kFP;
        double sc = -2.0;
        if (gate[pp]) {
          float q2 = 0.0f;
          const float* q = qv + pp * (kOC + 1) + mm * a.r;
#pragma unroll 4  // reads issued four at a time (a dependent LDS round trip per element otherwise)
          for (int i = 0; i < a.r; ++i) q2 = __builtin_fmaf(q[i], q[i], q2);
          sc = sqrt((double)q2) / sqrt((double)ffv[pp]);
          const long long en = ent[pp];
          const ModeGeom& md = a.md[(int)(en >> 40)];
          fscores[md.offset + (int64_t)(m0 + mm) * md.P + (en & ((1ll << 40) - 1))] = sc;
        }
        bsc[e] = sc;
      }
      C3H_SPROF(4);
      if (fpart) {
        lds_barrier();
        for (int mm = tid; mm < nm; mm += kBlock) {  // (score desc, scan order asc)
          double best = -2.0;
          long long bo = -1;
          for (int pp = 0; pp < kFP; ++pp) {
            if (!gate[pp]) continue;
            const double sc = bsc[mm * kFP + pp];
            const long long en = ent[pp];
            const long long o = a.order_base[(int)(en >> 40)] + (en & ((1ll << 40) - 1));
            if (sc > best || (sc == best && o < bo)) {
              best = sc;
              bo = o;
            }
          }
          ScorePartial* q = fpart + (int64_t)ch * a.M + m0 + mm;
          if (flists) {  // handed to another workgroup inside this launch: sc1 stores
            __hip_atomic_store(&q->score, best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&q->order, bo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } else {
            *q = ScorePartial{best, bo};
          }
        }
      }
    }
    lds_barrier();  // LDS is reused by the next chunk
  }
  if (fpart && flists) {
    // rank 1, fused replay: the last workgroup to finish reduces.  Hand-off per
    // MI355X_MICROARCH.md (inter-workgroup visibility, table row 1): sc1 stores, every
    // storing wave waits vmcnt(0), a barrier, one agent atomic add per workgroup; the
    // workgroup whose add returns total-1 reads the partials with sc1 loads.
    int& s_last = *reinterpret_cast<int*>(reinterpret_cast<char*>(ssm) + score_list_lds_bytes(D, a.mpg) - 16);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lds_barrier();
    if (tid == 0) {
      const uint32_t total = (uint32_t)min(nch, gdx) * gdy;
      s_last = atomicAdd(&fdone[a.epoch & 1], 1u) == total - 1;
    }
    lds_barrier();
    if (s_last) argmax_finalize(a, fpart, flists, fout, nch);
  }
  C3H_SPROF(7);
}

}  // namespace c3h
