// c3hlac_mfma.h -- dense C3-HLAC tiles on the i8 matrix cores (v_mfma_i32_16x16x64_i8).
//
// Same result as the dot4 tile body (c3hlac_dev.h), for tiles whose centre voxels are
// mostly occupied (config 5: 512^3 at 100 %), where compacting occupied voxels saves
// nothing.  Every bin is an exact integer correlation over the tile's centre voxels v
//   C_k[c][n] = sum_v X_c(v) * Y_n(v + r_k)
// of 12 channels (6 sin/cos LUT colour bytes r,r_,g,g_,b,b_ and 6 binary beta, 1-beta;
// all 0 for empty voxels) with the 13 half-neighbourhood offsets r_k (c3_hlac.cpp:177-202)
// plus k = 13, the centre's own channels (auto products, bin-pair counts).  That is one
// 16 x 16 x K integer GEMM per k with K = centre voxels:
//   A = X (row c = channel, 12 of 16 rows), B_k = Y shifted by r_k (column n = channel).
// u8 channel values are stored offset by -128 (byte ^ 0x80), which i8 holds exactly, and
// the exact sums are recovered with the tile's own row / column sums, which the padding
// rows / columns compute for free: row 15 of A and column 15 of B are constant 1, so
//   sum a b = C[c][n] + 128 (C[c][15] + C[15][n]) + 128^2 C[15][15]
// (an empty or masked position carries a = 0, i.e. -128, and the identity holds
// elementwise).  i32 accumulation is exact (|a' b'| <= 2^14, K <= 16 * 16 * 16 * 2).
//
// Mapping: one wave per tile (<= 16 x 16 centres per layer), walking the tile's layers
// in z.  Layer L (z = z0 - 1 + L) is built in LDS as 12 channel planes of (ly + 2) rows x
// 32 B (x = -1 at byte 0); a K step covers 4 rows x 16 x (lane group h = lane >> 4 takes
// row y = 4 ks + h, byte j = centre x j), so every A / B fragment of a lane is 16
// consecutive bytes of one plane row: two aligned ds_read_b128 and a byte shift
// (v_alignbyte) give the dx = -1, 0, +1 fragments of a row.  Per K step: 10 LDS reads, 14
// MFMAs.  The next layer's grid words are loaded into registers before the current
// layer's MFMAs and stored after them (three layer slots in a ring).
#pragma once
#include "c3hlac_dev.h"

namespace c3h {

typedef int mf_v4i __attribute__((ext_vector_type(4)));
constexpr int kMfWaves = kBlock / 64;
constexpr int kMfRowB = 32;  // bytes per plane row
constexpr int kMfCh = 12;
constexpr int kMfK = 14;     // 13 offsets + the centre's own channels
constexpr int kMfRaw = 384;  // dwords of one raw layer slot (<= 18 x 18 words, 6 DMA rounds)
constexpr int kMfRawSlots = 4;

__host__ __device__ inline int mf_slot_bytes(int ty) { return kMfCh * ty * kMfRowB; }
__host__ __device__ inline int mf_wave_bytes(int ty) {
  const int work = kMfRawSlots * kMfRaw * 4 + 3 * mf_slot_bytes(ty), epi = (kMfK * 256 + 984) * 4;
  return ((work > epi ? work : epi) + 15) & ~15;
}
// 3 x 256 channel-byte tables | per-wave regions
__host__ __device__ inline size_t mf_lds_bytes(int ty) { return 3072 + (size_t)kMfWaves * mf_wave_bytes(ty); }

// 16 bytes starting at byte s (0..2) of a 32-byte plane row held as two uint4
__device__ __forceinline__ mf_v4i mf_frag(const uint4& lo, const uint4& hi, int s) {
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  mf_v4i f;
  f[0] = (int)__builtin_amdgcn_alignbyte(w[1], w[0], s);
  f[1] = (int)__builtin_amdgcn_alignbyte(w[2], w[1], s);
  f[2] = (int)__builtin_amdgcn_alignbyte(w[3], w[2], s);
  f[3] = (int)__builtin_amdgcn_alignbyte(w[4], w[3], s);
  return f;
}

__device__ __forceinline__ void wave_lds_sync() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// wait until at most n of this wave's vector-memory operations (LDS DMA) are outstanding
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: __asm__ volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: __asm__ volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: __asm__ volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: __asm__ volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: __asm__ volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}

// channel plane of (type t: 0 colour LUT / 1 binary, reference channel c in 0..5): the
// planes hold per colour col the bytes {sin, cos, beta, 1 - beta} (4 col + s)
__device__ __forceinline__ int mf_plane(int t, int c) { return 4 * (c >> 1) + 2 * t + (c & 1); }

// corrected exact sum of tile T at (plane c, plane n)
__device__ __forceinline__ uint32_t mf_corr(const int32_t* T, int c, int n) {
  const long long v = (long long)T[c * 16 + n] + 128ll * ((long long)T[c * 16 + 15] + T[15 * 16 + n]) +
                      16384ll * T[15 * 16 + 15];
  return (uint32_t)v;
}

// wave wid of nw (all waves of this launch for frame fy); smem = mf_lds_bytes(TYmax)
__device__ __forceinline__ void c3hlac_mfma_body(const KArgs& a, int wid, int nw, int fy_, uint32_t* smem) {
  const int64_t fy = fy_;
  const uint32_t* __restrict__ fgrid = a.grids[fy];
  float* __restrict__ ffeat = a.feat + fy * a.s_feat;
  int32_t* __restrict__ fexist = a.exist + fy * a.s_h;
  unsigned long long* facc = a.acc64 ? a.acc64 + fy * a.s_acc : nullptr;
  const uint32_t* ftf = a.tf + fy * a.s_tf;
  const int32_t* __restrict__ fwork = a.work + fy * a.s_work;
  int32_t* frows = a.rows ? a.rows + fy * a.s_h : nullptr;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // channel-byte tables: T_col[v] = {sin, cos, beta, 1 - beta} ^ 0x80 (setColor LUT, thresholds)
  uint32_t* s_tab = smem;
  for (int i = threadIdx.x; i < 768; i += kBlock) {
    const int col = i >> 8, v = i & 255;
    const uint32_t l = a.lut[v];
    const int thr = col == 0 ? a.thr_r : (col == 1 ? a.thr_g : a.thr_b);
    const uint32_t be = v > thr ? 1u : 0u;
    s_tab[i] = ((l & 0xffu) | (l & 0xff00u) | (be << 16) | ((be ^ 1u) << 24)) ^ 0x80808080u;
  }
  __syncthreads();
  const int nwork = (int)ftf[2 + (a.epoch & 1)];
  if (2 * nwork < a.ntiles) return;  // sparse frame: the dot4 tile body takes it
  uint8_t* wl = reinterpret_cast<uint8_t*>(smem + 768) + (size_t)wave * mf_wave_bytes(a.mf_ty);
  uint32_t* raw = reinterpret_cast<uint32_t*>(wl);                       // kMfRawSlots x kMfRaw
  uint8_t* planes = wl + kMfRawSlots * kMfRaw * 4;                       // 3 layer slots
  const int F = a.variant;
  const int h4 = lane >> 4, n = lane & 15;
  const bool real = n < kMfCh;
  const mf_v4i kConst = n == 15 ? mf_v4i{0x01010101, 0x01010101, 0x01010101, 0x01010101} : mf_v4i{0, 0, 0, 0};

  for (int wi = wid; wi < nwork; wi += nw) {
    const int tile = fwork[wi];
    const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
    const int32_t* sx = a.segs + 3 * ix;
    const int32_t* sy = a.segs + 3 * (a.seg_stride + iy);
    const int32_t* sz = a.segs + 3 * (2 * a.seg_stride + iz);
    const int x0 = sx[0], lx = sx[1], y0 = sy[0], ly = sy[1], z0 = sz[0], lz = sz[1];
    const int64_t h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
    const int TY = ly + 2, TX = lx + 2, nks = (ly + 3) >> 2;
    const int nraw = TY * TX, ndma = (nraw + 63) >> 6;
    const int sb = mf_slot_bytes(TY);
    // layer L (z = z0 - 1 + L) -> raw slot L % 4 by LDS DMA: element e = row * TX + xo
    // (off-grid elements read word 0 and are masked at conversion)
    auto dma = [&](int L) {
      const int gz = z0 - 1 + L;
      uint32_t* dst = raw + (L % kMfRawSlots) * kMfRaw;
      for (int i = 0; i < ndma; ++i) {
        const int e = 64 * i + lane, row = e / TX, xo = e - row * TX;
        const int gy = y0 - 1 + row, gxx = x0 - 1 + xo;
        const bool in = e < nraw && (unsigned)gz < (unsigned)a.gz && (unsigned)gy < (unsigned)a.gy &&
                        (unsigned)gxx < (unsigned)a.gx;
        const uint32_t* src = in ? fgrid + ((int64_t)gz * a.gy + gy) * a.gx + gxx : fgrid;
        __builtin_amdgcn_global_load_lds(src, dst + 64 * i, 4, 0, 0);
      }
    };
    // raw layer -> 12 channel planes: (row, dword q) pairs, 4 voxels x = -1 + 4 q + j each;
    // table reads give 4 channel bytes per voxel and colour, a 4 x 4 byte transpose packs
    // them per channel
    auto convert = [&](int L) {
      const int gz = z0 - 1 + L;
      const uint32_t* src = raw + (L % kMfRawSlots) * kMfRaw;
      uint8_t* slot = planes + (size_t)(L % 3) * sb;
      for (int e = lane; e < TY * 5; e += 64) {
        const int row = e / 5, q = e - row * 5;
        const int gy = y0 - 1 + row;
        const bool rin = (unsigned)gz < (unsigned)a.gz && (unsigned)gy < (unsigned)a.gy;
        uint32_t t[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int xo = 4 * q + j, gxx = x0 - 1 + xo;
          const uint32_t w = (rin && xo < TX && (unsigned)gxx < (unsigned)a.gx) ? src[row * TX + xo] : 0u;
#pragma unroll
          for (int col = 0; col < 3; ++col)
            t[col][j] = w ? s_tab[col * 256 + ((w >> (16 - 8 * col)) & 0xffu)] : 0x80808080u;
        }
#pragma unroll
        for (int col = 0; col < 3; ++col) {
          const uint32_t u0 = __builtin_amdgcn_perm(t[col][1], t[col][0], 0x05010400u);
          const uint32_t u1 = __builtin_amdgcn_perm(t[col][1], t[col][0], 0x07030602u);
          const uint32_t u2 = __builtin_amdgcn_perm(t[col][3], t[col][2], 0x05010400u);
          const uint32_t u3 = __builtin_amdgcn_perm(t[col][3], t[col][2], 0x07030602u);
          const uint32_t o[4] = {__builtin_amdgcn_perm(u2, u0, 0x05040100u), __builtin_amdgcn_perm(u2, u0, 0x07060302u),
                                 __builtin_amdgcn_perm(u3, u1, 0x05040100u), __builtin_amdgcn_perm(u3, u1, 0x07060302u)};
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2)
            *reinterpret_cast<uint32_t*>(slot + ((size_t)(4 * col + s2) * TY + row) * kMfRowB + 4 * q) = o[s2];
        }
      }
    };
    // centre mask of A: bytes j >= lx are no centre (a = 0 -> 0x80)
    uint32_t keep[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) m |= (4 * d + b < lx ? 0xffu : 0u) << (8 * b);
      keep[d] = m;
    }
    mf_v4i acc[kMfK];
#pragma unroll
    for (int k = 0; k < kMfK; ++k) acc[k] = mf_v4i{0, 0, 0, 0};
    // prologue: layers 0..3 in flight, 0 and 1 converted
    wait_vm(0);
    for (int L = 0; L <= min(3, lz); ++L) dma(L);
    wait_vm(0);
    convert(0);
    convert(1);
    for (int z = 0; z < lz; ++z) {
      wave_lds_sync();
      const uint8_t* sp = planes + (size_t)(z % 3) * sb;        // dz = -1
      const uint8_t* sc = planes + (size_t)((z + 1) % 3) * sb;  // dz = 0
      const uint8_t* pc = sc + (size_t)(real ? n : 0) * TY * kMfRowB;
      const uint8_t* pp = sp + (size_t)(real ? n : 0) * TY * kMfRowB;
      for (int ks = 0; ks < nks; ++ks) {
        const int y = 4 * ks + h4;
        const bool ymask = y < ly;
        const int rm = min(y, TY - 1), rc = min(y + 1, TY - 1), rp = min(y + 2, TY - 1);
        auto row = [&](const uint8_t* plane, int r, uint4& lo, uint4& hi) {
          lo = *reinterpret_cast<const uint4*>(plane + r * kMfRowB);
          hi = *reinterpret_cast<const uint4*>(plane + r * kMfRowB + 16);
        };
        auto sel = [&](const mf_v4i& f) { return real ? f : kConst; };
        uint4 lo, hi;
        row(pc, rc, lo, hi);
        mf_v4i A = mf_frag(lo, hi, 1);
#pragma unroll
        for (int d = 0; d < 4; ++d)
          A[d] = ymask ? (int)(((uint32_t)A[d] & keep[d]) | (0x80808080u & ~keep[d])) : (int)0x80808080u;
        A = sel(A);
        acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, A, acc[13], 0, 0, 0);  // own channels
        acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, sel(mf_frag(lo, hi, 0)), acc[12], 0, 0, 0);  // (-1, 0, 0)
        row(pc, rm, lo, hi);  // (dx, -1, 0): k = 9 + dx + 1
#pragma unroll
        for (int dxi = 0; dxi < 3; ++dxi)
          acc[9 + dxi] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, sel(mf_frag(lo, hi, dxi)), acc[9 + dxi], 0, 0, 0);
        // (dx, dy, -1): k = 3 (dx + 1) + (dy + 1)
#pragma unroll
        for (int dyi = 0; dyi < 3; ++dyi) {
          row(pp, dyi == 0 ? rm : (dyi == 1 ? rc : rp), lo, hi);
#pragma unroll
          for (int dxi = 0; dxi < 3; ++dxi)
            acc[3 * dxi + dyi] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(A, sel(mf_frag(lo, hi, dxi)), acc[3 * dxi + dyi], 0, 0, 0);
        }
      }
      // layer z + 2 into the plane slot of layer z - 1; its DMA was issued two layers ago
      if (z + 2 <= lz) {
        wait_vm(z + 3 <= lz ? ndma : 0);
        convert(z + 2);
        if (z + 4 <= lz) dma(z + 4);
      }
    }
    wave_lds_sync();
    // epilogue: accumulator tiles -> LDS (C/D map: row 4 (lane >> 4) + r, column lane & 15)
    int32_t* T = reinterpret_cast<int32_t*>(wl);
    uint32_t* hist = reinterpret_cast<uint32_t*>(wl) + kMfK * 256;
#pragma unroll
    for (int k = 0; k < kMfK; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[k * 256 + (4 * h4 + r) * 16 + n] = acc[k][r];
    wave_lds_sync();
    const int32_t* T13 = T + 13 * 256;
    const long long K = T13[255];
    for (int e = lane; e < 981; e += 64) {
      int bin;
      uint32_t v;
      if (e < 936) {  // first order: k, type (colour / binary), c, n
        const int k = e / 72, rem = e - 72 * k, ty = rem / 36, c = (rem % 36) / 6, nn = rem % 6;
        bin = 495 * ty + bin981(k, c, nn);
        v = mf_corr(T + k * 256, mf_plane(ty, c), mf_plane(ty, nn));
      } else if (e < 957) {  // centre auto products (c <= n)
        const int q = e - 936;
        int c = 0;
        while (q >= tri6(c + 1, c + 1)) ++c;
        const int nn = c + (q - tri6(c, c));
        bin = 474 + q;
        v = mf_corr(T13, mf_plane(0, c), mf_plane(0, nn));
      } else if (e < 969) {  // centre bin-pair counts
        const int q = e - 957;
        const int c = q < 8 ? q / 4 : 2 + (q - 8) / 2, nn = q < 8 ? 2 + q % 4 : 4 + (q - 8) % 2;
        bin = 969 + q;
        v = mf_corr(T13, mf_plane(1, c), mf_plane(1, nn));
      } else {  // zero order: colour channels, then binary counts
        const int q = e - 969;
        bin = q < 6 ? q : 495 + (q - 6);
        v = (uint32_t)((long long)T13[mf_plane(q < 6 ? 0 : 1, q < 6 ? q : q - 6) * 16 + 15] + 128ll * K);
      }
      hist[bin] = v;
    }
    wave_lds_sync();
    if (a.atomic) {
      for (int i = lane; i < 981; i += 64) {
        const uint32_t v = hist[i];
        if (v) atomicAdd(&facc[h * 981 + i], (unsigned long long)v);
      }
    } else {
      float* out = ffeat + h * F;
      if (F == 981) {
        for (int i = lane; i < 981; i += 64) out[i] = (float)hist[i] * norm981(i);
      } else {
        for (int i = lane; i < 117; i += 64) out[i] = (float)fold117(hist, i) * norm117(i);
      }
      if (lane == 0) fexist[h] = exist_from((float)hist[0], (float)hist[1]);
    }
    if (frows && lane == 0) frows[wi] = (int32_t)h;
    wave_lds_sync();  // the tile's LDS is rebuilt by the next tile
  }
  wait_vm(0);  // no LDS DMA outlives the wave
}

}  // namespace c3h
