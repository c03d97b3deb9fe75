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
constexpr int kMfLoad = 2;  // (row, dword) pairs per lane of a layer (<= 18 rows x 5 dwords)
constexpr int kMfTyMax = 18;
#ifndef C3H_MF_EXP
#define C3H_MF_EXP 0  // diagnostics variants: 1 no K steps, 2 no conversion
#endif

__host__ __device__ inline int mf_slot_bytes(int ty) { return kMfCh * ty * kMfRowB; }
// per wave: 2 constant planes (rows 12..15 of A / columns 12..15 of B: zeros, and ones
// in 15), then 3 plane slots or (aliasing them) the epilogue's accumulator tiles
constexpr int kMfConstBytes = 2 * kMfTyMax * kMfRowB;
__host__ __device__ inline int mf_wave_bytes(int ty) {
  const int work = 3 * mf_slot_bytes(ty), epi = kMfK * 256 * 4;
  return kMfConstBytes + (((work > epi ? work : epi) + 15) & ~15);
}
// 3 x 256 channel-byte tables | 984 epilogue bin codes | per-wave regions
__host__ __device__ inline size_t mf_lds_bytes(int ty) { return 3072 + 3936 + (size_t)kMfWaves * mf_wave_bytes(ty); }

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

// channel plane of (type t: 0 colour LUT / 1 binary, reference channel c in 0..5): the
// planes hold per colour col the bytes {sin, cos, beta, 1 - beta} (4 col + s)
__host__ __device__ inline int mf_plane(int t, int c) { return 4 * (c >> 1) + 2 * t + (c & 1); }

// epilogue code of bin e (0..980): bin | kind << 10 | k << 12 | c << 16 | n << 20, kind 0 =
// product bin (offset k's tile at plane c, plane n), 1 = zero order (plane c's row sum)
__device__ inline uint32_t mf_bin_code(int e) {
  int bin, kind = 0, k = 13, c, nn;
  if (e < 936) {  // first order: k, type (colour / binary), c, n
    k = e / 72;
    const int rem = e - 72 * k, ty = rem / 36, cc = (rem % 36) / 6, n6 = rem % 6;
    bin = 495 * ty + bin981(k, cc, n6);
    c = mf_plane(ty, cc);
    nn = mf_plane(ty, n6);
  } else if (e < 957) {  // centre auto products (c <= n)
    const int q = e - 936;
    int cc = 0;
    while (q >= tri6(cc + 1, cc + 1)) ++cc;
    bin = 474 + q;
    c = mf_plane(0, cc);
    nn = mf_plane(0, cc + (q - tri6(cc, cc)));
  } else if (e < 969) {  // centre bin-pair counts
    const int q = e - 957;
    const int cc = q < 8 ? q / 4 : 2 + (q - 8) / 2, n6 = q < 8 ? 2 + q % 4 : 4 + (q - 8) % 2;
    bin = 969 + q;
    c = mf_plane(1, cc);
    nn = mf_plane(1, n6);
  } else {  // zero order: colour channels, then binary counts
    const int q = e - 969;
    bin = q < 6 ? q : 495 + (q - 6);
    kind = 1;
    c = mf_plane(q < 6 ? 0 : 1, q < 6 ? q : q - 6);
    nn = 15;
  }
  return (uint32_t)bin | ((uint32_t)kind << 10) | ((uint32_t)k << 12) | ((uint32_t)c << 16) | ((uint32_t)nn << 20);
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
  uint32_t* s_bins = smem + 768;
  for (int i = threadIdx.x; i < 768; i += kBlock) {
    const int col = i >> 8, v = i & 255;
    const uint32_t l = a.lut[v];
    const int thr = col == 0 ? a.thr_r : (col == 1 ? a.thr_g : a.thr_b);
    const uint32_t be = v > thr ? 1u : 0u;
    s_tab[i] = ((l & 0xffu) | (l & 0xff00u) | (be << 16) | ((be ^ 1u) << 24)) ^ 0x80808080u;
  }
  for (int e = threadIdx.x; e < 981; e += kBlock) s_bins[e] = mf_bin_code(e);
  uint8_t* cplanes = reinterpret_cast<uint8_t*>(smem + 768 + 984) + (size_t)wave * mf_wave_bytes(a.mf_ty);
  uint8_t* wl = cplanes + kMfConstBytes;  // 3 layer slots, or the epilogue
  uint8_t* planes = wl;
  for (int i = lane; i < 2 * kMfTyMax * kMfRowB / 4; i += 64)
    reinterpret_cast<uint32_t*>(cplanes)[i] = i >= kMfTyMax * kMfRowB / 4 ? 0x01010101u : 0u;
  __syncthreads();
  const int nwork = (int)ftf[2 + (a.epoch & 1)];
  if (2 * nwork < a.ntiles) return;  // sparse frame: the dot4 tile body takes it
  const int F = a.variant;
  const int h4 = lane >> 4, n = lane & 15;
  const bool real = n < kMfCh;

  for (int wi = wid; wi < nwork; wi += nw) {
    const int tile = fwork[wi];
    const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
    const int32_t* sx = a.segs + 3 * ix;
    const int32_t* sy = a.segs + 3 * (a.seg_stride + iy);
    const int32_t* sz = a.segs + 3 * (2 * a.seg_stride + iz);
    const int x0 = sx[0], lx = sx[1], y0 = sy[0], ly = sy[1], z0 = sz[0], lz = sz[1];
    const int64_t h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
    const int TY = ly + 2, nks = (ly + 3) >> 2, npair = TY * 5;
    const int sb = mf_slot_bytes(TY);
    // layer words in registers: (row, dword q) pairs e = lane + 64 i, x = x0 - 1 + 4 q + j;
    // two layers in flight
    uint32_t wv[2][kMfLoad][4];
    auto load_layer = [&](int L, uint32_t (&w)[kMfLoad][4]) {
      const int gz = z0 - 1 + L;
#pragma unroll
      for (int i = 0; i < kMfLoad; ++i) {
        const int e = lane + 64 * i, row = e / 5, q = e - row * 5;
        const int gy = y0 - 1 + row;
        const bool rowin = e < npair && (unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz;
        const uint32_t* src = fgrid + ((int64_t)gz * a.gy + gy) * a.gx;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gxx = x0 - 1 + 4 * q + j;
          w[i][j] = rowin && (unsigned)gxx < (unsigned)a.gx ? src[gxx] : 0u;
        }
      }
    };
    // 12 channel planes of layer L: per voxel and colour one table read gives the 4 channel
    // bytes, a 4 x 4 byte transpose packs them per channel (4 voxels per dword)
    auto store_layer = [&](int L, const uint32_t (&w)[kMfLoad][4]) {
#if C3H_MF_EXP & 2
      return;
#endif
      uint8_t* slot = planes + (size_t)(L % 3) * sb;
#pragma unroll
      for (int i = 0; i < kMfLoad; ++i) {
        const int e = lane + 64 * i, row = e / 5, q = e - row * 5;
        if (e >= npair) continue;
        uint32_t t[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int col = 0; col < 3; ++col)
            t[col][j] = w[i][j] ? s_tab[col * 256 + ((w[i][j] >> (16 - 8 * col)) & 0xffu)] : 0x80808080u;
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
    // centre mask of A: bytes j >= lx are no centre (a = 0 -> 0x80); the constant lanes keep all
    uint32_t keep[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) m |= (4 * d + b < lx ? 0xffu : 0u) << (8 * b);
      keep[d] = real ? m : 0xffffffffu;
    }
    mf_v4i acc[kMfK];
#pragma unroll
    for (int k = 0; k < kMfK; ++k) acc[k] = mf_v4i{0, 0, 0, 0};
    load_layer(0, wv[0]);
    load_layer(1, wv[1]);
    store_layer(0, wv[0]);
    store_layer(1, wv[1]);
    if (2 <= lz) load_layer(2, wv[0]);
    if (3 <= lz) load_layer(3, wv[1]);
    for (int z = 0; z < lz; ++z) {
      wave_lds_sync();
      const uint8_t* sp = planes + (size_t)(z % 3) * sb;        // dz = -1
      const uint8_t* sc = planes + (size_t)((z + 1) % 3) * sb;  // dz = 0
      // padding lanes read the constant planes (their rows are the same for every layer)
      const uint8_t* pc = real ? sc + (size_t)n * TY * kMfRowB : cplanes + (n == 15 ? kMfTyMax * kMfRowB : 0);
      const uint8_t* pp = real ? sp + (size_t)n * TY * kMfRowB : pc;
      for (int ks = 0; ks < ((C3H_MF_EXP & 1) ? 0 : nks); ++ks) {
        const int y = 4 * ks + h4;
        const bool ym = y < ly;
        const int rm = min(y, TY - 1), rc = min(y + 1, TY - 1), rp = min(y + 2, TY - 1);
        auto row = [&](const uint8_t* plane, int r, uint4& lo, uint4& hi) {
          lo = *reinterpret_cast<const uint4*>(plane + r * kMfRowB);
          hi = *reinterpret_cast<const uint4*>(plane + r * kMfRowB + 16);
        };
        uint4 lo, hi;
        row(pc, rc, lo, hi);
        mf_v4i A = mf_frag(lo, hi, 1);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t m = (ym || !real) ? keep[d] : 0u;
          A[d] = (int)(((uint32_t)A[d] & m) | (0x80808080u & ~m));
        }
        acc[13] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, A, acc[13], 0, 0, 0);  // own channels
        acc[12] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, mf_frag(lo, hi, 0), acc[12], 0, 0, 0);  // (-1, 0, 0)
        row(pc, rm, lo, hi);  // (dx, -1, 0): k = 9 + dx + 1
#pragma unroll
        for (int dxi = 0; dxi < 3; ++dxi)
          acc[9 + dxi] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, mf_frag(lo, hi, dxi), acc[9 + dxi], 0, 0, 0);
        // (dx, dy, -1): k = 3 (dx + 1) + (dy + 1)
#pragma unroll
        for (int dyi = 0; dyi < 3; ++dyi) {
          row(pp, dyi == 0 ? rm : (dyi == 1 ? rc : rp), lo, hi);
#pragma unroll
          for (int dxi = 0; dxi < 3; ++dxi)
            acc[3 * dxi + dyi] =
                __builtin_amdgcn_mfma_i32_16x16x64_i8(A, mf_frag(lo, hi, dxi), acc[3 * dxi + dyi], 0, 0, 0);
        }
      }
      // layer z + 2 into the plane slot of layer z - 1 (loaded two layers ago), then the
      // loads of layer z + 4 into its registers
      if (z + 2 <= lz) {
        if (z & 1) {
          store_layer(z + 2, wv[1]);
          if (z + 4 <= lz) load_layer(z + 4, wv[1]);
        } else {
          store_layer(z + 2, wv[0]);
          if (z + 4 <= lz) load_layer(z + 4, wv[0]);
        }
      }
    }
    wave_lds_sync();
    // epilogue: accumulator tiles -> LDS (C/D map: row 4 (lane >> 4) + r, column lane & 15);
    // the bins are formed from them directly (exact corrected sums, then the reference's
    // normalisation / the 117 fold)
    int32_t* T = reinterpret_cast<int32_t*>(wl);
#pragma unroll
    for (int k = 0; k < kMfK; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[k * 256 + (4 * h4 + r) * 16 + n] = acc[k][r];
    wave_lds_sync();
    const long long K = T[13 * 256 + 255];
    auto corr = [&](int k, int c, int nn) -> long long {
      const int32_t* Tk = T + k * 256;
      return (long long)Tk[c * 16 + nn] + 128ll * ((long long)Tk[c * 16 + 15] + Tk[15 * 16 + nn]) + 16384ll * K;
    };
    auto code_value = [&](uint32_t code) -> uint32_t {
      const int kind = (code >> 10) & 3, k = (code >> 12) & 15, c = (code >> 16) & 15, nn = (code >> 20) & 15;
      return (uint32_t)(kind ? (long long)T[k * 256 + c * 16 + 15] + 128ll * K : corr(k, c, nn));
    };
    if (a.atomic) {
      for (int e = lane; e < 981; e += 64) {
        const uint32_t code = s_bins[e], v = code_value(code);
        if (v) atomicAdd(&facc[h * 981 + (code & 1023)], (unsigned long long)v);
      }
    } else {
      float* out = ffeat + h * F;
      if (F == 981) {
        for (int e = lane; e < 981; e += 64) {
          const uint32_t code = s_bins[e];
          const int bin = code & 1023;
          out[bin] = (float)code_value(code) * norm981(bin);
        }
      } else {  // color_chlac.hpp:1647-1743: first-order bins summed over the 13 offsets
        for (int i = lane; i < 117; i += 64) {
          uint32_t v;
          if (i < 6 || (i >= 63 && i < 69)) {  // zero order
            const int t = i < 6 ? 0 : 1, c = i < 6 ? i : i - 63;
            v = (uint32_t)((long long)T[13 * 256 + mf_plane(t, c) * 16 + 15] + 128ll * K);
          } else if (i < 42 || (i >= 69 && i < 105)) {  // first order, all offsets
            const int t = i < 42 ? 0 : 1, q = i < 42 ? i - 6 : i - 69, c = q / 6, nn = q % 6;
            long long sum = 0;
            for (int k = 0; k < 13; ++k) sum += corr(k, mf_plane(t, c), mf_plane(t, nn));
            v = (uint32_t)sum;
          } else {  // centre auto products / bin-pair counts: codes 936.. / 957..
            v = code_value(s_bins[i < 63 ? 936 + (i - 42) : 957 + (i - 105)]);
          }
          out[i] = (float)v * norm117(i);
        }
      }
      if (lane == 0) {  // exist_voxel_num from the zero-order r sums (search_c3_hlac.h:60-61)
        const uint32_t s0 = (uint32_t)((long long)T[13 * 256 + mf_plane(0, 0) * 16 + 15] + 128ll * K);
        const uint32_t s1 = (uint32_t)((long long)T[13 * 256 + mf_plane(0, 1) * 16 + 15] + 128ll * K);
        fexist[h] = exist_from((float)s0, (float)s1);
      }
    }
    if (frows && lane == 0) frows[wi] = (int32_t)h;
    wave_lds_sync();  // the tile's LDS is rebuilt by the next tile
  }
}

}  // namespace c3h
