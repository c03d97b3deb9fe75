// c3hlac.hip -- C3-HLAC (colour cubic higher-order local auto-correlation) on gfx950.
//
// Replaces C3HLAC{981,117}Estimation::computeFeature (c3_hlac/src/c3_hlac.cpp:252-416)
// and the binary-only c3_hlac_core kernel (c3_hlac_core/include/c3_hlac_core/
// c3_hlac_core.h:44-53), whose arithmetic is the open twin color_chlac.hpp:168-1781.
//
// Formulation.  Per occupied centre voxel v the reference adds, for each of the 13
// half-neighbourhood offsets k (c3_hlac.cpp:177-202) with an occupied neighbour w,
//   a_c(v) * a_n(w)  into bin(k,c,n)   (6x6 colour channels r,r_,g,g_,b,b_ from the
//                                       sin/cos LUT of setColor)
//   b_c(v) * b_n(w)  into 495+bin(k,c,n) (binarised channels b,1-b)
// plus zero-order terms.  Every bin is therefore sum_v X(v) * Y(v) for two byte-valued
// per-voxel "channels"; with four voxels packed per dword one v_dot4_u32_u8 does four
// voxel-MACs exactly in integers.  All 981 bins are the 180 (type, k, n) columns x 6
// centre channels c of
//   k = 0..12  neighbour k's channel n (0 when the neighbour is empty / off-grid)
//   k = 13     the centre's own channel n      (auto-products, bin-pair counts)
//   k = 14     the constant 1                  (zero-order sums)
// The 117-dim rotation-invariant feature is the sum over k of the 981 first-order bins
// (color_chlac.hpp:1647-1743), so both variants share one exact integer pass and the
// epilogue folds / normalises with the reference's float constants.  Results equal the
// reference whenever its fp32 running sums stay below 2^24, else differ by its own
// rounding (<= a few ulp); exist_voxel_num is reproduced bit-exactly from the integer
// zero-order sums (search_c3_hlac.h:60-61).
//
// Mapping.  One 256-thread workgroup per tile; a tile is one subdivision (or a <=16^3
// piece of one: partial sums then go through 64-bit atomics + a finalize kernel).
//   1. stage the (lx+2) x (ly+2) x (lz+1) halo of packed grid words in LDS
//   2. compact the occupied centre voxels into an LDS list (wave ballot)
//   3. per chunk of 64 list entries: 240 threads build the packed operand dwords
//      (16 groups x 15 k x {colour, binary} x 6 channels) in LDS
//   4. 180 threads accumulate 6 dot4 products per group into u32 registers
//   5. scatter the 981 integer bins to LDS, fold/normalise, coalesced store
// Tiles are enumerated x-fastest and dealt to XCDs in contiguous ranges so neighbouring
// tiles (which share halo lines) run on the same L2.
#include "c3h_internal.h"

namespace c3h {
namespace {

constexpr int kArrStride = 192;  // dwords per group: 2 types x 15 k x 6 n = 180, padded
constexpr int kGroups = kChunk / 4;

// relative_coordinates (c3_hlac.cpp:180-201)
__constant__ int kRel[13][3] = {{-1, -1, -1}, {-1, 0, -1}, {-1, 1, -1}, {0, -1, -1}, {0, 0, -1},
                                {0, 1, -1},   {1, -1, -1}, {1, 0, -1},  {1, 1, -1},  {-1, -1, 0},
                                {0, -1, 0},   {1, -1, 0},  {-1, 0, 0}};

__device__ __forceinline__ int bin981(int k, int c, int n) {
  return k <= 8 ? 6 + 78 * c + 9 * n + k : 60 + 78 * c + 4 * n + (k - 9);
}
__device__ __forceinline__ int tri6(int c, int n) { return 6 * c - c * (c - 1) / 2 + (n - c); }

// bin of accumulator (type, k, n, c); -1 when that product is not a feature bin
__device__ __forceinline__ int bin_of(int type, int k, int n, int c) {
  if (k <= 12) return (type ? 495 : 0) + bin981(k, c, n);
  if (k == 13) {
    if (type == 0) return c <= n ? 474 + tri6(c, n) : -1;
    if (c <= 1 && n >= 2) return 969 + 4 * c + (n - 2);
    if ((c == 2 || c == 3) && n >= 4) return 977 + 2 * (c - 2) + (n - 4);
    return -1;
  }
  return n == 0 ? (type ? 495 : 0) + c : -1;
}

__device__ __forceinline__ float norm981(int i) {
  return i < 6 ? kNorm0 : (i < 495 ? kNorm1 : 1.0f);
}
__device__ __forceinline__ float norm117(int i) {
  return i < 6 ? kNorm0 : i < 42 ? kNorm117_1 : i < 63 ? kNorm1 : i < 69 ? 1.0f : i < 105 ? kNorm117_1Bin : 1.0f;
}

template <class T>
__device__ __forceinline__ T fold117(const T* hist, int i) {
  if (i < 6) return hist[i];
  if (i < 42) {
    const int c = (i - 6) / 6, n = (i - 6) % 6;
    T s = 0;
    for (int k = 0; k < 13; ++k) s += hist[bin981(k, c, n)];
    return s;
  }
  if (i < 63) return hist[474 + (i - 42)];
  if (i < 69) return hist[495 + (i - 63)];
  if (i < 105) {
    const int c = (i - 69) / 6, n = (i - 69) % 6;
    T s = 0;
    for (int k = 0; k < 13; ++k) s += hist[495 + bin981(k, c, n)];
    return s;
  }
  return hist[969 + (i - 105)];
}

// exist_voxel_num[h] = (int)((f[0] + f[1]) * 2 + 0.001), f = float sums * float(1/255)
__device__ __forceinline__ int32_t exist_from(float s0, float s1) {
  const float f0 = s0 * kNorm0;
  const float f1 = s1 * kNorm0;
  const float t = (f0 + f1) * 2.0f;
  return (int32_t)((double)t + 0.001);
}

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t n) {
  const int64_t q = n / 8, r = n % 8, xcd = b % 8, loc = b / 8;
  return xcd < r ? xcd * (q + 1) + loc : r * (q + 1) + (xcd - r) * q + loc;
}

struct KArgs {
  const uint32_t* grid;
  int gx, gy, gz;
  const int32_t* segs;
  int ns0, ns1, ns2, seg_stride;
  int sbx, sby;
  int tw_max, list_max;
  int thr_r, thr_g, thr_b;
  int variant, atomic;
  const uint32_t* lut;
  float* feat;
  int32_t* exist;
  unsigned long long* acc64;
  int64_t ntiles;
};

__global__ __launch_bounds__(kBlock) void c3hlac_tile_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_lut = smem;                       // 256
  uint32_t* s_tile = s_lut + 256;               // tw_max
  uint16_t* s_list = reinterpret_cast<uint16_t*>(s_tile + a.tw_max);  // list_max (u16)
  uint32_t* s_arr = s_tile + a.tw_max + ((a.list_max + 7) / 8) * 4;   // kGroups*kArrStride
  uint32_t* s_misc = s_arr + kGroups * kArrStride;                  // counter
  uint32_t* s_hist = s_arr;                                          // epilogue alias

  const int tid = threadIdx.x;
  const int64_t tile = xcd_remap(blockIdx.x, a.ntiles);
  const int ix = (int)(tile % a.ns0);
  const int iy = (int)((tile / a.ns0) % a.ns1);
  const int iz = (int)(tile / ((int64_t)a.ns0 * a.ns1));
  const int32_t* sx = a.segs + 3 * ix;
  const int32_t* sy = a.segs + 3 * (a.seg_stride + iy);
  const int32_t* sz = a.segs + 3 * (2 * a.seg_stride + iz);
  const int x0 = sx[0], lx = sx[1], y0 = sy[0], ly = sy[1], z0 = sz[0], lz = sz[1];
  const int64_t h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
  const int TX = lx + 2, TY = ly + 2, TXY = TX * TY;
  const int TW = TXY * (lz + 1);

  s_lut[tid] = a.lut[tid];
  if (tid == 0) s_misc[0] = 0;
  // 1. halo tile: x in [x0-1, x0+lx], y in [y0-1, y0+ly], z in [z0-1, z0+lz-1]
  for (int i = tid; i < TW; i += kBlock) {
    const int tz = i / TXY, rem = i - tz * TXY, ty = rem / TX, tx = rem - ty * TX;
    const int gx = x0 - 1 + tx, gy = y0 - 1 + ty, gz = z0 - 1 + tz;
    uint32_t w = 0;
    if ((unsigned)gx < (unsigned)a.gx && (unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz)
      w = a.grid[((int64_t)gz * a.gy + gy) * a.gx + gx];
    s_tile[i] = w;
  }
  __syncthreads();

  // 2. compact occupied centres (tile index) into the list
  const int V = lx * ly * lz, lxy = lx * ly;
  const int lane = tid & 63;
  for (int v0 = 0; v0 < V; v0 += kBlock) {
    const int v = v0 + tid;
    int ti = 0;
    bool occ = false;
    if (v < V) {
      const int cz = v / lxy, rem = v - cz * lxy, cy = rem / lx, cx = rem - cy * lx;
      ti = (cx + 1) + (cy + 1) * TX + (cz + 1) * TXY;
      occ = s_tile[ti] != 0;
    }
    const unsigned long long m = __ballot(occ);
    const int tot = __popcll(m);
    uint32_t base = 0;
    if (lane == 0 && tot) base = atomicAdd(&s_misc[0], (uint32_t)tot);
    base = __shfl(base, 0, 64);
    if (occ) s_list[base + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)ti;
  }
  __syncthreads();
  const int nlist = (int)s_misc[0];
  const int F = a.variant;

  if (nlist == 0) {  // empty subdivision: zero feature
    if (!a.atomic) {
      for (int i = tid; i < F; i += kBlock) a.feat[h * F + i] = 0.0f;
      if (tid == 0) a.exist[h] = 0;
    }
    return;
  }

  // per-thread roles
  const int bg = tid / 15, bk = tid - bg * 15;  // build job (group, k), tid < 240
  int delta = 0;
  if (tid < 240 && bk < 13) delta = kRel[bk][0] + kRel[bk][1] * TX + kRel[bk][2] * TXY;
  const int at = tid / 90, arem = tid - at * 90, ak = arem / 6, an = arem - ak * 6;
  uint32_t acc[6] = {0, 0, 0, 0, 0, 0};

  for (int c0 = 0; c0 < nlist; c0 += kChunk) {
    // 3. build packed operands for list entries [c0, c0+64)
    if (tid < 240) {
      uint32_t nb[6] = {0, 0, 0, 0, 0, 0}, bb[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = c0 + bg * 4 + j;
        if (e >= nlist) break;
        const int ti = s_list[e];
        const uint32_t w = s_tile[ti + delta];
        if (!w) continue;
        const int sh = 8 * j;
        if (bk == 14) {
#pragma unroll
          for (int n = 0; n < 6; ++n) {
            nb[n] |= 1u << sh;
            bb[n] |= 1u << sh;
          }
          continue;
        }
        const uint32_t r = (w >> 16) & 0xffu, g = (w >> 8) & 0xffu, b = w & 0xffu;
        const uint32_t lr = s_lut[r], lg = s_lut[g], lb = s_lut[b];
        nb[0] |= (lr & 0xffu) << sh;
        nb[1] |= (lr >> 8) << sh;
        nb[2] |= (lg & 0xffu) << sh;
        nb[3] |= (lg >> 8) << sh;
        nb[4] |= (lb & 0xffu) << sh;
        nb[5] |= (lb >> 8) << sh;
        const uint32_t br = (int)r > a.thr_r, bgn = (int)g > a.thr_g, bbl = (int)b > a.thr_b;
        bb[0] |= br << sh;
        bb[1] |= (br ^ 1u) << sh;
        bb[2] |= bgn << sh;
        bb[3] |= (bgn ^ 1u) << sh;
        bb[4] |= bbl << sh;
        bb[5] |= (bbl ^ 1u) << sh;
      }
      uint32_t* dst = s_arr + bg * kArrStride + bk * 6;
#pragma unroll
      for (int n = 0; n < 6; ++n) {
        dst[n] = nb[n];
        dst[90 + n] = bb[n];
      }
    }
    __syncthreads();
    // 4. exact integer accumulation: acc[c] += sum_g dot4(A_c[g], N_{k,n}[g])
    if (tid < 180) {
      const int ng = (min(nlist - c0, kChunk) + 3) >> 2;
      const uint32_t* col = s_arr + at * 90 + ak * 6 + an;
      const uint32_t* ctr = s_arr + at * 90 + 13 * 6;
      for (int g = 0; g < ng; ++g) {
        const uint32_t nv = col[g * kArrStride];
#pragma unroll
        for (int c = 0; c < 6; ++c)
          acc[c] = __builtin_amdgcn_udot4(ctr[g * kArrStride + c], nv, acc[c], false);
      }
    }
    __syncthreads();
  }

  // 5. epilogue: integer bins -> LDS, then fold / normalise / store
  if (tid < 180) {
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const int bi = bin_of(at, ak, an, c);
      if (bi >= 0) s_hist[bi] = acc[c];
    }
  }
  __syncthreads();
  if (a.atomic) {
    for (int i = tid; i < 981; i += kBlock) {
      const uint32_t v = s_hist[i];
      if (v) atomicAdd(&a.acc64[h * 981 + i], (unsigned long long)v);
    }
    return;
  }
  float* out = a.feat + h * F;
  if (F == 981) {
    for (int i = tid; i < 981; i += kBlock) out[i] = (float)s_hist[i] * norm981(i);
  } else {
    for (int i = tid; i < 117; i += kBlock) out[i] = (float)fold117(s_hist, i) * norm117(i);
  }
  if (tid == 0) a.exist[h] = exist_from((float)s_hist[0], (float)s_hist[1]);
}

// multi-tile subdivisions: 64-bit exact partial sums -> features
__global__ __launch_bounds__(kBlock) void c3_finalize_kernel(const unsigned long long* acc64,
                                                             int variant, float* feat,
                                                             int32_t* exist) {
  const int64_t h = blockIdx.x;
  const unsigned long long* hist = acc64 + h * 981;
  float* out = feat + h * variant;
  if (variant == 981) {
    for (int i = threadIdx.x; i < 981; i += kBlock) out[i] = (float)hist[i] * norm981(i);
  } else {
    for (int i = threadIdx.x; i < 117; i += kBlock) out[i] = (float)fold117(hist, i) * norm117(i);
  }
  if (threadIdx.x == 0) exist[h] = exist_from((float)hist[0], (float)hist[1]);
}

}  // namespace

size_t c3hlac_lds_bytes(int tw_max, int list_max) {
  return sizeof(uint32_t) * (256 + tw_max + ((list_max + 7) / 8) * 4 + kGroups * kArrStride + 4);
}

hipError_t launch_c3hlac(const C3Launch& l, hipStream_t s) {
  KArgs a;
  a.grid = l.grid;
  a.gx = l.gx;
  a.gy = l.gy;
  a.gz = l.gz;
  a.segs = l.segs;
  a.ns0 = l.nseg[0];
  a.ns1 = l.nseg[1];
  a.ns2 = l.nseg[2];
  a.seg_stride = l.seg_stride;
  a.sbx = l.sbx;
  a.sby = l.sby;
  a.tw_max = (l.lmax[0] + 2) * (l.lmax[1] + 2) * (l.lmax[2] + 1);
  a.list_max = l.lmax[0] * l.lmax[1] * l.lmax[2];
  a.thr_r = l.thr[0];
  a.thr_g = l.thr[1];
  a.thr_b = l.thr[2];
  a.variant = l.variant;
  a.atomic = l.atomic;
  a.lut = l.lut;
  a.feat = l.feat;
  a.exist = l.exist;
  a.acc64 = l.acc64;
  a.ntiles = l.ntiles;
  const size_t lds = c3hlac_lds_bytes(a.tw_max, a.list_max);
  c3hlac_tile_kernel<<<(unsigned)l.ntiles, kBlock, lds, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_c3_finalize(const unsigned long long* acc64, int64_t hist_num, int variant,
                              float* feat, int32_t* exist, hipStream_t s) {
  c3_finalize_kernel<<<(unsigned)hist_num, kBlock, 0, s>>>(acc64, variant, feat, exist);
  return hipGetLastError();
}

}  // namespace c3h
