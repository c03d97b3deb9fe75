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
// Mapping.  Two passes per frame (frame = launch y index, several frames per launch):
//   pass 1 (c3_occupancy_kernel) streams the packed grid once and stamps the tiles (a
//     subdivision, or a <=16^3 piece of one) holding occupied centre voxels, appending
//     them to a dense work list;
//   pass 2 (c3hlac_tile_kernel), persistent 256-thread workgroups over the work list:
//   1. stage the (lx+2) x (ly+2) x (lz+1) halo of packed grid words in LDS
//   2. compact the occupied centre voxels into an LDS list (wave ballot)
//   3. per chunk of 128 list entries, (group, k) jobs build the packed operand dwords
//      (32 groups x 15 k x {colour, binary} x 6 channels: 4 voxels' bytes per dword)
//   4. 180 threads, one (type, k, n) column each, accumulate 6 dot4 products per group
//      into u32 registers
//   5. scatter the 981 integer bins to LDS, fold/normalise, coalesced store
//   Leading zero-role workgroups write the all-zero rows of the unstamped subdivisions.
//   Pieces of split subdivisions go through 64-bit atomics + c3_finalize_kernel.
#include <algorithm>
#include <cstdlib>

#include "c3h_internal.h"

namespace c3h {
namespace {

constexpr int kArrStride = 196;  // dwords per group: 2 types x 15 k x 6 n = 180, padded so
                                 // groups start 4 banks apart (192 would alias all groups)
constexpr int kChunk = 128;      // list entries per packed-operand chunk
constexpr int kGroups = kChunk / 4;

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

__device__ __forceinline__ int xcd_remap32(int b, int n) {
  const int q = n >> 3, r = n & 7, xcd = b & 7, loc = b >> 3;
  return xcd < r ? xcd * (q + 1) + loc : r * (q + 1) + (xcd - r) * q + loc;
}

__device__ __forceinline__ int64_t xcd_remap(int64_t b, int64_t n) {
  const int64_t q = n / 8, r = n % 8, xcd = b % 8, loc = b / 8;
  return xcd < r ? xcd * (q + 1) + loc : r * (q + 1) + (xcd - r) * q + loc;
}

// ---------------------------------------------------------------- pass 1: occupancy
// Streams the packed grid once (16-B loads, x-rows of 4 voxels when gx % 4 == 0) and
// flags every tile (subdivision or <=16^3 piece of one) holding an occupied centre
// voxel; the first flagger appends the tile to the work list.  axmap_[xyz][c] gives the
// tile segment of centre coordinate c along that axis (-1 when c is no centre, e.g.
// below the subdivision offset): the reference's float subdivision arithmetic is baked
// into these host-built tables.
constexpr int kOccUnroll = 16;  // 16-B loads per thread in flight per chunk (256 B / lane)
constexpr int kOccSet = 1024;  // LDS set of tiles touched by one workgroup (4 KB)

// Flags are epoch stamps: tile t is non-empty in this frame iff flags[t] == epoch, so
// nothing is reset between frames.  Each workgroup streams contiguous 16-KB chunks
// (4096 voxels: coalesced 16-B loads, all issued before use), collects the tiles of its
// occupied centre voxels in an LDS set, and only then stamps them: one global atomic
// per (workgroup, tile), off the streaming path; the first stamper of a tile appends it
// to the work list.  The set overflows only for tiny subdivisions (then tiles are
// stamped directly).
__device__ __forceinline__ void stamp_tile(int t, uint32_t epoch, uint32_t* flags, uint32_t* cnt,
                                           int32_t* work) {
  if (atomicExch(&flags[t], epoch) != epoch) work[atomicAdd(cnt, 1u)] = t;
}

__device__ __forceinline__ void set_insert(int* s_set, int t, uint32_t epoch, uint32_t* flags,
                                           uint32_t* cnt, int32_t* work) {
  int h = (int)(((uint32_t)t * 0x9E3779B1u) >> 22);  // 10-bit hash
  static_assert(kOccSet == 1024 && kOccSet % kBlock == 0, "set slots per thread");
  for (int probe = 0; probe < kOccSet; ++probe, h = (h + 1) & (kOccSet - 1)) {
    const int cur = s_set[h];
    if (cur == t) return;
    if (cur == -1) {
      const int old = atomicCAS(&s_set[h], -1, t);
      if (old == -1 || old == t) return;
    }
  }
  stamp_tile(t, epoch, flags, cnt, work);  // set full
}

struct OccArgs {
  const uint32_t* grid[kMaxBatch];  // frame f = blockIdx.y
  int gx, gy, gz;
  const int16_t* axmap;
  int ns0, ns1;
  int ntiles;
  uint32_t epoch;
  uint32_t* tf;    // per frame: [2] reserved | [2] work counters | [ntiles] stamps
  int32_t* work;   // per frame: [ntiles]
  int64_t s_tf, s_work;
};

// Bitmap variant (every tile one bit of LDS, ntiles <= kOccBitsMax): an occupied centre
// voxel costs VALU plus one fire-and-forget ds_or, so no LDS round trip sits behind the
// stream data.  Per chunk the axis lookups are batched: x is fixed per lane whenever gx
// divides the chunk stride (4 voxels, at most 4 x-segments, looked up once per chunk),
// the 16 rows' (y, z) segments are looked up together.  The flush compacts the set bits
// into an LDS list and stamps kBlock tiles at a time, every exchange in flight together.
constexpr int kOccBitsMax = 1 << 17;  // 16 KB of LDS bits
constexpr int kOccBitsUnroll = 8;     // 16-B non-temporal loads per lane in flight per chunk
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kAxLds = 3072;  // axis-map entries kept in LDS (gx + gy + gz <= 3072)

// exclusive prefix sum over the workgroup (kBlock threads); total returned in *total
__device__ __forceinline__ int block_excl_scan(int v, int* s_wsum, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_wsum[wid] = x;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBlock / 64; ++i) {
    const int t = s_wsum[i];
    off += i < wid ? t : 0;
    tot += t;
  }
  __syncthreads();  // s_wsum is reused by the next scan
  *total = tot;
  return off + x - v;
}

__device__ __forceinline__ void occ_flush_bits(const uint32_t* s_bits, int nwords, int* s_list,
                                               int* s_wsum, uint32_t epoch, uint32_t* flags,
                                               uint32_t* cnt, int32_t* work) {
  const int tid = threadIdx.x, lane = tid & 63;
  for (int w0 = 0; w0 < nwords; w0 += kBlock) {  // one bitmap word per thread per round
    const int wi = w0 + tid;
    const uint32_t m = wi < nwords ? s_bits[wi] : 0u;
    int total;
    const int base = block_excl_scan(__popc(m), s_wsum, &total);
    for (int l0 = 0; l0 < total; l0 += kOccSet) {  // list slices of kOccSet tiles
      uint32_t mm = m;
      for (int idx = base; mm; ++idx) {
        const int bit = __ffs(mm) - 1;
        mm &= mm - 1;
        if (idx >= l0 && idx < l0 + kOccSet) s_list[idx - l0] = wi * 32 + bit;
      }
      __syncthreads();
      const int nl = min(total - l0, kOccSet);
      int ts[kOccSet / kBlock];
      bool fresh[kOccSet / kBlock];
#pragma unroll
      for (int j = 0; j < kOccSet / kBlock; ++j) {  // all exchanges in flight together
        const int e = tid + j * kBlock;
        ts[j] = e < nl ? s_list[e] : -1;
        fresh[j] = ts[j] >= 0 && atomicExch(&flags[ts[j]], epoch) != epoch;
      }
#pragma unroll
      for (int j = 0; j < kOccSet / kBlock; ++j) {
        const unsigned long long b = __ballot(fresh[j]);
        if (b) {
          uint32_t b0 = 0;
          if (lane == 0) b0 = atomicAdd(cnt, (uint32_t)__popcll(b));
          b0 = __shfl(b0, 0, 64);
          if (fresh[j]) work[b0 + __popcll(b & ((1ull << lane) - 1))] = ts[j];
        }
      }
      __syncthreads();  // s_list is refilled by the next slice
    }
  }
}

template <bool kAx>
__global__ __launch_bounds__(kBlock) void c3_occupancy_bits_kernel(OccArgs oa) {
  const int f = blockIdx.y;
  const uint32_t* __restrict__ grid = oa.grid[f];
  const int gx = oa.gx, gy = oa.gy, gz = oa.gz;
  const int ns0 = oa.ns0, ns1 = oa.ns1;
  const uint32_t epoch = oa.epoch;
  uint32_t* __restrict__ flags = oa.tf + f * oa.s_tf + 4;
  uint32_t* __restrict__ cnt = oa.tf + f * oa.s_tf + 2 + (epoch & 1);
  int32_t* __restrict__ work = oa.work + f * oa.s_work;
  extern __shared__ __attribute__((aligned(16))) uint32_t s_bits[];  // ceil(ntiles / 32)
  __shared__ int s_list[kOccSet];
  __shared__ int s_wsum[kBlock / 64];
  __shared__ int16_t s_ax[kAx ? kAxLds : 1];
  const int tid = threadIdx.x;
  const int nwords = (oa.ntiles + 31) >> 5;
  const int16_t* mx = kAx ? s_ax : oa.axmap;
  const int16_t* my = mx + gx;
  const int16_t* mz = my + gy;
  for (int i = tid; i < nwords; i += kBlock) s_bits[i] = 0u;
  if (kAx)
    for (int i = tid; i < gx + gy + gz; i += kBlock) s_ax[i] = oa.axmap[i];
  __syncthreads();
  const int64_t n4 = ((int64_t)gx * gy * gz) >> 2;
  const uint4* g4 = reinterpret_cast<const uint4*>(grid);
  constexpr int kChunk4 = kBlock * kOccBitsUnroll;
  // consecutive j of one thread are kBlock*4 voxels apart: step (x, y, z) incrementally
  const int dxs = (kBlock * 4) % gx, drs = (kBlock * 4) / gx;
  int last = -1;
  for (int64_t c0 = blockIdx.x * (int64_t)kChunk4; c0 < n4; c0 += (int64_t)gridDim.x * kChunk4) {
    uint4 w[kOccBitsUnroll];
#pragma unroll
    for (int j = 0; j < kOccBitsUnroll; ++j) {  // all loads first: bytes in flight, not latency
      const int64_t i = c0 + j * kBlock + tid;
      // non-temporal: the grid is read once here (the tile pass re-reads only the few
      // occupied tiles' halos); measured 6.9-7.0 TB/s vs 6.0-6.3 for default-policy loads
      const v4u t = i < n4 ? __builtin_nontemporal_load(reinterpret_cast<const v4u*>(g4) + i) : v4u{0, 0, 0, 0};
      w[j] = make_uint4(t.x, t.y, t.z, t.w);
    }
    const uint32_t v0 = (uint32_t)((c0 + tid) << 2);  // nvox < 2^32 (host-checked)
    const uint32_t row0 = v0 / (uint32_t)gx;
    int x = (int)(v0 - row0 * (uint32_t)gx);
    int y = (int)(row0 % (uint32_t)gy), z = (int)(row0 / (uint32_t)gy);
    // the rows' (y, z) segments of all j, looked up together (clamped past the grid end)
    int tyz[kOccBitsUnroll];
    int txj[kOccBitsUnroll];  // x of row j (differs per j only when dxs != 0)
#pragma unroll
    for (int j = 0; j < kOccBitsUnroll; ++j) {
      const int ty = my[y], tz = mz[min(z, gz - 1)];
      tyz[j] = (ty >= 0 && tz >= 0 && z < gz) ? ns0 * (ty + ns1 * tz) : -1;
      txj[j] = x;
      x += dxs;
      int dy = drs;
      if (x >= gx) {
        x -= gx;
        ++dy;
      }
      y += dy;
      while (y >= gy) {
        y -= gy;
        ++z;
      }
    }
    int tx0[4];
    if (dxs == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) tx0[k] = mx[txj[0] + k];
    }
#pragma unroll
    for (int j = 0; j < kOccBitsUnroll; ++j) {
      const uint32_t ws[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
      if ((ws[0] | ws[1] | ws[2] | ws[3]) == 0 || tyz[j] < 0) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!ws[k]) continue;
        const int tx = dxs == 0 ? tx0[k] : mx[txj[j] + k];
        if (tx < 0) continue;
        const int t = tx + tyz[j];
        if (t == last) continue;
        last = t;
        atomicOr(&s_bits[t >> 5], 1u << (t & 31));  // result unused: ds_or_b32, no wait
      }
    }
  }
  __syncthreads();
  occ_flush_bits(s_bits, nwords, s_list, s_wsum, epoch, flags, cnt, work);
}



// kAx: the axis map lives in LDS, so the per-voxel tile lookup is LDS-only (no global
// load in the chain behind the stream data)
template <bool kVec, bool kAx>
__global__ __launch_bounds__(kBlock) void c3_occupancy_kernel(OccArgs oa) {
  const int f = blockIdx.y;
  const uint32_t* __restrict__ grid = oa.grid[f];
  const int gx = oa.gx, gy = oa.gy, gz = oa.gz;
  const int ns0 = oa.ns0, ns1 = oa.ns1;
  const uint32_t epoch = oa.epoch;
  uint32_t* __restrict__ flags = oa.tf + f * oa.s_tf + 4;
  uint32_t* __restrict__ cnt = oa.tf + f * oa.s_tf + 2;
  int32_t* __restrict__ work = oa.work + f * oa.s_work;
  __shared__ int s_set[kOccSet];
  __shared__ int16_t s_ax[kAx ? kAxLds : 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int64_t nvox = (int64_t)gx * gy * gz;
  const int16_t* mx = kAx ? s_ax : oa.axmap;
  const int16_t* my = mx + gx;
  const int16_t* mz = my + gy;
  cnt += epoch & 1;
  for (int i = tid; i < kOccSet; i += kBlock) s_set[i] = -1;
  if (kAx)
    for (int i = tid; i < gx + gy + gz; i += kBlock) s_ax[i] = oa.axmap[i];
  __syncthreads();
  int last = -1;
  if (kVec) {
    const int64_t n4 = nvox >> 2;
    const uint4* g4 = reinterpret_cast<const uint4*>(grid);
    constexpr int kChunk4 = kBlock * kOccUnroll;
    // consecutive j of one thread are kBlock*4 voxels apart: step (x, y, z) incrementally
    const int dxs = (kBlock * 4) % gx, drs = (kBlock * 4) / gx;
    for (int64_t c0 = blockIdx.x * (int64_t)kChunk4; c0 < n4; c0 += (int64_t)gridDim.x * kChunk4) {
      uint4 w[kOccUnroll];
#pragma unroll
      for (int j = 0; j < kOccUnroll; ++j) {  // all loads first: bytes in flight, not latency
        const int64_t i = c0 + j * kBlock + tid;
        w[j] = i < n4 ? g4[i] : make_uint4(0, 0, 0, 0);
      }
      const uint32_t v0 = (uint32_t)((c0 + tid) << 2);  // nvox < 2^32 (host-checked)
      const uint32_t row0 = v0 / (uint32_t)gx;
      int x = (int)(v0 - row0 * (uint32_t)gx);
      int y = (int)(row0 % (uint32_t)gy), z = (int)(row0 / (uint32_t)gy);
#pragma unroll
      for (int j = 0; j < kOccUnroll; ++j) {
        if ((w[j].x | w[j].y | w[j].z | w[j].w) != 0) {
          const int ty = my[y], tz = z < gz ? mz[z] : -1;
          if (ty >= 0 && tz >= 0) {
            const int tyz = ns0 * (ty + ns1 * tz);
            const uint32_t ws[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if (!ws[k]) continue;
              const int tx = mx[x + k];
              if (tx < 0) continue;
              const int t = tx + tyz;
              if (t == last) continue;
              last = t;
              set_insert(s_set, t, epoch, flags, cnt, work);
            }
          }
        }
        x += dxs;
        int dy = drs;
        if (x >= gx) {
          x -= gx;
          ++dy;
        }
        y += dy;
        while (y >= gy) {
          y -= gy;
          ++z;
        }
      }
    }
  } else {
    for (int64_t v = blockIdx.x * (int64_t)kBlock + tid; v < nvox; v += (int64_t)gridDim.x * kBlock) {
      if (!grid[v]) continue;
      const uint32_t row = (uint32_t)v / (uint32_t)gx;
      const int x = (int)((uint32_t)v - row * (uint32_t)gx);
      const int y = (int)(row % (uint32_t)gy), z = (int)(row / (uint32_t)gy);
      const int tx = mx[x], ty = my[y], tz = mz[z];
      if (tx < 0 || ty < 0 || tz < 0) continue;
      const int t = tx + ns0 * (ty + ns1 * tz);
      if (t == last) continue;
      last = t;
      set_insert(s_set, t, epoch, flags, cnt, work);
    }
  }
  __syncthreads();
  // flush: one stamp per (workgroup, tile); new tiles appended with one add per wave
  int ts[kOccSet / kBlock];
  bool fresh[kOccSet / kBlock];
#pragma unroll
  for (int j = 0; j < kOccSet / kBlock; ++j) {  // all exchanges in flight together
    ts[j] = s_set[tid + j * kBlock];
    fresh[j] = ts[j] >= 0 && atomicExch(&flags[ts[j]], epoch) != epoch;
  }
#pragma unroll
  for (int j = 0; j < kOccSet / kBlock; ++j) {
    const unsigned long long m = __ballot(fresh[j]);
    if (m) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(cnt, (uint32_t)__popcll(m));
      base = __shfl(base, 0, 64);
      if (fresh[j]) work[base + __popcll(m & ((1ull << lane) - 1))] = ts[j];
    }
  }
}

// ---------------------------------------------------------------- pass 2: features
struct KArgs {
  const uint32_t* grids[kMaxBatch];  // frame f = blockIdx.y; per-frame buffers at f * stride
  int64_t s_feat, s_h, s_acc, s_tf, s_work;
  uint32_t* tf;  // frame 0's [2] reserved | [2] work counters | [ntiles] stamps
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
  const uint32_t* flags;  // tile epoch stamps of pass 1
  const int32_t* work;    // non-empty tiles of pass 1
  uint32_t* workcnt;      // [2] work-list counters by epoch parity
  int32_t* rows;          // direct mode: non-empty subdivisions of this frame (nullable)
  uint32_t epoch;
  int ntiles;
  int zero_feat;          // zero role writes feature rows too (else exist only)
  int zblocks;            // leading workgroups that zero the rows of unstamped tiles
                          // (direct mode, every subdivision one tile: h == tile), else 0
  long long* prof;  // diagnostics only (C3H_PROF): per-block phase timestamps [grid][8]
  int debug;  // diagnostics only (C3H_C3_DEBUG): 1 stop after the loads, 2 after compaction,
             // 3 skip the tile kernel
};

constexpr int kMaxLoads = 4;  // uint4 tile loads per thread kept in flight together
constexpr int kSegLds = 64;   // segment tables up to 64 segments per axis live in LDS

// Persistent workgroups.  Phase Z zero-fills the feature rows of the tiles pass 1 left
// unflagged (direct mode); phase T walks the work list: stage the (lx+2)x(ly+2)x(lz+1)
// halo in LDS (all loads issued before the first LDS store), compact the occupied
// centres, build the packed dot4 operands and accumulate exactly (see the header).
#define C3H_PROF(k, cond) \
  if (fprof && tid == 0 && (cond)) fprof[blockIdx.x * 8 + (k)] = (long long)wall_clock64()

__global__ __launch_bounds__(kBlock) void c3hlac_tile_kernel(KArgs a) {
  // this frame's buffers (frame = blockIdx.y); the argument struct itself is not copied
  const int64_t fy = blockIdx.y;
  const uint32_t* __restrict__ fgrid = a.grids[fy];
  float* __restrict__ ffeat = a.feat + fy * a.s_feat;
  int32_t* __restrict__ fexist = a.exist + fy * a.s_h;
  unsigned long long* facc = a.acc64 ? a.acc64 + fy * a.s_acc : nullptr;
  uint32_t* ftf = a.tf + fy * a.s_tf;
  const uint32_t* __restrict__ fflags = ftf + 4;
  uint32_t* fworkcnt = ftf + 2;
  const int32_t* __restrict__ fwork = a.work + fy * a.s_work;
  int32_t* frows = a.rows ? a.rows + fy * a.s_h : nullptr;
  long long* fprof = fy ? nullptr : a.prof;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* s_lut = smem;                       // 256
  uint32_t* s_tile = s_lut + 256;               // tw_max (16-B aligned)
  uint16_t* s_list = reinterpret_cast<uint16_t*>(s_tile + a.tw_max);  // list_max (u16)
  uint32_t* s_arr = s_tile + a.tw_max + ((a.list_max + 7) / 8) * 4;   // kGroups*kArrStride
  uint32_t* s_misc = s_arr + kGroups * kArrStride;                  // counters [4]
  int32_t* s_segs = reinterpret_cast<int32_t*>(s_misc + 4);         // segment table copy
  uint32_t* s_hist = s_arr;                                          // epilogue alias
  const int tid = threadIdx.x, lane = tid & 63;
  const int F = a.variant;
  C3H_PROF(0, true);
  // issued together: the work count, this workgroup's first work item, its phase-Z flags
  if (blockIdx.x == 0 && tid == 0) {  // the next frame's counters
    fworkcnt[(a.epoch + 1) & 1] = 0;
  }
  if ((int)blockIdx.x < a.zblocks) {
    // zero role (direct mode, every subdivision one tile: h == tile): exist of the tiles
    // pass 1 left unstamped (their feature rows stay stale unless zero_feat)
    if (!a.zero_feat) {
      for (int t = (int)blockIdx.x * kBlock + tid; t < a.ntiles; t += a.zblocks * kBlock)
        if (fflags[t] != a.epoch) fexist[t] = 0;
      return;
    }
    // rows too, one wave-wide store per 64 floats
    for (int t0 = (int)blockIdx.x * kBlock; t0 < a.ntiles; t0 += a.zblocks * kBlock) {
      const int t = t0 + tid;
      unsigned long long m = __ballot(t < a.ntiles && fflags[t] != a.epoch);
      while (m) {
        const int q = __ffsll((long long)m) - 1;
        m &= m - 1;
        const int tj = (t0 + (tid & ~63)) + q;
        float* row = ffeat + (int64_t)tj * F;
        for (int c = lane; c < F; c += 64) row[c] = 0.0f;
        if (lane == 0) fexist[tj] = 0;
      }
    }
    return;
  }
  // work role: workgroup b takes items b, b + G, ... of the dense work list (balanced)
  const int G = (int)gridDim.x - a.zblocks;
  int wi = (int)blockIdx.x - a.zblocks;
  int tile_next = wi < a.ntiles ? fwork[wi] : 0;  // speculative; used only if wi < nwork
  const int nwork = (int)fworkcnt[a.epoch & 1];
  if (a.debug == 3) return;  // diagnostics: occupancy pass only
  s_lut[tid] = a.lut[tid];
  const bool segs_lds = a.seg_stride <= kSegLds;
  const int32_t* segs = segs_lds ? s_segs : a.segs;
  if (segs_lds)
    for (int e = tid; e < 9 * a.seg_stride; e += kBlock) s_segs[e] = a.segs[e];
  const int at = tid / 90, arem = tid - at * 90, ak = arem / 6, an = arem - ak * 6;
  lds_barrier();
  C3H_PROF(1, true);

  for (; wi < (a.debug == 4 ? 0 : nwork); wi += G) {
    const int tile = tile_next;
    if (wi + G < nwork) tile_next = fwork[wi + G];
    const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
    const int32_t* sx = segs + 3 * ix;
    const int32_t* sy = segs + 3 * (a.seg_stride + iy);
    const int32_t* sz = segs + 3 * (2 * a.seg_stride + iz);
    const int x0 = sx[0], lx = sx[1], y0 = sy[0], ly = sy[1], z0 = sz[0], lz = sz[1];
    const int64_t h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
    const bool vec = (a.gx & 3) == 0 && x0 >= 1 && ((x0 + lx + 1 + 3) & ~3) <= a.gx;
    const int xs = vec ? ((x0 - 1) & ~3) : x0 - 1;
    const int TX = vec ? (((x0 + lx + 1 - xs) + 3) & ~3) : lx + 2;
    const int TY = ly + 2, TXY = TX * TY;
    const int nrows = TY * (lz + 1);
    if (tid == 0) s_misc[0] = 0;

    // 1. halo tile; every load of a thread is issued before its first LDS store
    if (vec) {
      const int q4 = TX >> 2, n = nrows * q4;
      uint4 w[kMaxLoads];
      int idx[kMaxLoads];
      int q = tid / q4, r = tid - q * q4;
      const int sq = kBlock / q4, sr = kBlock - sq * q4;
#pragma unroll
      for (int j = 0; j < kMaxLoads; ++j) {
        const int e = tid + j * kBlock;
        idx[j] = e;
        w[j] = make_uint4(0, 0, 0, 0);
        if (e < n) {
          const int ty = q % TY, tz = q / TY;
          const int gy = y0 - 1 + ty, gz = z0 - 1 + tz;
          if ((unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz)
            w[j] = *reinterpret_cast<const uint4*>(fgrid + ((int64_t)gz * a.gy + gy) * a.gx + xs + 4 * r);
        }
        q += sq;
        r += sr;
        if (r >= q4) {
          r -= q4;
          ++q;
        }
      }
#pragma unroll
      for (int j = 0; j < kMaxLoads; ++j)
        if (idx[j] < n) *reinterpret_cast<uint4*>(&s_tile[4 * idx[j]]) = w[j];
      for (int e = tid + kMaxLoads * kBlock; e < n; e += kBlock) {  // larger tiles
        const int qq = e / q4, rr = e - qq * q4;
        const int gy = y0 - 1 + qq % TY, gz = z0 - 1 + qq / TY;
        uint4 v = make_uint4(0, 0, 0, 0);
        if ((unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz)
          v = *reinterpret_cast<const uint4*>(fgrid + ((int64_t)gz * a.gy + gy) * a.gx + xs + 4 * rr);
        *reinterpret_cast<uint4*>(&s_tile[4 * e]) = v;
      }
    } else {
      const int n = nrows * TX;
      for (int e = tid; e < n; e += kBlock) {
        const int qq = e / TX, rr = e - qq * TX;
        const int gy = y0 - 1 + qq % TY, gz = z0 - 1 + qq / TY, gxx = xs + rr;
        s_tile[e] = ((unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz &&
                     (unsigned)gxx < (unsigned)a.gx)
                        ? fgrid[((int64_t)gz * a.gy + gy) * a.gx + gxx] : 0u;
      }
    }
    lds_barrier();
    C3H_PROF(3, wi == (int)blockIdx.x - a.zblocks);
    if (a.debug == 1) {
      if (tid == 0 && s_tile[0] == 0xdeadbeefu) fexist[0] = 1;  // keep the loads live
      lds_barrier();
      continue;
    }

    // 2. compact the occupied centres (tile index) into the list
    {
      const int V = lx * ly * lz;
      int cx = tid % lx, rq = tid / lx;  // v = tid + kBlock*i -> (cx, rq = cy + ly*cz)
      const int sq = kBlock / lx, sr = kBlock - sq * lx;
      for (int v0 = 0; v0 < V; v0 += kBlock) {
        const int v = v0 + tid;
        int ti = 0;
        bool occ = false;
        if (v < V) {
          const int cy = rq % ly, cz = rq / ly;
          ti = (x0 - xs + cx) + (cy + 1) * TX + (cz + 1) * TXY;
          occ = s_tile[ti] != 0;
        }
        const unsigned long long m = __ballot(occ);
        if (m) {
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(&s_misc[0], (uint32_t)__popcll(m));
          base = __shfl(base, 0, 64);
          if (occ) s_list[base + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)ti;
        }
        cx += sr;
        rq += sq;
        if (cx >= lx) {
          cx -= lx;
          ++rq;
        }
      }
    }
    lds_barrier();
    C3H_PROF(4, wi == (int)blockIdx.x - a.zblocks);
    const int nlist = (int)s_misc[0];
    if (a.debug == 2) {
      if (tid == 0 && nlist == 0x7fffffff) fexist[0] = 1;
      lds_barrier();
      continue;
    }

    uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
    for (int c0 = 0; c0 < nlist; c0 += kChunk) {
      // 3. build packed operands for list entries [c0, c0+kChunk): job = (group, k);
      //    branch-free so each job's LDS reads (list, tile, LUT) issue back to back
      for (int job = tid; job < kGroups * 15; job += kBlock) {
        const int jg = job / 15, jk = job - jg * 15;
        // relative_coordinates (c3_hlac.cpp:180-201), arithmetically: k <= 8 -> (k/3-1, k%3-1, -1),
        // k = 9..11 -> (k-10, -1, 0), k = 12 -> (-1, 0, 0); 13, 14 = centre / ones columns
        const int rdx = jk <= 8 ? jk / 3 - 1 : (jk <= 11 ? jk - 10 : -1);
        const int rdy = jk <= 8 ? jk % 3 - 1 : (jk <= 11 ? -1 : 0);
        const int rdz = jk <= 8 ? -1 : 0;
        const int delta = jk < 13 ? rdx + rdy * TX + rdz * TXY : 0;
        // every LDS read unconditional (indices clamped, results masked) so the 4 list,
        // 4 tile and 12 LUT reads issue as three back-to-back batches
        uint32_t li[4], w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) li[j] = s_list[min(c0 + jg * 4 + j, nlist - 1)];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = s_tile[li[j] + delta];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = (c0 + jg * 4 + j < nlist) ? w[j] : 0u;
        uint32_t lr[4], lg[4], lb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          lr[j] = s_lut[(w[j] >> 16) & 0xffu];
          lg[j] = s_lut[(w[j] >> 8) & 0xffu];
          lb[j] = s_lut[w[j] & 0xffu];
        }
        uint32_t nb[6] = {0, 0, 0, 0, 0, 0}, bb[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sh = 8 * j;
          const uint32_t occ = w[j] ? 1u : 0u;
          const uint32_t m8 = occ ? 0xffu : 0u;
          if (jk == 14) {  // the ones column: occupancy in every channel
#pragma unroll
            for (int n = 0; n < 6; ++n) {
              nb[n] |= occ << sh;
              bb[n] |= occ << sh;
            }
          } else {
            const uint32_t r = (w[j] >> 16) & 0xffu, g = (w[j] >> 8) & 0xffu, b = w[j] & 0xffu;
            nb[0] |= (lr[j] & m8) << sh;
            nb[1] |= ((lr[j] >> 8) & m8) << sh;
            nb[2] |= (lg[j] & m8) << sh;
            nb[3] |= ((lg[j] >> 8) & m8) << sh;
            nb[4] |= (lb[j] & m8) << sh;
            nb[5] |= ((lb[j] >> 8) & m8) << sh;
            const uint32_t br = (int)r > a.thr_r, bgn = (int)g > a.thr_g, bbl = (int)b > a.thr_b;
            bb[0] |= (occ & br) << sh;
            bb[1] |= (occ & (br ^ 1u)) << sh;
            bb[2] |= (occ & bgn) << sh;
            bb[3] |= (occ & (bgn ^ 1u)) << sh;
            bb[4] |= (occ & bbl) << sh;
            bb[5] |= (occ & (bbl ^ 1u)) << sh;
          }
        }
        uint32_t* dst = s_arr + jg * kArrStride + jk * 6;
#pragma unroll
        for (int n = 0; n < 6; ++n) {
          dst[n] = nb[n];
          dst[90 + n] = bb[n];
        }
      }
      lds_barrier();
      C3H_PROF(2, c0 == 0 && wi == (int)blockIdx.x - a.zblocks);
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
      lds_barrier();
    }
    C3H_PROF(5, wi == (int)blockIdx.x - a.zblocks);
    // 5. epilogue: integer bins -> LDS, then fold / normalise / store
    if (tid < 180) {
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int bi = bin_of(at, ak, an, c);
        if (bi >= 0) s_hist[bi] = acc[c];
      }
    }
    lds_barrier();
    if (a.atomic) {
      for (int i = tid; i < 981; i += kBlock) {
        const uint32_t v = s_hist[i];
        if (v) atomicAdd(&facc[h * 981 + i], (unsigned long long)v);
      }
    } else {
      float* out = ffeat + h * F;
      if (F == 981) {
        for (int i = tid; i < 981; i += kBlock) out[i] = (float)s_hist[i] * norm981(i);
      } else {
        for (int i = tid; i < 117; i += kBlock) out[i] = (float)fold117(s_hist, i) * norm117(i);
      }
      if (tid == 0) fexist[h] = exist_from((float)s_hist[0], (float)s_hist[1]);
    }
    // direct mode: tile == subdivision and the work list is dense, so the row list of
    // the sparse compress is the work list in subdivision terms (count = work count)
    if (frows && tid == 0) frows[wi] = (int32_t)h;
    lds_barrier();  // LDS is reused by the next tile
    C3H_PROF(6, wi == (int)blockIdx.x - a.zblocks);
  }
  C3H_PROF(7, true);
}

// multi-tile subdivisions: 64-bit exact partial sums -> features
__global__ __launch_bounds__(kBlock) void c3_finalize_kernel(const unsigned long long* acc64,
                                                             int variant, float* feat,
                                                             int32_t* exist, int64_t hist_num) {
  const int64_t h = blockIdx.x;
  acc64 += blockIdx.y * hist_num * 981;
  feat += blockIdx.y * hist_num * variant;
  exist += blockIdx.y * hist_num;
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
  return sizeof(uint32_t) * (256 + tw_max + ((list_max + 7) / 8) * 4 + kGroups * kArrStride + 4 + 9 * kSegLds);
}

// persistent grid: every workgroup resident at once (occupancy from LDS and VGPRs)
int64_t c3hlac_grid(const C3Launch& l) {
  // work workgroups: two per CU (a frame's few hundred non-empty tiles finish in a couple
  // of rounds while the rest of the chip stays free for the other frames in flight),
  // capped by what is resident at once; plus the zero-role workgroups
  const int tx_max = ((l.lmax[0] + 2) + 3 + 3) & ~3;
  const size_t lds = c3hlac_lds_bytes(tx_max * (l.lmax[1] + 2) * (l.lmax[2] + 1), l.lmax[0] * l.lmax[1] * l.lmax[2]);
  static thread_local size_t c_lds = 0;
  static thread_local int c_per_cu = 0, c_ncu = 0, c_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (lds != c_lds || dev != c_dev) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c3hlac_tile_kernel, kBlock, lds) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    c_lds = lds;
    c_per_cu = per_cu;
    c_ncu = n_cu;
    c_dev = dev;
  }
  int64_t work = std::min<int64_t>(l.ntiles, (int64_t)c_ncu * std::min(c_per_cu, 2));
  if (const char* g = getenv("C3H_TILE_GRID")) work = std::max<int64_t>(1, std::min<int64_t>(l.ntiles, atoi(g)));
  const int64_t zero = l.zero_empty ? std::min<int64_t>(64, l.ntiles) : 0;
  return std::max<int64_t>(work, 1) + zero;
}

hipError_t launch_c3hlac(const C3Launch& l, hipStream_t s) {
  // pass 1: occupancy flags + work list (flags/work zeroed by the caller)
  const int64_t nvox = (int64_t)l.gx * l.gy * l.gz;
  const bool vec = (l.gx & 3) == 0;
  const int64_t items = vec ? nvox / 4 : nvox;
  // HBM-bound: bytes in flight, not workgroups, set the rate; 256 B per lane lets few
  // workgroups (CU slots) cover the latency, leaving the rest to the other stages
  int occ_cap = 256;  // per frame: ~16 MB in flight at 64 KB per workgroup
  if (const char* g = getenv("C3H_OCC_GRID")) occ_cap = std::max(1, atoi(g));  // diagnostics
  const bool bits = vec && l.ntiles <= kOccBitsMax;
  const int unroll = bits ? kOccBitsUnroll : kOccUnroll;
  int g1 = (int)std::min<int64_t>((items + kBlock * unroll - 1) / (kBlock * unroll), occ_cap);
  if (g1 < 1) g1 = 1;
  if (l.nframes < 1 || l.nframes > kMaxBatch) return hipErrorInvalidValue;
  OccArgs oa;
  for (int f = 0; f < kMaxBatch; ++f) oa.grid[f] = f < l.nframes ? l.grid[f] : nullptr;
  oa.gx = l.gx;
  oa.gy = l.gy;
  oa.gz = l.gz;
  oa.axmap = l.axmap;
  oa.ns0 = l.nseg[0];
  oa.ns1 = l.nseg[1];
  oa.epoch = l.epoch;
  oa.tf = l.tf;
  oa.work = l.work;
  oa.s_tf = l.s_tf;
  oa.s_work = l.s_work;
  const dim3 g1d((unsigned)g1, (unsigned)l.nframes);
  const bool ax = l.gx + l.gy + l.gz <= kAxLds;
  oa.ntiles = (int)l.ntiles;
  if (bits) {
    const size_t lds = sizeof(uint32_t) * (size_t)((l.ntiles + 31) / 32);
    if (ax)
      c3_occupancy_bits_kernel<true><<<g1d, kBlock, lds, s>>>(oa);
    else
      c3_occupancy_bits_kernel<false><<<g1d, kBlock, lds, s>>>(oa);
  } else if (vec && ax)
    c3_occupancy_kernel<true, true><<<g1d, kBlock, 0, s>>>(oa);
  else if (vec)
    c3_occupancy_kernel<true, false><<<g1d, kBlock, 0, s>>>(oa);
  else if (ax)
    c3_occupancy_kernel<false, true><<<g1d, kBlock, 0, s>>>(oa);
  else
    c3_occupancy_kernel<false, false><<<g1d, kBlock, 0, s>>>(oa);
  KArgs a;
  for (int f = 0; f < kMaxBatch; ++f) a.grids[f] = f < l.nframes ? l.grid[f] : nullptr;
  a.s_feat = l.s_feat;
  a.s_h = l.s_h;
  a.s_acc = l.s_acc;
  a.s_tf = l.s_tf;
  a.s_work = l.s_work;
  a.grid = l.grid[0];
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
  const int tx_max = ((l.lmax[0] + 2) + 3 + 3) & ~3;
  a.tw_max = tx_max * (l.lmax[1] + 2) * (l.lmax[2] + 1);
  a.list_max = l.lmax[0] * l.lmax[1] * l.lmax[2];
  a.zero_feat = l.zero_feat;
  a.thr_r = l.thr[0];
  a.thr_g = l.thr[1];
  a.thr_b = l.thr[2];
  a.variant = l.variant;
  a.atomic = l.atomic;
  a.lut = l.lut;
  a.feat = l.feat;
  a.exist = l.exist;
  a.acc64 = l.acc64;
  a.tf = l.tf;
  a.flags = l.tf + 4;
  a.work = l.work;
  a.workcnt = l.tf + 2;
  a.rows = l.rows;
  a.epoch = l.epoch;
  a.zblocks = l.zero_empty ? (int)std::min<int64_t>(64, l.ntiles) : 0;
  a.ntiles = (int)l.ntiles;
  a.debug = l.debug;
  a.prof = l.prof;
  const size_t lds = c3hlac_lds_bytes(a.tw_max, a.list_max);
  const int grid = (int)c3hlac_grid(l);
  c3hlac_tile_kernel<<<dim3((unsigned)grid, (unsigned)l.nframes), kBlock, lds, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_c3_finalize(const unsigned long long* acc64, int64_t hist_num, int variant,
                              float* feat, int32_t* exist, int nframes, hipStream_t s) {
  c3_finalize_kernel<<<dim3((unsigned)hist_num, (unsigned)nframes), kBlock, 0, s>>>(acc64, variant, feat, exist,
                                                                                    hist_num);
  return hipGetLastError();
}

}  // namespace c3h
