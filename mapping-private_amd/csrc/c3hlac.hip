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

#include "c3hlac_dev.h"
#include "c3hlac_mfma.h"

namespace c3h {
namespace {

// kAx: the axis map lives in LDS, so the per-voxel tile lookup is LDS-only (no global
// load in the chain behind the stream data)
// Large stand-alone grids (config 5, >= 65,536 tiles): a sampled density check before the
// occupancy stream.  Every block reads the same 4,096 sampled words (a multiplicative-hash
// spread over the grid); when at least half of them are occupied the grid is dense -- the
// matrix-core body then takes every tile anyway (>= half non-empty) -- so every tile is
// stamped and listed (identity work list) and the 4 B/voxel occupancy stream is skipped.
// Empty tiles of such a grid are computed as zero rows with exist 0: the same result.
constexpr int kDenseSamples = 4096;
__global__ __launch_bounds__(kBlock) void dense_probe_kernel(OccArgs oa, uint32_t* dense) {
  __shared__ int s_cnt;
  const int tid = threadIdx.x;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const uint32_t* __restrict__ grid = oa.grid[0];
  const uint64_t nvox = (uint64_t)oa.gx * oa.gy * oa.gz;
  int c = 0;
  for (int j = tid; j < kDenseSamples; j += kBlock) {
    const uint64_t v = (((uint64_t)j + 1) * 0x9E3779B97F4A7C15ull >> 16) % nvox;
    c += grid[v] != 0u;
  }
  atomicAdd(&s_cnt, c);
  __syncthreads();
  const bool dn = 2 * s_cnt >= kDenseSamples;
  if (blockIdx.x == 0 && tid == 0) *dense = dn ? 1u : 0u;
  if (!dn) return;
  uint32_t* __restrict__ flags = oa.tf + 4;
  for (int t = blockIdx.x * kBlock + tid; t < oa.ntiles; t += gridDim.x * kBlock) {
    flags[t] = oa.epoch;
    oa.work[t] = t;
  }
  if (blockIdx.x == 0 && tid == 0) oa.tf[2 + (oa.epoch & 1)] = (uint32_t)oa.ntiles;
}

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

// c3h_extract of the grid the last c3h_voxelize wrote (round 6): the
// voxeliser's scatter listed every occupied voxel's grid index, so the tiles of the
// occupied centre voxels (c3_occupancy_kernel's rule: word != 0, every axis map >= 0) are
// stamped from that list -- ~4 B per occupied voxel instead of a 4 B/voxel stream of the
// whole grid (67 MB at 256^3 for ~0.3 % occupancy).  One workgroup per list segment;
// neighbouring entries mostly share a tile (the scatter lists them in point order), so a
// lane skips its predecessor's tile, the rest go through the LDS set and its flush.
__global__ __launch_bounds__(kBlock) void c3_list_stamp_kernel(OccArgs oa, const uint32_t* __restrict__ words,
                                                               const int32_t* __restrict__ counts, int seg,
                                                               int count_stride) {
  const int gx = oa.gx, gy = oa.gy, gz = oa.gz;
  const int ns0 = oa.ns0, ns1 = oa.ns1;
  const uint32_t epoch = oa.epoch;
  uint32_t* __restrict__ flags = oa.tf + 4;
  uint32_t* __restrict__ cnt = oa.tf + 2 + (epoch & 1);
  int32_t* __restrict__ work = oa.work;
  __shared__ int s_set[kOccSet];
  const int tid = threadIdx.x, lane = tid & 63;
  const int16_t* mx = oa.axmap;
  const int16_t* my = mx + gx;
  const int16_t* mz = my + gy;
  for (int i = tid; i < kOccSet; i += kBlock) s_set[i] = -1;
  __syncthreads();
  const int nn = counts[(size_t)blockIdx.x * count_stride];
  const uint32_t* wl = words + (size_t)blockIdx.x * seg;
  const uint32_t nvox = (uint32_t)gx * (uint32_t)gy * (uint32_t)gz;  // < 2^31 (host-checked)
  for (int i0 = 0; i0 < nn; i0 += kBlock) {  // wave-uniform trip count (the neighbour shuffle)
    const int i = i0 + tid;
    int t = -1;
    if (i < nn) {
      const uint32_t v = wl[i];
      if (v < nvox) {  // (kNoT entries: none on a completed voxelize)
        const uint32_t row = v / (uint32_t)gx;
        const int x = (int)(v - row * (uint32_t)gx);
        const int y = (int)(row % (uint32_t)gy), z = (int)(row / (uint32_t)gy);
        const int tx = mx[x], ty = my[y], tz = mz[z];
        if (tx >= 0 && ty >= 0 && tz >= 0) t = tx + ns0 * (ty + ns1 * tz);
      }
    }
    const int tp = __shfl_up(t, 1, 64);
    if (t >= 0 && !(lane > 0 && tp == t)) set_insert(s_set, t, epoch, flags, cnt, work);
  }
  __syncthreads();
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

// dense frames: one tile per wave on the i8 matrix cores (c3hlac_mfma.h)
#ifndef C3H_MF_MINB
#define C3H_MF_MINB 3
#endif
template <int LOAD>
__global__ __launch_bounds__(kBlock, C3H_MF_MINB) void c3hlac_mfma_kernel(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t mf_tab[kMfStaticWords];
  extern __shared__ __attribute__((aligned(16))) uint32_t mf_smem[];
  c3hlac_mfma_body<LOAD>(a, blockIdx.x * kMfWaves + (threadIdx.x >> 6), gridDim.x * kMfWaves, blockIdx.y, mf_tab,
                         mf_smem);
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

// Centroid-derived cells (voxelize.hip vox_centroid_kernel).  The tile pass adds every
// occupied voxel's centre contribution at its own cell; the reference takes the voxel's
// subdivision (floor(c / voxel_size) - min_b - offset, c3_hlac.cpp:349-354, skipped when
// negative) and its 13 neighbours (PCL getNeighborCentroidIndices: floor(c * inv_leaf) +
// relative coordinates, in-bounds only, c3_hlac.cpp:377) from its centroid c.  For each
// recorded off-cell voxel this adds the centroid-based contribution and subtracts the
// cell-based one in the exact 64-bit sums (two's complement), before c3_finalize_kernel.
// One thread per record (there are few).  A subdivision past the last one (a centroid
// rounding beyond max_b, out of bounds in the reference) contributes nothing.
struct OffcellArgs {
  const int32_t* rec;  // {linear index, neighbour-base cell xyz, subdivision cell xyz, 0}
  int nrec;
  const uint32_t* grid;
  int gx, gy, gz;
  int hist1;           // hist_num == 1: every voxel feeds histogram 0
  int off[3], sb[3];
  float inv_s;
  const uint32_t* lut;
  int thr[3];
  unsigned long long* acc64;
};

__device__ __forceinline__ void channels(uint32_t word, const uint32_t* lut, const int thr[3], int a[6], int beta[6]) {
  const int v[3] = {(int)((word >> 16) & 0xff), (int)((word >> 8) & 0xff), (int)(word & 0xff)};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const uint32_t l = lut[v[ch]];
    a[2 * ch] = (int)(l & 0xff);
    a[2 * ch + 1] = (int)((l >> 8) & 0xff);
    beta[2 * ch] = v[ch] > thr[ch] ? 1 : 0;
    beta[2 * ch + 1] = 1 - beta[2 * ch];
  }
}

// sign * (contribution of centre word `w` with subdivision cell `sc` and neighbour base `nb`)
__device__ void offcell_contrib(const OffcellArgs& o, uint32_t w, const int sc[3], const int nb[3], long long sign) {
  int64_t h = 0;
  if (!o.hist1) {
    int ijk[3];
    for (int ax = 0; ax < 3; ++ax) {
      const int t = sc[ax] - o.off[ax];
      if (t < 0) return;  // c3_hlac.cpp:355: voxels below the offset are skipped
      ijk[ax] = (int)floorf((float)t * o.inv_s);
      if (ijk[ax] >= o.sb[ax]) return;
    }
    h = ijk[0] + (int64_t)o.sb[0] * (ijk[1] + (int64_t)o.sb[1] * ijk[2]);
  }
  unsigned long long* hist = o.acc64 + h * 981;
  const unsigned long long sg = (unsigned long long)sign;
  int a[6], be[6];
  channels(w, o.lut, o.thr, a, be);
  for (int c = 0; c < 6; ++c) {
    if (be[c]) atomicAdd(&hist[495 + c], sg);
    atomicAdd(&hist[c], sg * (unsigned long long)a[c]);
    for (int n = c; n < 6; ++n) atomicAdd(&hist[474 + tri6(c, n)], sg * (unsigned long long)(a[c] * a[n]));
  }
  for (int c = 0; c < 4; ++c)
    for (int n = (c < 2 ? 2 : 4); n < 6; ++n)
      if (be[c] && be[n]) atomicAdd(&hist[c < 2 ? 969 + 4 * c + (n - 2) : 977 + 2 * (c - 2) + (n - 4)], sg);
  const int dims[3] = {o.gx, o.gy, o.gz};
  for (int k = 0; k < 13; ++k) {  // relative coordinates, c3_hlac.cpp:177-202
    const int rel[3] = {k < 9 ? k / 3 - 1 : (k < 12 ? k - 10 : -1), k < 9 ? k % 3 - 1 : (k < 12 ? -1 : 0),
                        k < 9 ? -1 : 0};
    int q[3];
    bool in = true;
    for (int ax = 0; ax < 3; ++ax) {
      q[ax] = nb[ax] + rel[ax];
      in = in && q[ax] >= 0 && q[ax] < dims[ax];
    }
    if (!in) continue;
    const uint32_t nw = o.grid[q[0] + (int64_t)o.gx * (q[1] + (int64_t)o.gy * q[2])];
    if (!nw) continue;
    int na[6], nbe[6];
    channels(nw, o.lut, o.thr, na, nbe);
    for (int c = 0; c < 6; ++c)
      for (int n = 0; n < 6; ++n) {
        atomicAdd(&hist[bin981(k, c, n)], sg * (unsigned long long)(a[c] * na[n]));
        if (be[c] && nbe[n]) atomicAdd(&hist[495 + bin981(k, c, n)], sg);
      }
  }
}

__global__ __launch_bounds__(64) void offcell_delta_kernel(OffcellArgs o) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= o.nrec) return;
  const int32_t* r = o.rec + 8 * (int64_t)i;
  const int64_t idx = r[0];
  const uint32_t w = o.grid[idx];
  const int own[3] = {(int)(idx % o.gx), (int)((idx / o.gx) % o.gy), (int)(idx / ((int64_t)o.gx * o.gy))};
  offcell_contrib(o, w, own, own, -1);
  const int nb[3] = {r[1], r[2], r[3]}, sc[3] = {r[4], r[5], r[6]};
  offcell_contrib(o, w, sc, nb, 1);
}

// ---- off-cell fixup of points-in batches (round 4; dot4 recompute, round 5) ------------
// After the tile role of a batch: for every voxel the exact pass moved (its centroid cell is
// not its own), the subdivisions of its own cell and of its centroid cell are recomputed
// from the canvas: every occupied cell of the subdivision as a centre at its own cell, except
// the moved voxels, which take their centroid cell as subdivision and neighbour base
// (c3_hlac.cpp:349-377).  The cell-centred part runs the tile body's exact dot4
// formulation (halo in LDS, compacted centres with the moved ones left out, packed
// operands, v_dot4_u32_u8); the moved voxels whose centroid lies in the subdivision add
// their bins by LDS atomics (round 4 did every centre that way: ~1,000 LDS atomics per
// centre on 981 shared bins, 179 us per 32-frame batch on the tick's stream).  Normalised as
// the tile role does; the exist gate is rewritten; a subdivision the tile role never saw is
// stamped and appended to the row list the compress role reads.  One workgroup per (frame,
// job), jobs deduplicated.
__device__ __forceinline__ int fix_centre_sub(const PointFixup& a, const int c[3], int* tile) {
  for (int ax = 0; ax < 3; ++ax)
    if (c[ax] < 0 || c[ax] >= a.C[ax]) return -1;
  const int ix = a.axmap[c[0]], iy = a.axmap[a.C[0] + c[1]], iz = a.axmap[a.C[0] + a.C[1] + c[2]];
  if (ix < 0 || iy < 0 || iz < 0) return -1;
  *tile = ix + a.ns0 * (iy + a.ns1 * iz);
  return a.segs[3 * ix + 2] + a.sbx * (a.segs[3 * (a.seg_stride + iy) + 2] +
                                       a.sby * a.segs[3 * (2 * a.seg_stride + iz) + 2]);
}

// centre word w at neighbour base b (canvas coordinates; the frame's grid is [0, dv)) into
// the 981-bin layout (117 is folded from it at the end, as the tile body does)
__device__ void fix_contrib(const PointFixup& a, const uint32_t* __restrict__ grid, const uint32_t* lut,
                            uint32_t w, const int b[3], const int dv[3], uint32_t* hist) {
  int ca[6], be[6];
  channels(w, lut, a.thr, ca, be);
  for (int c = 0; c < 6; ++c) {
    if (be[c]) atomicAdd(&hist[495 + c], 1u);
    atomicAdd(&hist[c], (uint32_t)ca[c]);
    for (int n = c; n < 6; ++n) atomicAdd(&hist[474 + tri6(c, n)], (uint32_t)(ca[c] * ca[n]));
  }
  for (int c = 0; c < 4; ++c)
    for (int n = (c < 2 ? 2 : 4); n < 6; ++n)
      if (be[c] && be[n]) atomicAdd(&hist[969 + (c < 2 ? 4 * c + (n - 2) : 8 + 2 * (c - 2) + (n - 4))], 1u);
  for (int k = 0; k < 13; ++k) {  // relative coordinates, c3_hlac.cpp:177-202
    const int rel[3] = {k < 9 ? k / 3 - 1 : (k < 12 ? k - 10 : -1), k < 9 ? k % 3 - 1 : (k < 12 ? -1 : 0),
                        k < 9 ? -1 : 0};
    int q[3];
    bool in = true;
    for (int ax = 0; ax < 3; ++ax) {
      q[ax] = b[ax] + rel[ax];
      in = in && q[ax] >= 0 && q[ax] < dv[ax];
    }
    if (!in) continue;
    const uint32_t nw = grid[q[0] + (int64_t)a.C[0] * (q[1] + (int64_t)a.C[1] * q[2])];
    if (!nw) continue;
    int na[6], nbe[6];
    channels(nw, lut, a.thr, na, nbe);
    for (int c = 0; c < 6; ++c)
      for (int n = 0; n < 6; ++n) {
        const int bn = bin981(k, c, n);
        atomicAdd(&hist[bn], (uint32_t)(ca[c] * na[n]));
        if (be[c] && nbe[n]) atomicAdd(&hist[495 + bn], 1u);
      }
  }
}

// dynamic LDS of point_fixup_kernel: lut | moved | jobs | misc | exclusion bits | halo | list | operands
__host__ __device__ inline int fix_halo_words(const int lmax[3]) { return (lmax[0] + 2) * (lmax[1] + 2) * (lmax[2] + 1); }
__host__ __device__ inline int fix_list_max(const int lmax[3]) { return lmax[0] * lmax[1] * lmax[2]; }
__host__ __device__ inline size_t fix_lds_words(const int lmax[3]) {
  return 256 + 4 * (size_t)kVbMovedCap + 4 * (size_t)kVbMovedCap + 4 + ((fix_list_max(lmax) + 127) / 128) * 4 +
         ((fix_halo_words(lmax) + 3) & ~3) + ((fix_list_max(lmax) + 7) / 8) * 4 + (size_t)kGroups * kArrStride;
}

__global__ __launch_bounds__(kBlock) void point_fixup_kernel(PointFixup a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t fx_smem[];
  uint32_t* s_lut = fx_smem;                                                     // 256
  VoxMoved* s_mv = reinterpret_cast<VoxMoved*>(s_lut + 256);                     // kVbMovedCap x 4 words
  int* s_h = reinterpret_cast<int*>(s_mv + kVbMovedCap);                         // 2 kVbMovedCap
  int* s_t = s_h + 2 * kVbMovedCap;                                              // 2 kVbMovedCap
  uint32_t* s_misc = reinterpret_cast<uint32_t*>(s_t + 2 * kVbMovedCap);         // 4
  const int list_max = fix_list_max(a.lmax);
  uint32_t* s_excl = s_misc + 4;                                                 // list_max bits
  uint32_t* s_tile = s_excl + ((list_max + 127) / 128) * 4;                      // halo words
  uint16_t* s_list = reinterpret_cast<uint16_t*>(s_tile + ((fix_halo_words(a.lmax) + 3) & ~3));
  uint32_t* s_arr = s_tile + ((fix_halo_words(a.lmax) + 3) & ~3) + ((list_max + 7) / 8) * 4;
  uint32_t* s_hist = s_arr;  // epilogue alias (981 words)
  const int f = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const VoxFrameRec& rec = a.info[f];
  const int nm = (int)min(a.xcnt[4 * f + 2], (uint32_t)kVbMovedCap);
  if (nm == 0 || rec.err) return;  // uniform
  if ((int)blockIdx.x >= 2 * nm) return;
  const uint32_t* __restrict__ grid = a.grid[f];
  const int Cx = a.C[0], Cy = a.C[1];
  const int dv[3] = {rec.max_b[0] - rec.min_b[0] + 1, rec.max_b[1] - rec.min_b[1] + 1,
                     rec.max_b[2] - rec.min_b[2] + 1};
  for (int i = tid; i < 256; i += kBlock) s_lut[i] = a.lut[i];
  for (int i = tid; i < nm; i += kBlock) {
    const VoxMoved m = a.moved[(size_t)f * kVbMovedCap + i];
    s_mv[i] = m;
    const int own[3] = {(int)(m.idx % (uint32_t)Cx), (int)((m.idx / (uint32_t)Cx) % (uint32_t)Cy),
                        (int)(m.idx / ((uint32_t)Cx * (uint32_t)Cy))};
    int t0 = -1, t1 = -1;
    s_h[2 * i] = fix_centre_sub(a, own, &t0);
    s_h[2 * i + 1] = fix_centre_sub(a, m.base, &t1);
    s_t[2 * i] = t0;
    s_t[2 * i + 1] = t1;
  }
  __syncthreads();
  float* ffeat = a.feat + (int64_t)f * a.s_feat;
  int32_t* fexist = a.exist + (int64_t)f * a.s_h;
  int32_t* frows = a.rows + (int64_t)f * a.s_h;
  uint32_t* ftf = a.tf + (int64_t)f * a.s_tf;
  const int at = tid / 90, arem = tid - at * 90, ak = arem / 6, an = arem - ak * 6;
  for (int j = blockIdx.x; j < 2 * nm; j += gridDim.x) {
    const int h = s_h[j], tile = s_t[j];
    bool skip = h < 0;
    for (int k = 0; k < j && !skip; ++k) skip = s_h[k] == h;  // recomputed by job k
    if (skip) continue;  // uniform
    const int sx = tile % a.ns0, sy = (tile / a.ns0) % a.ns1, sz = tile / (a.ns0 * a.ns1);
    const int x0 = a.segs[3 * sx], lx = a.segs[3 * sx + 1];
    const int y0 = a.segs[3 * (a.seg_stride + sy)], ly = a.segs[3 * (a.seg_stride + sy) + 1];
    const int z0 = a.segs[3 * (2 * a.seg_stride + sz)], lz = a.segs[3 * (2 * a.seg_stride + sz) + 1];
    const int TX = lx + 2, TY = ly + 2, TXY = TX * TY, V = lx * ly * lz;
    // the moved voxels whose own cell is a centre of this tile: left out of the cell-centred sum
    for (int i = tid; i < (V + 31) / 32; i += kBlock) s_excl[i] = 0u;
    if (tid == 0) s_misc[0] = 0;
    __syncthreads();
    for (int i = tid; i < nm; i += kBlock) {
      const uint32_t idx = s_mv[i].idx;
      const int cx = (int)(idx % (uint32_t)Cx) - x0, cy = (int)((idx / (uint32_t)Cx) % (uint32_t)Cy) - y0,
                cz = (int)(idx / ((uint32_t)Cx * (uint32_t)Cy)) - z0;
      if (cx >= 0 && cx < lx && cy >= 0 && cy < ly && cz >= 0 && cz < lz) {
        const int v = cx + lx * (cy + ly * cz);
        atomicOr(&s_excl[v >> 5], 1u << (v & 31));
      }
    }
    // 1. halo (lx+2) x (ly+2) x (lz+1) from (x0-1, y0-1, z0-1); outside the canvas: empty
    for (int e = tid; e < TXY * (lz + 1); e += kBlock) {
      const int qq = e / TX, rr = e - qq * TX;
      const int gx = x0 - 1 + rr, gy = y0 - 1 + qq % TY, gz = z0 - 1 + qq / TY;
      s_tile[e] = ((unsigned)gx < (unsigned)Cx && (unsigned)gy < (unsigned)Cy && (unsigned)gz < (unsigned)a.C[2])
                      ? grid[gx + (int64_t)Cx * (gy + (int64_t)Cy * gz)] : 0u;
    }
    __syncthreads();
    // 2. occupied centres, the moved ones left out
    for (int v0 = 0; v0 < V; v0 += kBlock) {
      const int v = v0 + tid;
      int ti = 0;
      bool occ = false;
      if (v < V) {
        const int cx = v % lx, cy = (v / lx) % ly, cz = v / (lx * ly);
        ti = (cx + 1) + (cy + 1) * TX + (cz + 1) * TXY;
        occ = s_tile[ti] != 0 && !((s_excl[v >> 5] >> (v & 31)) & 1u);
      }
      const unsigned long long m = __ballot(occ);
      if (m) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_misc[0], (uint32_t)__popcll(m));
        base = __shfl(base, 0, 64);
        if (occ) s_list[base + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)ti;
      }
    }
    __syncthreads();
    const int nlist = (int)s_misc[0];
    // 3-4. packed operands and exact dot4 accumulation (c3hlac_tile_body's steps 3-4)
    uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
    for (int c0 = 0; c0 < nlist; c0 += kChunk) {
      for (int job = tid; job < kGroups * 15; job += kBlock) {
        const int jg = job / 15, jk = job - jg * 15;
        const int rdx = jk <= 8 ? jk / 3 - 1 : (jk <= 11 ? jk - 10 : -1);
        const int rdy = jk <= 8 ? jk % 3 - 1 : (jk <= 11 ? -1 : 0);
        const int rdz = jk <= 8 ? -1 : 0;
        const int delta = jk < 13 ? rdx + rdy * TX + rdz * TXY : 0;
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int li = c0 + jg * 4 + q;
          w[q] = li < nlist ? s_tile[s_list[li] + delta] : 0u;
        }
        uint32_t nb[6] = {0, 0, 0, 0, 0, 0}, bb[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int sh = 8 * q;
          const uint32_t occ = w[q] ? 1u : 0u;
          const uint32_t m8 = occ ? 0xffu : 0u;
          if (jk == 14) {  // the ones column: occupancy in every channel
#pragma unroll
            for (int n = 0; n < 6; ++n) {
              nb[n] |= occ << sh;
              bb[n] |= occ << sh;
            }
          } else {
            const uint32_t r = (w[q] >> 16) & 0xffu, g = (w[q] >> 8) & 0xffu, bl = w[q] & 0xffu;
            const uint32_t lr = s_lut[r], lg = s_lut[g], lb = s_lut[bl];
            nb[0] |= (lr & m8) << sh;
            nb[1] |= ((lr >> 8) & m8) << sh;
            nb[2] |= (lg & m8) << sh;
            nb[3] |= ((lg >> 8) & m8) << sh;
            nb[4] |= (lb & m8) << sh;
            nb[5] |= ((lb >> 8) & m8) << sh;
            const uint32_t br = (int)r > a.thr[0], bgn = (int)g > a.thr[1], bbl = (int)bl > a.thr[2];
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
      __syncthreads();
      if (tid < 180) {
        const int ng = (min(nlist - c0, kChunk) + 3) >> 2;
        const uint32_t* col = s_arr + at * 90 + ak * 6 + an;
        const uint32_t* ctr = s_arr + at * 90 + 13 * 6;
        for (int g = 0; g < ng; ++g) {
          const uint32_t nv = col[g * kArrStride];
#pragma unroll
          for (int c = 0; c < 6; ++c) acc[c] = __builtin_amdgcn_udot4(ctr[g * kArrStride + c], nv, acc[c], false);
        }
      }
      __syncthreads();
    }
    // 5. the cell-centred bins, then the moved voxels whose centroid lies here
    for (int i = tid; i < 981; i += kBlock) s_hist[i] = 0u;
    __syncthreads();
    if (tid < 180) {
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        const int bi = bin_of(at, ak, an, c);
        if (bi >= 0) s_hist[bi] = acc[c];
      }
    }
    __syncthreads();
    for (int i = tid; i < nm; i += kBlock)
      if (s_h[2 * i + 1] == h) fix_contrib(a, grid, s_lut, grid[s_mv[i].idx], s_mv[i].base, dv, s_hist);
    __syncthreads();
    float* out = ffeat + (int64_t)h * a.variant;
    if (a.variant == 981) {
      for (int i = tid; i < 981; i += kBlock) out[i] = (float)s_hist[i] * norm981(i);
    } else {
      for (int i = tid; i < 117; i += kBlock) out[i] = (float)fold117(s_hist, i) * norm117(i);
    }
    if (tid == 0) {
      fexist[h] = exist_from((float)s_hist[0], (float)s_hist[1]);
      // a subdivision the tile role did not see: stamp it and list its row for the compress
      if (atomicExch(&ftf[4 + tile], a.epoch) != a.epoch) frows[atomicAdd(&ftf[2 + (a.epoch & 1)], 1u)] = h;
    }
    __syncthreads();  // LDS is reused by the next job
  }
}

}  // namespace

constexpr size_t kFixLdsMax = 160 * 1024;
bool point_fixup_fits(const int lmax[3]) { return 4 * fix_lds_words(lmax) <= kFixLdsMax; }

#ifndef C3H_FIX_BLOCKS
#define C3H_FIX_BLOCKS 8
#endif
hipError_t launch_point_fixup(const PointFixup& a, hipStream_t s) {
  if (a.nf <= 0) return hipSuccess;
  // jobs per frame: 2 per moved voxel; frames without moved voxels exit at once
  const size_t lds = 4 * fix_lds_words(a.lmax);
  if (lds > kFixLdsMax) return hipErrorInvalidValue;  // callers check point_fixup_fits first
  if (lds > 65536)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&point_fixup_kernel),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  // 8 workgroups per frame (round 6; 32 until round 5): a frame's jobs (2 per moved voxel,
  // ~2.4 per view on the reference's own Kinect views) loop over them, and the launch of a
  // batch without moved voxels is 512 empty workgroups, not 2,048 that queue behind the
  // voxeliser's 48 KB-LDS blocks for their own LDS (65-80 us on the tick's stream)
  point_fixup_kernel<<<dim3(C3H_FIX_BLOCKS, (unsigned)a.nf), kBlock, lds, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_offcell_delta(const int32_t* rec, int nrec, const C3Launch& l, int hist1, const int off[3],
                                const int sb[3], float inv_s, hipStream_t s) {
  if (nrec <= 0) return hipSuccess;
  OffcellArgs o{};
  o.rec = rec;
  o.nrec = nrec;
  o.grid = l.grid[0];
  o.gx = l.gx;
  o.gy = l.gy;
  o.gz = l.gz;
  o.hist1 = hist1;
  for (int ax = 0; ax < 3; ++ax) {
    o.off[ax] = off[ax];
    o.sb[ax] = sb[ax];
    o.thr[ax] = l.thr[ax];
  }
  o.inv_s = inv_s;
  o.lut = l.lut;
  o.acc64 = l.acc64;
  offcell_delta_kernel<<<(nrec + 63) / 64, 64, 0, s>>>(o);
  return hipGetLastError();
}

size_t c3hlac_lds_bytes(int tw_max, int list_max) {
  return sizeof(uint32_t) * (256 + tw_max + ((list_max + 7) / 8) * 4 + kGroups * kArrStride + 4 + 9 * kSegLds);
}

// C3-HLAC-117 per-wave tiles apply (exact u32 sums need <= ~5000 centres per tile; the
// halo must fit the prefetch registers)
bool wave117_ok(const C3Launch& l) {
  if (const char* e = diag_env("C3H_WAVE117"))  // diagnostics: 0 forces the block body
    if (!atoi(e)) return false;
  const int tw = w117_halo_words(l.lmax[0], l.lmax[1], l.lmax[2]);
  return l.variant == 117 && !l.atomic && l.debug == 0 && tw <= 64 * kW117HaloRegs &&
         w117_lds_bytes(tw, l.lmax[0] * l.lmax[1] * l.lmax[2]) <= 65536;
}

// persistent grid: every workgroup resident at once (occupancy from LDS and VGPRs)
int64_t c3hlac_grid(const C3Launch& l) {
  // work workgroups: two per CU (a frame's few hundred non-empty tiles finish in a couple
  // of rounds while the rest of the chip stays free for the other frames in flight),
  // capped by what is resident at once; plus the zero-role workgroups.  Per-wave tiles:
  // four tiles per workgroup in flight.
  const bool w117 = wave117_ok(l);
  const int tx_max = ((l.lmax[0] + 2) + 3 + 3) & ~3;
  const int list_max = l.lmax[0] * l.lmax[1] * l.lmax[2];
  const size_t lds = w117 ? w117_lds_bytes(w117_halo_words(l.lmax[0], l.lmax[1], l.lmax[2]), list_max)
                          : c3hlac_lds_bytes(tx_max * (l.lmax[1] + 2) * (l.lmax[2] + 1), list_max);
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
  const int64_t items = w117 ? (l.ntiles + kW117Waves - 1) / kW117Waves : l.ntiles;
  // dense grids (far more tiles than resident workgroups) take the whole chip: 512^3
  // dense C3-981 runs 28 % faster at full occupancy than at 2 workgroups per CU
  const int cap = items > (int64_t)c_ncu * 8 ? c_per_cu : std::min(c_per_cu, 2);
  int64_t work = std::min<int64_t>(items, (int64_t)c_ncu * cap);
  if (const char* g = diag_env("C3H_TILE_GRID")) work = std::max<int64_t>(1, std::min<int64_t>(items, atoi(g)));
  const int64_t zero = l.zero_empty ? std::min<int64_t>(64, l.ntiles) : 0;
  return std::max<int64_t>(work, 1) + zero;
}

// occupancy + tile pass arguments of one C3 launch (also used by the pipelined tick)
C3Args build_c3_args(const C3Launch& l) {
  C3Args c{};
  // pass 1: occupancy flags + work list (flags/work zeroed by the caller)
  const int64_t nvox = (int64_t)l.gx * l.gy * l.gz;
  const bool vec = (l.gx & 3) == 0;
  const int64_t items = vec ? nvox / 4 : nvox;
  // HBM-bound: bytes in flight, not workgroups, set the rate; 256 B per lane lets few
  // workgroups (CU slots) cover the latency, leaving the rest to the other stages
  int occ_cap = 256;  // per frame: ~16 MB in flight at 64 KB per workgroup
  if (const char* g = diag_env("C3H_OCC_GRID")) occ_cap = std::max(1, atoi(g));  // diagnostics
  c.bits = vec && l.ntiles <= kOccBitsMax;
  c.ax = l.gx + l.gy + l.gz <= kAxLds;
  c.vec = vec;
  const int unroll = c.bits ? kOccBitsUnroll : kOccUnroll;
  c.g1 = (int)std::max<int64_t>(1, std::min<int64_t>((items + kBlock * unroll - 1) / (kBlock * unroll), occ_cap));
  c.occ_lds = c.bits ? occ_bits_lds_bytes(l.ntiles) : 0;
  OccArgs& oa = c.oa;
  for (int f = 0; f < kMaxBatch; ++f) oa.grid[f] = f < l.nframes ? l.grid[f] : nullptr;
  oa.gx = l.gx;
  oa.gy = l.gy;
  oa.gz = l.gz;
  oa.axmap = l.axmap;
  oa.ar_s = kOccArith ? l.ar_s : 0;
  oa.ar_oy = l.ar_oy;
  oa.ar_oz = l.ar_oz;
  oa.ar_magic = l.ar_magic;
  oa.ns0 = l.nseg[0];
  oa.ns1 = l.nseg[1];
  oa.epoch = l.epoch;
  oa.tf = l.tf;
  oa.work = l.work;
  oa.s_tf = l.s_tf;
  oa.s_work = l.s_work;
  oa.contiguous = 0;  // the tick keeps the rotated order (frames' occupancy varies with y)
  oa.ntiles = (int)l.ntiles;
  KArgs& a = c.ka;
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
  a.feat16 = l.feat16;
  a.feat16_flag = l.feat16_flag;
  a.f16s = l.f16s;
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
  a.wave117 = wave117_ok(l) ? 1 : 0;
  a.mf_pb = mf_plane_bytes(l.lmax[0], l.lmax[1]);
  a.mfma = 0;  // set by launch_c3hlac (the stand-alone path), never in the tick
  if (a.wave117) a.tw_max = w117_halo_words(l.lmax[0], l.lmax[1], l.lmax[2]);
  c.tile_lds = a.wave117 ? w117_lds_bytes(a.tw_max, a.list_max) : c3hlac_lds_bytes(a.tw_max, a.list_max);
  c.tgrid = (int)c3hlac_grid(l);
  c.nframes = l.nframes;
  return c;
}

__global__ __launch_bounds__(kBlock) void feat16_to_f32_kernel(const _Float16* __restrict__ f16, int f16s,
                                                                const uint32_t* __restrict__ flag, int64_t H, int F,
                                                                float* __restrict__ out) {
  if (!*flag) return;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < H * F; i += (int64_t)gridDim.x * kBlock) {
    const int64_t h = i / F;
    out[i] = (float)f16[h * f16s + (i - h * F)];
  }
}

hipError_t launch_feat16_to_f32(const _Float16* f16, int f16s, const uint32_t* flag, int64_t H, int F, float* out,
                                hipStream_t s) {
  const int64_t g = std::min<int64_t>((H * F + kBlock - 1) / kBlock, 8192);
  if (g > 0) feat16_to_f32_kernel<<<(unsigned)g, kBlock, 0, s>>>(f16, f16s, flag, H, F, out);
  return hipGetLastError();
}

// dense-tile MFMA kernel: tiles up to 16 x 16 per layer, resident persistent grid
static bool mfma_ok(const C3Launch& l) { return l.lmax[0] <= 16 && l.lmax[1] <= 16 && l.debug == 0; }

static int64_t mfma_grid(const C3Launch& l, size_t lds) {
  static thread_local size_t c_lds = 0;
  static thread_local int c_per_cu = 0, c_ncu = 0, c_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (lds != c_lds || dev != c_dev) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c3hlac_mfma_kernel<kMfLoad>, kBlock, lds) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    int n_cu = 256;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    c_lds = lds;
    c_per_cu = per_cu;
    c_ncu = n_cu;
    c_dev = dev;
  }
  const int64_t tiles_per_block = kMfWaves;
  return std::max<int64_t>(1, std::min<int64_t>((l.ntiles + tiles_per_block - 1) / tiles_per_block,
                                                 (int64_t)c_ncu * c_per_cu));
}

hipError_t launch_c3hlac(const C3Launch& l, hipStream_t s) {
  if (l.nframes < 1 || l.nframes > kMaxBatch) return hipErrorInvalidValue;
  C3Args c = build_c3_args(l);
  // a grid stamped from the voxeliser's list is below 1/16 occupancy (extract_frames' rule):
  // its tiles are sparse whatever their count, so the dot4 body takes them all and the
  // matrix-core body is not launched (round 6: its early exit cost a launch, ~4.5 us)
  const bool mf = mfma_ok(l) && !(l.vl_words && l.nframes == 1);
  c.ka.mfma = mf ? 1 : 0;
#ifndef C3H_OCC_CONTIG
#define C3H_OCC_CONTIG 1
#endif
  c.oa.contiguous = C3H_OCC_CONTIG && l.ntiles >= 65536 ? 1 : 0;  // large grids (config 5): contiguous chunk ranges
  const dim3 g1d((unsigned)c.g1, (unsigned)l.nframes);
  if (l.vl_words && l.nframes == 1) {  // the voxeliser's list of occupied voxels
    if (l.vl_nseg > 0)
      c3_list_stamp_kernel<<<(unsigned)l.vl_nseg, kBlock, 0, s>>>(c.oa, l.vl_words, l.vl_counts, l.vl_seg,
                                                                  l.vl_count_stride);
  } else if (l.dense && l.nframes == 1 && c.bits && mf) {  // config 5: skip the stream of a dense grid
    dense_probe_kernel<<<64, kBlock, 0, s>>>(c.oa, l.dense);
    c.oa.dense = l.dense;
  }
  if (l.vl_words && l.nframes == 1) {
    // stamped above
  } else if (c.bits) {
    if (c.ax)
      c3_occupancy_bits_kernel<true><<<g1d, kBlock, c.occ_lds, s>>>(c.oa);
    else
      c3_occupancy_bits_kernel<false><<<g1d, kBlock, c.occ_lds, s>>>(c.oa);
  } else if (c.vec && c.ax)
    c3_occupancy_kernel<true, true><<<g1d, kBlock, 0, s>>>(c.oa);
  else if (c.vec)
    c3_occupancy_kernel<true, false><<<g1d, kBlock, 0, s>>>(c.oa);
  else if (c.ax)
    c3_occupancy_kernel<false, true><<<g1d, kBlock, 0, s>>>(c.oa);
  else
    c3_occupancy_kernel<false, false><<<g1d, kBlock, 0, s>>>(c.oa);
  c3hlac_tile_kernel<<<dim3((unsigned)c.tgrid, (unsigned)l.nframes), kBlock, c.tile_lds, s>>>(c.ka);
  if (mf) {  // both kernels read the frame's work count; each takes the frames of its kind
    const size_t lds = mf_lds_bytes(c.ka.mf_pb);
    const size_t dyn = mf_dyn_lds_bytes(c.ka.mf_pb);
    const dim3 g((unsigned)mfma_grid(l, lds), (unsigned)l.nframes);
    if (mf_load_items(l.lmax[0], l.lmax[1]) <= 1)
      c3hlac_mfma_kernel<1><<<g, kBlock, dyn, s>>>(c.ka);
    else
      c3hlac_mfma_kernel<kMfLoad><<<g, kBlock, dyn, s>>>(c.ka);
  }
  return hipGetLastError();
}

// exist_voxel_num of caller-supplied feature rows (c3h_set_features), with the reference's
// float / int arithmetic: rule 0 setC3HLAC ((f0 + f1) * 2 + 0.001, search_c3_hlac.h:60-61),
// 1 setVOSCH / setConVOSCH ((f20 + f21) * 2 + 0.001, search_new.h:41-43), 2 setGRSD (an
// int accumulating f0..f19 one float add at a time, then / 26, search_new.h:69-74)
__global__ void exist_rule_kernel(const float* __restrict__ feat, int64_t H, int dim, int rule,
                                  int32_t* __restrict__ exist) {
  for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < H; h += (int64_t)gridDim.x * blockDim.x) {
    const float* f = feat + h * dim;
    int32_t e;
    if (rule == 2) {
      e = 0;
      for (int i = 0; i < 20; ++i) e = (int32_t)((float)e + f[i]);
      e /= 26;
    } else {
      const int i0 = rule == 1 ? 20 : 0;
      const float t = (f[i0] + f[i0 + 1]) * 2.0f;
      e = (int32_t)((double)t + 0.001);
    }
    exist[h] = e;
  }
}

hipError_t launch_exist_rule(const float* feat, int64_t H, int dim, int rule, int32_t* exist, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((H + 255) / 256, 4096);
  exist_rule_kernel<<<(unsigned)std::max<int64_t>(blocks, 1), 256, 0, s>>>(feat, H, dim, rule, exist);
  return hipGetLastError();
}

hipError_t launch_c3_finalize(const unsigned long long* acc64, int64_t hist_num, int variant,
                              float* feat, int32_t* exist, int nframes, hipStream_t s) {
  c3_finalize_kernel<<<dim3((unsigned)hist_num, (unsigned)nframes), kBlock, 0, s>>>(acc64, variant, feat, exist,
                                                                                    hist_num);
  return hipGetLastError();
}

}  // namespace c3h
