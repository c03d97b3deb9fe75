// c3hlac_dev.h -- device bodies of the C3-HLAC stages (occupancy pass, tile pass),
// shared by the stand-alone kernels (c3hlac.hip) and the pipelined tick kernel
// (pipeline.hip).  Bodies take their block coordinates and LDS base explicitly so one
// launch can host several stages (block-role dispatch).  See c3hlac.hip for the method.
#pragma once
#include <type_traits>

#include "c3h_internal.h"

namespace c3h {

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
constexpr int kOccProbes = 32;  // linear-probe bound of the set

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
  // bounded probing: once the set is (nearly) full -- dense grids, tiny subdivisions --
  // a miss costs a few probes and a direct stamp, not a walk over the whole table
  for (int probe = 0; probe < kOccProbes; ++probe, h = (h + 1) & (kOccSet - 1)) {
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
  int contiguous;  // 1: workgroup b streams one contiguous chunk range (large stand-alone grids)
  // tail stealing (the tick, row-wave fast path only): each frame's chunks from steal_from
  // on are cut into units of steal_unit chunks and pooled over the nframes frames; a
  // workgroup done with its own chunks takes units off the pool (counter tf[0] of frame 0;
  // steal_wgs workgroups in the launch), streaming and flushing each into its frame's stamps
  int steal_from = 0, steal_unit = 0, steal_units = 0, nframes = 0, steal_wgs = 0;
  int ar_s = 0, ar_oy = 0, ar_oz = 0;  // closed-form y / z maps (C3Launch), 0 = the LDS maps
  uint32_t ar_magic = 0;
  // stand-alone large grids: dense_probe_kernel's verdict (non-zero: every tile was listed
  // and stamped, the stream is skipped); nullptr elsewhere (the tick)
  const uint32_t* dense = nullptr;
};

// Bitmap variant (every tile one bit of LDS, ntiles <= kOccBitsMax): an occupied centre
// voxel costs VALU plus one fire-and-forget ds_or, so no LDS round trip sits behind the
// stream data.  Per chunk the axis lookups are batched: x is fixed per lane whenever gx
// divides the chunk stride (4 voxels, at most 4 x-segments, looked up once per chunk),
// the 16 rows' (y, z) segments are looked up together.  The flush compacts the set bits
// into an LDS list and stamps kBlock tiles at a time, every exchange in flight together.
constexpr int kOccBitsMax = 1 << 18;  // 32 KB of LDS bits (512^3 at S >= 8)
// 16 loads per lane issued together, not software-pipelined: the same 64 VGPRs of data in
// flight as 2 x 8 pipelined, 4 % shorter tick (profiles/r1/v2_occ_variants.log, v3)
#ifndef C3H_OCC_UNROLL
#define C3H_OCC_UNROLL 16
#endif
#ifndef C3H_OCC_PIPE
#define C3H_OCC_PIPE 0
#endif
// occupied rows: a row's (y, z) subdivision by scalar arithmetic when the maps are uniform
#ifndef C3H_OCC_ARITH
#define C3H_OCC_ARITH 1
#endif
constexpr bool kOccArith = C3H_OCC_ARITH;
// occupied rows: a lane's (at most two) subdivisions precomputed (row-wave fast path)
#ifndef C3H_OCC_PAIR
#define C3H_OCC_PAIR 1
#endif
// rolling load ring over the whole chunks of the row-wave fast path (see there): 1 buffer
// loads, 2 global loads.  Off: the stream alone gets 1.3 % faster with it, but the whole
// tick 5-8 % slower -- a stream that never drains keeps the HBM queue longer for the
// latency-bound roles (profiles/r3/occ_ring_ab/)
#ifndef C3H_OCC_RING
#define C3H_OCC_RING 0
#endif
constexpr int kOccBitsUnroll = C3H_OCC_UNROLL;  // 16-B non-temporal loads per lane per chunk
constexpr bool kOccPipe = C3H_OCC_PIPE;         // next chunk's loads issued before this one is used
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
    if (!__syncthreads_or(m != 0u)) continue;  // no tile of these words touched (uniform)
    int total;
    const int base = block_excl_scan(__popc(m), s_wsum, &total);
    uint32_t mm = m;  // this thread's bits not yet listed (slices take them in order)
    int idx = base;
    for (int l0 = 0; l0 < total; l0 += kOccSet) {  // list slices of kOccSet tiles
      for (; mm && idx < l0 + kOccSet; ++idx) {  // each bit visited once over all slices
        const int bit = __ffs(mm) - 1;
        mm &= mm - 1;
        s_list[idx - l0] = wi * 32 + bit;
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

// LDS of the bitmap occupancy body: bits | list | wave sums | axis map
__host__ __device__ inline size_t occ_bits_lds_bytes(int64_t ntiles) {
  return 4 * (size_t)(((ntiles + 31) / 32 + 3) & ~3) + 4 * kOccSet + 4 * 16 + 2 * kAxLds;
}

// block bx of gdx for frame f; smem: occ_bits_lds_bytes(ntiles) bytes
template <bool kAx>
__device__ __forceinline__ void occupancy_bits_body(const OccArgs& oa, int bx, int f, int gdx, uint32_t* smem) {
  const uint32_t* __restrict__ grid = oa.grid[f];
  const int gx = oa.gx, gy = oa.gy, gz = oa.gz;
  const int ns0 = oa.ns0, ns1 = oa.ns1;
  const uint32_t epoch = oa.epoch;
  uint32_t* __restrict__ flags = oa.tf + f * oa.s_tf + 4;
  uint32_t* __restrict__ cnt = oa.tf + f * oa.s_tf + 2 + (epoch & 1);
  int32_t* __restrict__ work = oa.work + f * oa.s_work;
  uint32_t* s_bits = smem;  // ceil(ntiles / 32)
  int* s_list = reinterpret_cast<int*>(smem + ((((oa.ntiles + 31) >> 5) + 3) & ~3));
  int* s_wsum = s_list + kOccSet;
  int16_t* s_ax = reinterpret_cast<int16_t*>(s_wsum + 16);
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
  // kOccBitsUnroll 16-B loads per lane issued together (with kOccPipe, chunk c+1's loads
  // are issued before chunk c is processed: 2 x kOccBitsUnroll in flight).  Non-temporal: the grid
  // is read once here (the tile pass re-reads only the occupied tiles' halos); measured
  // 6.9-7.0 TB/s vs 6.0-6.3 for default-policy loads.  Past the grid end the address is
  // clamped and the value zeroed (no per-element branch around the load).
  const int64_t cstride = (int64_t)gdx * kChunk4;
  auto load_chunk = [&](uint4 (&dst)[kOccBitsUnroll], int64_t c) {
#pragma unroll
    for (int j = 0; j < kOccBitsUnroll; ++j) {
      const int64_t i = c + j * kBlock + tid;
      const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(g4) + (i < n4 ? i : n4 - 1));
      dst[j] = i < n4 ? make_uint4(t.x, t.y, t.z, t.w) : make_uint4(0, 0, 0, 0);
    }
  };
  // Row-wave fast path (gx = 256, 512 or 1024, axis maps in LDS): a wave's 64 lanes x 4
  // voxels of step j are 256 consecutive voxels of ONE grid row (chunk, wave and j offsets
  // are multiples of 256 and j steps whole rows), so the row's (y, z) segment is
  // wave-uniform: its two lookups per j are uniform-address LDS reads, all 2 x unroll issued
  // together and moved to SGPRs, and a lane's 4 x-segments are loop invariant.  The general
  // path below steps and looks up (x, y, z) per lane and per j.
  if (kAx && (gx & 255) == 0 && 1024 % gx == 0) {
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int rpj = (kBlock * 4) / gx;                 // rows per j step
    const int xl = (wv * 256) % gx + 4 * (tid & 63);   // this lane's x (every chunk, every j)
    int tx0[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) tx0[k] = mx[xl + k];
    // A lane's 4 voxels lie in at most two subdivisions along x when S >= 4: precompute
    // them (tA, tB) and which voxels each holds (mA, mB), so an occupied row costs a lane
    // two masked LDS ors from a 4-bit occupancy code instead of four tests and ors
    // (the stream's per-slot instructions are on the tick's critical path)
    int tA = -1, tB = -1;
    uint32_t mA = 0, mB = 0;
    bool cplx = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (tx0[k] < 0) continue;
      if (tA < 0 || tx0[k] == tA) {
        tA = tx0[k];
        mA |= 1u << k;
      } else if (tB < 0 || tx0[k] == tB) {
        tB = tx0[k];
        mB |= 1u << k;
      } else {
        cplx = true;
      }
    }
    const bool pair_ok = C3H_OCC_PAIR && __ballot(cplx) == 0ull;  // uniform
    // Chunk i of this workgroup is chunk i * gdx + (bx + i) % gdx of the frame: rotated, so
    // every workgroup visits every y band of the grid (a fixed stride would give workgroup
    // bx the same rows of every plane, and frames' occupancy varies with y: the workgroups of
    // one frame ended up to 70 us apart, profiles/r1/tq3_occ_spread.txt).
    const int lg = gx == 256 ? 8 : gx == 512 ? 9 : 10;
    const int64_t nch = (n4 + kChunk4 - 1) / kChunk4;
    uint4 w[kOccBitsUnroll];
    // large stand-alone grids: contiguous ranges (a tile's 10 planes meet few workgroups,
    // so the flush stamps each tile ~2.5x fewer times on a dense 512^3 frame)
    const int64_t per = (nch + gdx - 1) / gdx;
    auto chunk_of = [&](int64_t i) {
      return oa.contiguous ? (i < per ? bx * per + i : nch) : i * gdx + (bx + i) % gdx;
    };
    // the tick's tail stealing (row-wave path): this frame's own chunks end at nstat
    const int64_t nstat = oa.steal_unit > 0 ? oa.steal_from : nch;
    // rows are mostly empty: skip a row unless some lane of the wave holds a voxel of it
    // (one ballot), look its (y, z) segment up only then
    auto proc = [&](uint32_t row0) {
      int y = (int)(row0 % (uint32_t)gy), z = (int)(row0 / (uint32_t)gy);
#pragma unroll
      for (int j = 0; j < kOccBitsUnroll; ++j) {
        const int yj = y, zjj = z;
        y += rpj;
        while (y >= gy) {
          y -= gy;
          ++z;
        }
        const uint32_t ws[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
        if (__ballot((ws[0] | ws[1] | ws[2] | ws[3]) != 0u) == 0ull || zjj >= gz) continue;
        int a, b;
        if (oa.ar_s) {  // uniform: scalar arithmetic, no LDS round trip
          a = yj >= oa.ar_oy ? (int)__umulhi((uint32_t)(yj - oa.ar_oy), oa.ar_magic) : -1;
          b = zjj >= oa.ar_oz ? (int)__umulhi((uint32_t)(zjj - oa.ar_oz), oa.ar_magic) : -1;
        } else {
          a = __builtin_amdgcn_readfirstlane(my[yj]);
          b = __builtin_amdgcn_readfirstlane(mz[zjj]);
        }
        if (a < 0 || b < 0) continue;  // uniform: not a centre row
        const int tyz = ns0 * (a + ns1 * b);
        if (pair_ok) {  // any non-zero word is occupied (as in the general path and the tile pass)
          const uint32_t o = min(ws[0], 1u) | (min(ws[1], 1u) << 1) | (min(ws[2], 1u) << 2) | (min(ws[3], 1u) << 3);
          const int ta = tA + tyz, tb = tB + tyz;
          if (o & mA) atomicOr(&s_bits[ta >> 5], 1u << (ta & 31));
          if (o & mB) atomicOr(&s_bits[tb >> 5], 1u << (tb & 31));
          continue;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int t = tx0[k] + tyz;
          if (ws[k] && tx0[k] >= 0 && t != last) {
            last = t;
            atomicOr(&s_bits[t >> 5], 1u << (t & 31));
          }
        }
      }
    };
#if C3H_OCC_RING
    // Rolling ring over whole chunks: slot j of the next chunk is loaded the moment slot j
    // of this chunk has been read, so each lane keeps kOccBitsUnroll loads in flight all
    // the time (the oldest is always the one waited for: vmcnt(unroll - 1)) instead of
    // draining to zero at every chunk end.  The loads carry no predicate (whole chunks
    // only), so none is sunk into a branch (a predicated load forces vmcnt(0) before the
    // first use).  A partial last chunk, if any, takes the loop below.
    const int64_t nfull = min(n4 / kChunk4, nstat);  // whole chunks of this frame's own share
    int64_t ri = 0;
    if (chunk_of(0) < nfull) {
      // buffer loads off a per-chunk descriptor: one address VGPR (tid * 16) for all
      // slots, the slot offset j * 4 KB in an SGPR, non-temporal (aux 2)
      const uint32_t voff = (uint32_t)tid * 16u;
#if C3H_OCC_RING == 2  // diagnostics: global loads off a per-chunk base
      auto chunk_rsrc = [&](int64_t c) { return reinterpret_cast<const char*>(g4 + c * kChunk4); };
      auto ring_load = [&](const char* r, int j) {
        return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(r + voff + j * kBlock * 16));
      };
#else
      auto chunk_rsrc = [&](int64_t c) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(g4 + c * kChunk4), (short)0, kChunk4 * 16, 0x00020000);
      };
      auto ring_load = [&](__amdgpu_buffer_rsrc_t r, int j) {
        return __builtin_amdgcn_raw_buffer_load_b128(r, voff, j * kBlock * 16, 2);
      };
#endif
      int64_t cur = chunk_of(0);
      {
        const auto r = chunk_rsrc(cur);
#pragma unroll
        for (int j = 0; j < kOccBitsUnroll; ++j) {
          const v4u t = ring_load(r, j);
          w[j] = make_uint4(t.x, t.y, t.z, t.w);
        }
      }
      // one chunk; kIssue: slot j of chunk nxt is loaded right after slot j is read
      auto run_chunk = [&](auto issue, int64_t c, int64_t nxt) {
        const uint32_t row0 = (uint32_t)(((uint64_t)c * kChunk4 * 4 + (uint64_t)wv * 256) >> lg);
        int y = (int)(row0 % (uint32_t)gy), z = (int)(row0 / (uint32_t)gy);
        const auto rn = chunk_rsrc(decltype(issue)::value ? nxt : c);
        auto refill = [&](int j) {  // slot j of the next chunk, once slot j is consumed
          if constexpr (decltype(issue)::value) {
            const v4u t = ring_load(rn, j);
            w[j] = make_uint4(t.x, t.y, t.z, t.w);
          }
        };
#pragma unroll
        for (int j = 0; j < kOccBitsUnroll; ++j) {
          if (j > 0) refill(j - 1);  // the previous slot is dead: its registers are reused
          const uint32_t ws[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
          const int yj = y, zjj = z;
          y += rpj;
          while (y >= gy) {
            y -= gy;
            ++z;
          }
          if (__ballot((ws[0] | ws[1] | ws[2] | ws[3]) != 0u) == 0ull || zjj >= gz) continue;
          const int a = __builtin_amdgcn_readfirstlane(my[yj]), b = __builtin_amdgcn_readfirstlane(mz[zjj]);
          if (a < 0 || b < 0) continue;  // uniform: not a centre row
          const int tyz = ns0 * (a + ns1 * b);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int t = tx0[k] + tyz;
            if (ws[k] && tx0[k] >= 0 && t != last) {
              last = t;
              atomicOr(&s_bits[t >> 5], 1u << (t & 31));
            }
          }
        }
        refill(kOccBitsUnroll - 1);
      };
      for (;;) {  // chunk_of is increasing: the ring covers exactly the chunks below nfull
        const int64_t nxt = chunk_of(ri + 1);
        ++ri;
        if (nxt < nfull) {  // uniform
          run_chunk(std::true_type{}, cur, nxt);
          cur = nxt;
        } else {
          run_chunk(std::false_type{}, cur, 0);
          break;
        }
      }
    }
    for (int64_t i = ri; i * gdx < nch; ++i) {
      if (chunk_of(i) < nfull) continue;  // streamed by the ring (uniform)
#else
    if (kOccPipe && chunk_of(0) < nch) load_chunk(w, chunk_of(0) * kChunk4);
    for (int64_t i = 0; i * gdx < nch; ++i) {
#endif
      const int64_t cidx = chunk_of(i);
      if (cidx >= nstat) continue;  // uniform: the last, partial round / the pooled tail
      const int64_t c0 = cidx * kChunk4;
      uint4 nx[kOccBitsUnroll];
      if constexpr (kOccPipe) {  // the next chunk's loads in flight while this one is processed
        const int64_t cn = chunk_of(i + 1);
        if (cn < nch) load_chunk(nx, cn * kChunk4);
      } else {
        load_chunk(w, c0);
      }
      // uniform 32-bit row arithmetic (rows < 2^24: nvox < 2^32 is host-checked): the
      // chunk's first row, then (y, z) stepped by whole rows per j
      const uint32_t row0 = (uint32_t)(((uint64_t)c0 * 4 + (uint64_t)wv * 256) >> lg);
#ifdef C3H_OCC_NOPROC  // diagnostics: stream only (the words are OR-reduced into one bit)
      {
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < kOccBitsUnroll; ++j) o |= w[j].x | w[j].y | w[j].z | w[j].w;
        if (o == 0x12345678u) atomicOr(&s_bits[0], 1u);
        continue;
      }
#endif
      proc(row0);
      if constexpr (kOccPipe) {
#pragma unroll
        for (int j = 0; j < kOccBitsUnroll; ++j) w[j] = nx[j];
      }
    }
    __syncthreads();
    occ_flush_bits(s_bits, nwords, s_list, s_wsum, epoch, flags, cnt, work);
    if (oa.steal_unit > 0) {  // the pooled tails of every frame of the launch
      // self-resetting: every workgroup's last dequeue fails; the last of those (counted in
      // tf[1]) returns both words to 0 for the next launch on this buffer set
      uint32_t* pool = oa.tf;
      for (;;) {
        __syncthreads();  // the flush is done with the bitmap, list and scan scratch
        if (tid == 0) s_wsum[15] = (int)atomicAdd(pool, 1u);
        __syncthreads();
        const int u = s_wsum[15];
        if (u >= oa.steal_units) {  // uniform
          if (tid == 0 && atomicAdd(oa.tf + 1, 1u) == (uint32_t)oa.steal_wgs - 1) {
            atomicExch(pool, 0u);
            atomicExch(oa.tf + 1, 0u);
          }
          break;
        }
        const int fu = u % oa.nframes, ju = u / oa.nframes;
        for (int i = tid; i < nwords; i += kBlock) s_bits[i] = 0u;
        last = -1;  // another frame's bitmap
        g4 = reinterpret_cast<const uint4*>(oa.grid[fu]);
        __syncthreads();
        const int64_t cb = nstat + (int64_t)ju * oa.steal_unit, ce = min(nch, cb + oa.steal_unit);
        for (int64_t c = cb; c < ce; ++c) {
          load_chunk(w, c * kChunk4);
          proc((uint32_t)(((uint64_t)c * kChunk4 * 4 + (uint64_t)wv * 256) >> lg));
        }
        __syncthreads();
        occ_flush_bits(s_bits, nwords, s_list, s_wsum, epoch, oa.tf + fu * oa.s_tf + 4,
                       oa.tf + fu * oa.s_tf + 2 + (epoch & 1), oa.work + fu * oa.s_work);
      }
    }
    return;
  }
  uint4 w[kOccBitsUnroll];
  int64_t c0 = bx * (int64_t)kChunk4;
  if (c0 < n4) load_chunk(w, c0);
  for (; c0 < n4; c0 += cstride) {
    uint4 nx[kOccBitsUnroll];
    if (kOccPipe && c0 + cstride < n4) load_chunk(nx, c0 + cstride);
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
    if (kOccPipe) {
#pragma unroll
      for (int j = 0; j < kOccBitsUnroll; ++j) w[j] = nx[j];
    } else if (c0 + cstride < n4) {
      load_chunk(w, c0 + cstride);
    }
  }
  __syncthreads();
  occ_flush_bits(s_bits, nwords, s_list, s_wsum, epoch, flags, cnt, work);
}

namespace {
template <bool kAx>
__global__ __launch_bounds__(kBlock) void c3_occupancy_bits_kernel(OccArgs oa) {
  extern __shared__ __attribute__((aligned(16))) uint32_t occ_smem[];
  if (oa.dense && *oa.dense) return;  // uniform: a dense grid's tiles are all listed already
  occupancy_bits_body<kAx>(oa, blockIdx.x, blockIdx.y, gridDim.x, occ_smem);
}
}  // namespace



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
  int wave117;      // C3-HLAC-117 per-wave tiles (c3hlac_wave117_body), else the block body
  int mfma;         // the dense-tile MFMA kernel runs beside (c3hlac_mfma.h): frames with
                    // >= half of their tiles non-empty are left to it
  int mf_pb;        // its largest channel-plane size (mf_plane_bytes of the largest tile)
  _Float16* feat16;     // C3Launch::feat16 (nullable), its row stride, the frame's flag
  uint32_t* feat16_flag;
  int f16s;
  int debug;  // diagnostics only (C3H_C3_DEBUG): 1 stop after the loads, 2 after compaction,
             // 3 skip the tile kernel
};

constexpr int kMaxLoads = 4;  // uint4 tile loads per thread kept in flight together
constexpr int kSegLds = 64;   // segment tables up to 64 segments per axis live in LDS
#ifndef C3H_TILE_PREFETCH
#define C3H_TILE_PREFETCH 0  // 1: the next tile's halo into LDS by global_load_lds during this tile's dot4 + epilogue (measured neutral, round 6: DESIGN §8)
#endif
// 16 zero bytes: the LDS-DMA source of halo words outside the grid (a lane's LDS-DMA
// destination is fixed by its lane index, so it cannot be skipped, only pointed at zeros)
static __device__ const uint4 kHaloZero16 = {0u, 0u, 0u, 0u};

// The (vec-path) halo geometry of a tile: its rows of q4 16-byte pieces starting at x = xs
struct HaloGeo {
  int y0, z0, ly, TY, q4, n, xs;
  bool vec;
};
__device__ __forceinline__ HaloGeo halo_geo(const KArgs& a, const int32_t* segs, int tile);

// Persistent workgroups.  Phase Z zero-fills the feature rows of the tiles pass 1 left
// unflagged (direct mode); phase T walks the work list: stage the (lx+2)x(ly+2)x(lz+1)
// halo in LDS (all loads issued before the first LDS store), compact the occupied
// centres, build the packed dot4 operands and accumulate exactly (see the header).
#define C3H_PROF(k, cond) \
  if (fprof && tid == 0 && (cond)) fprof[bx * 8 + (k)] = (long long)wall_clock64()

__device__ __forceinline__ HaloGeo halo_geo(const KArgs& a, const int32_t* segs, int tile) {
  const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
  const int32_t* sx = segs + 3 * ix;
  const int32_t* sy = segs + 3 * (a.seg_stride + iy);
  const int32_t* sz = segs + 3 * (2 * a.seg_stride + iz);
  HaloGeo g;
  const int x0 = sx[0], lx = sx[1];
  g.y0 = sy[0];
  g.ly = sy[1];
  g.z0 = sz[0];
  const int lz = sz[1];
  g.vec = (a.gx & 3) == 0 && x0 >= 1 && ((x0 + lx + 1 + 3) & ~3) <= a.gx;
  g.xs = g.vec ? ((x0 - 1) & ~3) : x0 - 1;
  const int TX = g.vec ? (((x0 + lx + 1 - g.xs) + 3) & ~3) : lx + 2;
  g.TY = g.ly + 2;
  g.q4 = TX >> 2;
  g.n = g.TY * (lz + 1) * g.q4;
  return g;
}

// block bx of gdx for frame fy; smem: c3hlac_lds_bytes(tw_max, list_max) bytes
__device__ __forceinline__ void c3hlac_tile_body(const KArgs& a, int bx, int fy_, int gdx, uint32_t* smem) {
  // this frame's buffers; the argument struct itself is not copied
  const int64_t fy = fy_;
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
  if (bx == 0 && tid == 0) {  // the next frame's counters
    fworkcnt[(a.epoch + 1) & 1] = 0;
  }
  if (bx < a.zblocks) {
    // zero role (direct mode, every subdivision one tile: h == tile): exist of the tiles
    // pass 1 left unstamped (their feature rows stay stale unless zero_feat)
    if (!a.zero_feat) {
      for (int t = bx * kBlock + tid; t < a.ntiles; t += a.zblocks * kBlock)
        if (fflags[t] != a.epoch) fexist[t] = 0;
      return;
    }
    // rows too, one wave-wide store per 64 floats
    for (int t0 = bx * kBlock; t0 < a.ntiles; t0 += a.zblocks * kBlock) {
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
  const int G = gdx - a.zblocks;
  int wi = bx - a.zblocks;
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

  if (a.mfma && 2 * nwork >= a.ntiles) return;  // dense frame: c3hlac_mfma_body takes it
  bool pre = false;  // s_tile already holds this tile's halo (prefetched by the previous tile)
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

    // 1. halo tile; every load of a thread is issued before its first LDS store (or, when
    //    the previous tile prefetched it, the LDS-DMA retired here)
    if (pre) {
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (vec) {
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
    pre = false;  // consumed; the last chunk below may prefetch the next tile
    C3H_PROF(3, wi == bx - a.zblocks);
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
    C3H_PROF(4, wi == bx - a.zblocks);
    const int nlist = (int)s_misc[0];
    if (a.debug == 2) {
      if (tid == 0 && nlist == 0x7fffffff) fexist[0] = 1;
      lds_barrier();
      continue;
    }

    uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
    for (int c0 = 0; c0 < nlist; c0 += kChunk) {
      // 3. build packed operands for list entries [c0, c0+kChunk): job = (group, k);
      //    branch-free so each job's LDS reads (list, tile, LUT) issue back to back.  Only
      //    the chunk's groups: a surface tile holds a few dozen centres, and the dot4 pass
      //    reads groups g < ng only (round 6: the 32 groups were all built before)
      const int njobs = ((min(nlist - c0, kChunk) + 3) >> 2) * 15;
      for (int job = tid; job < njobs; job += kBlock) {
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
      C3H_PROF(2, c0 == 0 && wi == bx - a.zblocks);
      if (c0 + kChunk >= nlist) {
        // the last chunk's operands are built: s_tile is free, so the next tile's halo goes
        // into it by LDS-DMA while this tile's dot4 and epilogue run (round 6; the halo's
        // global latency was ~2 of ~6.6 us per surface tile).  Retired by the vmcnt wait
        // at the next tile's phase 1; lds_barrier keeps it in flight (no vmcnt).
        if (C3H_TILE_PREFETCH && wi + G < nwork) {
          const HaloGeo g = halo_geo(a, segs, tile_next);
          if (g.vec && g.n <= kMaxLoads * kBlock) {
            pre = true;
            int q = tid / g.q4, r = tid - q * g.q4;
            const int sq = kBlock / g.q4, sr = kBlock - sq * g.q4;
#pragma unroll
            for (int j = 0; j < kMaxLoads; ++j) {
              const int e = tid + j * kBlock;
              if (j * kBlock >= g.n) break;  // uniform
              if (e < g.n) {
                const int gy = g.y0 - 1 + q % g.TY, gz = g.z0 - 1 + q / g.TY;
                const uint4* src = ((unsigned)gy < (unsigned)a.gy && (unsigned)gz < (unsigned)a.gz)
                                       ? reinterpret_cast<const uint4*>(fgrid + ((int64_t)gz * a.gy + gy) * a.gx + g.xs + 4 * r)
                                       : &kHaloZero16;
                // wave-uniform LDS base + lane * 16: element e lands at s_tile[4 e]
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 reinterpret_cast<void*>(s_tile + 4 * (j * kBlock + (tid & ~63))),
                                                 16, 0, 0);
              }
              q += sq;
              r += sr;
              if (r >= g.q4) {
                r -= g.q4;
                ++q;
              }
            }
          }
        }
      }
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
    C3H_PROF(5, wi == bx - a.zblocks);
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
    C3H_PROF(6, wi == bx - a.zblocks);
  }
  C3H_PROF(7, true);
}

// ---------------------------------------------------------------- pass 2, per wave (117)
// C3-HLAC-117 with one tile per wave.  Every 117 bin is an exact integer dot product over
// the tile's occupied centre voxels v of two per-voxel channels X(v) * Y(v) taken from
//   0 ones | 1..6 A_c (sin/cos LUT bytes r,r_,g,g_,b,b_) | 7..12 b_c (beta, 1-beta per
//   colour) | 13..18 N_n = sum_k A_n(w_k) | 19..24 B_n = sum_k b_n(w_k)
// over the 13 half-neighbourhood offsets k (c3_hlac.cpp:177-202; empty / off-grid
// neighbours add 0): the rotation-invariant feature sums the 981 first-order bins over k
// (color_chlac.hpp:1647-1743), so A_c(v) * sum_k A_n(w_k) is exactly its (c, n) bin.
// Channel values fit u16 (N_n <= 13 * 255), so one v_dot2_u32_u16 is two voxel-MACs and
// every sum stays exact in u32 (<= 13 * 255 * 255 * S^3 < 2^32 for S <= 10).
// Waves are independent (no workgroup barrier after the shared LUT / segment tables are
// staged): each walks the dense work list with stride = all waves of its frame, keeps the
// next tile's halo in registers while it computes the current one, and owns an LDS slice:
//   halo (lx+2)(ly+2)(lz+1) packed words | centre list (u16) | channel table [25][kCh]
constexpr int kW117Ch = 25;
constexpr int kW117ChStride = 36;  // dwords per channel row (64 u16 + pad: 16-B aligned rows 4 banks apart)
constexpr int kW117HaloRegs = 26;  // halo dwords per lane kept in flight (<= 1664-word halos)
constexpr int kW117Waves = 3;      // tile waves per workgroup (the 4th exits: LDS <= 40 KB at S=10)

__host__ __device__ inline int w117_halo_words(int lx, int ly, int lz) { return (lx + 2) * (ly + 2) * (lz + 1); }
// per-wave LDS words (halo + list + channel table), 4-dword aligned
__host__ __device__ inline int w117_wave_words(int tw, int list_max) {
  return ((tw + 3) & ~3) + (((list_max + 1) / 2 + 3) & ~3) + kW117Ch * kW117ChStride;
}
__host__ __device__ inline size_t w117_lds_bytes(int tw, int list_max) {
  return 4 * ((size_t)256 + 9 * kSegLds + kW117Waves * (size_t)w117_wave_words(tw, list_max));
}

// channels (X, Y) of 117-bin b (Appendix A of SURVEY.md; the same layout fold117 builds)
__device__ __forceinline__ void w117_bin_channels(int b, int& X, int& Y) {
  if (b < 6) { X = 0; Y = 1 + b; }                                        // zero order
  else if (b < 42) { X = 1 + (b - 6) / 6; Y = 13 + (b - 6) % 6; }         // A_c * N_n
  else if (b < 63) {                                                      // auto upper triangle
    int t = b - 42, c = 0;
    while (t >= 6 - c) { t -= 6 - c; ++c; }
    X = 1 + c; Y = 1 + c + t;
  } else if (b < 69) { X = 0; Y = 7 + (b - 63); }                         // bin zero order
  else if (b < 105) { X = 7 + (b - 69) / 6; Y = 19 + (b - 69) % 6; }      // b_c * B_n
  else {                                                                  // bin pair counts
    const int t = b - 105;
    if (t < 8) { X = 7 + t / 4; Y = 7 + 2 + t % 4; }
    else { X = 7 + 2 + (t - 8) / 2; Y = 7 + 4 + (t - 8) % 2; }
  }
}

// zero role: exist (and with zero_feat the feature rows) of the tiles pass 1 left
// unstamped (direct mode, every subdivision one tile: h == tile)
__device__ __forceinline__ void c3_zero_role(const KArgs& a, int bx, const uint32_t* fflags, float* ffeat,
                                             int32_t* fexist) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (!a.zero_feat) {
    for (int t = bx * kBlock + tid; t < a.ntiles; t += a.zblocks * kBlock)
      if (fflags[t] != a.epoch) fexist[t] = 0;
    return;
  }
  for (int t0 = bx * kBlock; t0 < a.ntiles; t0 += a.zblocks * kBlock) {
    const int t = t0 + tid;
    unsigned long long m = __ballot(t < a.ntiles && fflags[t] != a.epoch);
    while (m) {
      const int q = __ffsll((long long)m) - 1;
      m &= m - 1;
      const int tj = (t0 + (tid & ~63)) + q;
      float* row = ffeat + (int64_t)tj * a.variant;
      for (int c = lane; c < a.variant; c += 64) row[c] = 0.0f;
      if (lane == 0) fexist[tj] = 0;
    }
  }
}

struct W117Geom {
  int x0, lx, y0, ly, z0, lz;
  int64_t h;
};

__device__ __forceinline__ W117Geom w117_geom(const KArgs& a, const int32_t* segs, int tile) {
  const int ix = tile % a.ns0, iy = (tile / a.ns0) % a.ns1, iz = tile / (a.ns0 * a.ns1);
  const int32_t* sx = segs + 3 * ix;
  const int32_t* sy = segs + 3 * (a.seg_stride + iy);
  const int32_t* sz = segs + 3 * (2 * a.seg_stride + iz);
  W117Geom g;
  g.x0 = sx[0]; g.lx = sx[1]; g.y0 = sy[0]; g.ly = sy[1]; g.z0 = sz[0]; g.lz = sz[1];
  g.h = sx[2] + (int64_t)sy[2] * a.sbx + (int64_t)sz[2] * a.sbx * a.sby;
  return g;
}

// issue the halo loads of tile g into registers (element e = lane + 64 j, row-major
// (z, y, x) over (lz+1) x (ly+2) x (lx+2) from (z0-1, y0-1, x0-1); off-grid words 0)
__device__ __forceinline__ void w117_load_halo(const KArgs& a, const uint32_t* __restrict__ fgrid, const W117Geom& g,
                                               bool valid, int lane, uint32_t (&hv)[kW117HaloRegs]) {
  const int TX = g.lx + 2, TY = g.ly + 2, n = valid ? TX * TY * (g.lz + 1) : 0;
  int q = lane / TX, r = lane - (lane / TX) * TX;  // e -> (row q, col r), stepped by 64
  const int sq = 64 / TX, sr = 64 - sq * TX;
#pragma unroll
  for (int j = 0; j < kW117HaloRegs; ++j) {
    const int e = lane + 64 * j;
    const int yy = g.y0 - 1 + q % TY, zz = g.z0 - 1 + q / TY, xx = g.x0 - 1 + r;
    const bool in = e < n && (unsigned)xx < (unsigned)a.gx && (unsigned)yy < (unsigned)a.gy &&
                    (unsigned)zz < (unsigned)a.gz;
    // clamped address + select: a "load or zero" per element would be a branch per load
    const uint32_t v = fgrid[in ? ((int64_t)zz * a.gy + yy) * a.gx + xx : 0];
    hv[j] = in ? v : 0u;
    q += sq;
    r += sr;
    if (r >= TX) {
      r -= TX;
      ++q;
    }
  }
}

// wave-local LDS hand-off: this wave's LDS ops complete, no compiler reordering across
__device__ __forceinline__ void wave_lds_fence() { __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

typedef unsigned short w117_u16x2 __attribute__((ext_vector_type(2)));

// LUT entry (sin | cos << 8) -> the channel pair sin | cos << 16
__device__ __forceinline__ uint32_t w117_pk(uint32_t l) { return (l & 0xffu) | ((l & 0xff00u) << 8); }
// binarised colour -> the channel pair beta | (1 - beta) << 16
__device__ __forceinline__ uint32_t w117_beta(bool bt) { return bt ? 1u : 0x10000u; }

__device__ __forceinline__ uint32_t udot2(uint32_t x, uint32_t y, uint32_t acc) {
  return __builtin_amdgcn_udot2(__builtin_bit_cast(w117_u16x2, x), __builtin_bit_cast(w117_u16x2, y), acc, false);
}

// block bx of gdx for frame fy; smem: w117_lds_bytes(tw_max, list_max)
__device__ __forceinline__ void c3hlac_wave117_body(const KArgs& a, int bx, int fy_, int gdx, uint32_t* smem) {
  const int64_t fy = fy_;
  const uint32_t* __restrict__ fgrid = a.grids[fy];
  float* __restrict__ ffeat = a.feat + fy * a.s_feat;
  int32_t* __restrict__ fexist = a.exist + fy * a.s_h;
  uint32_t* ftf = a.tf + fy * a.s_tf;
  const uint32_t* __restrict__ fflags = ftf + 4;
  uint32_t* fworkcnt = ftf + 2;
  const int32_t* __restrict__ fwork = a.work + fy * a.s_work;
  int32_t* frows = a.rows ? a.rows + fy * a.s_h : nullptr;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  long long* fprof = fy ? nullptr : a.prof;  // diagnostics: wave 0 of each block, first tile
  C3H_PROF(0, true);
  if (bx == 0 && tid == 0) fworkcnt[(a.epoch + 1) & 1] = 0;  // the next frame's counter
  if (bx < a.zblocks) {
    c3_zero_role(a, bx, fflags, ffeat, fexist);
    return;
  }
  uint32_t* s_lut = smem;                                        // 256
  int32_t* s_segs = reinterpret_cast<int32_t*>(smem + 256);      // 9 * kSegLds
  const int ww = w117_wave_words(a.tw_max, a.list_max);
  uint32_t* s_halo = smem + 256 + 9 * kSegLds + wave * ww;
  uint16_t* s_list = reinterpret_cast<uint16_t*>(s_halo + ((a.tw_max + 3) & ~3));
  uint32_t* s_ch = s_halo + ((a.tw_max + 3) & ~3) + (((a.list_max + 1) / 2 + 3) & ~3);
  uint16_t* s_ch16 = reinterpret_cast<uint16_t*>(s_ch);
  // work items of this frame: wave gw takes gw, gw + NW, ...; the next two are in flight
  const int NW = (gdx - a.zblocks) * kW117Waves;
  int wi = (bx - a.zblocks) * kW117Waves + wave;
  int t_cur = wi < a.ntiles ? fwork[wi] : 0;             // speculative: used only below nwork
  int t_nxt = wi + NW < a.ntiles ? fwork[wi + NW] : 0;
  const int nwork = (int)fworkcnt[a.epoch & 1];
  s_lut[tid] = a.lut[tid];
  const bool segs_lds = a.seg_stride <= kSegLds;
  const int32_t* segs = segs_lds ? s_segs : a.segs;
  if (segs_lds)
    for (int e = tid; e < 9 * a.seg_stride; e += kBlock) s_segs[e] = a.segs[e];
  lds_barrier();  // the only workgroup barrier: LUT and segment tables staged
  C3H_PROF(1, true);
  if (wave >= kW117Waves || wi >= nwork) return;
  bool first = true;
  // this lane's two bins (lane, lane + 64) and their channel rows
  int X0, Y0, X1 = 0, Y1 = 0;
  w117_bin_channels(lane, X0, Y0);
  const bool has1 = lane + 64 < 117;
  if (has1) w117_bin_channels(lane + 64, X1, Y1);
  uint32_t hv[kW117HaloRegs];
  W117Geom g = w117_geom(a, segs, t_cur);
  w117_load_halo(a, fgrid, g, true, lane, hv);
  const int thr_r = a.thr_r, thr_g = a.thr_g, thr_b = a.thr_b;
  for (; wi < nwork; wi += NW) {
    // 1. stage the halo held in registers and, from the same registers, compact the
    //    occupied centres (halo index, ascending) into the list: no LDS read-back
    const int TX = g.lx + 2, TY = g.ly + 2, TXY = TX * TY;
    const int nh = TXY * (g.lz + 1);
    int nlist = 0;
    {
      int q = lane / TX, r = lane - q * TX;  // e = lane + 64 j -> (row q = y + TY z, col r)
      int qy = q % TY, qz = q / TY;
      const int sq = 64 / TX, sr = 64 - sq * TX;
#pragma unroll
      for (int j = 0; j < kW117HaloRegs; ++j) {
        const int e = lane + 64 * j;
        if (e < nh) s_halo[e] = hv[j];
        // centre: 1 <= x <= lx, 1 <= y <= ly, z >= 1 (plane 0 is the -z halo)
        const bool occ = e < nh && hv[j] != 0u && (unsigned)(r - 1) < (unsigned)g.lx &&
                         (unsigned)(qy - 1) < (unsigned)g.ly && qz >= 1;
        const unsigned long long m = __ballot(occ);
        if (occ) s_list[nlist + __popcll(m & ((1ull << lane) - 1))] = (uint16_t)e;
        nlist += __popcll(m);
        r += sr;
        qy += sq;
        if (r >= TX) {
          r -= TX;
          ++qy;
        }
        while (qy >= TY) {
          qy -= TY;
          ++qz;
        }
      }
    }
    // 2. prefetch: the tile after next's index, the next tile's halo (in flight during 4-5)
    const W117Geom gc = g;
    const bool more = wi + NW < nwork;
    const int t_after = wi + 2 * NW < a.ntiles ? fwork[wi + 2 * NW] : 0;
    if (more) {
      g = w117_geom(a, segs, t_nxt);
      w117_load_halo(a, fgrid, g, true, lane, hv);
    }
    t_nxt = t_after;
    wave_lds_fence();
    C3H_PROF(2, first);
    C3H_PROF(3, first);
    // 4. per 64-voxel chunk: lane = voxel builds its 25 channels; lane = bin accumulates
    uint32_t acc0 = 0, acc1 = 0;
    for (int c0 = 0; c0 < nlist; c0 += 64) {
      // channel pairs packed lo | hi << 16 (every channel < 2^16, sums never carry):
      // cA = A pairs (r, r_), (g, g_), (b, b_); cB = beta pairs; cN / cQ = neighbour sums
      uint32_t one = 0, cA[3] = {0, 0, 0}, cB[3] = {0, 0, 0}, cN[3] = {0, 0, 0}, cQ[3] = {0, 0, 0};
      if (c0 + lane < nlist) {
        const int ti = s_list[c0 + lane];
        uint32_t wn[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) {  // relative_coordinates (c3_hlac.cpp:180-201), arithmetically
          const int rdx = k <= 8 ? k / 3 - 1 : (k <= 11 ? k - 10 : -1);
          const int rdy = k <= 8 ? k % 3 - 1 : (k <= 11 ? -1 : 0);
          const int rdz = k <= 8 ? -1 : 0;
          wn[k] = s_halo[ti + rdx + rdy * TX + rdz * TXY];
        }
        const uint32_t w = s_halo[ti];
        const uint32_t r = (w >> 16) & 0xffu, gg = (w >> 8) & 0xffu, b = w & 0xffu;
        one = 1;
        cA[0] = w117_pk(s_lut[r]);
        cA[1] = w117_pk(s_lut[gg]);
        cA[2] = w117_pk(s_lut[b]);
        cB[0] = w117_beta((int)r > thr_r);
        cB[1] = w117_beta((int)gg > thr_g);
        cB[2] = w117_beta((int)b > thr_b);
#pragma unroll
        for (int k = 0; k < 13; ++k) {
          const uint32_t v = wn[k];
          if (v) {
            const uint32_t nr = (v >> 16) & 0xffu, ng = (v >> 8) & 0xffu, nb = v & 0xffu;
            cN[0] += w117_pk(s_lut[nr]);
            cN[1] += w117_pk(s_lut[ng]);
            cN[2] += w117_pk(s_lut[nb]);
            cQ[0] += w117_beta((int)nr > thr_r);
            cQ[1] += w117_beta((int)ng > thr_g);
            cQ[2] += w117_beta((int)nb > thr_b);
          }
        }
      }
      constexpr int RS = 2 * kW117ChStride;  // u16 per channel row
      s_ch16[lane] = (uint16_t)one;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        s_ch16[(1 + 2 * i) * RS + lane] = (uint16_t)cA[i];
        s_ch16[(2 + 2 * i) * RS + lane] = (uint16_t)(cA[i] >> 16);
        s_ch16[(7 + 2 * i) * RS + lane] = (uint16_t)cB[i];
        s_ch16[(8 + 2 * i) * RS + lane] = (uint16_t)(cB[i] >> 16);
        s_ch16[(13 + 2 * i) * RS + lane] = (uint16_t)cN[i];
        s_ch16[(14 + 2 * i) * RS + lane] = (uint16_t)(cN[i] >> 16);
        s_ch16[(19 + 2 * i) * RS + lane] = (uint16_t)cQ[i];
        s_ch16[(20 + 2 * i) * RS + lane] = (uint16_t)(cQ[i] >> 16);
      }
      wave_lds_fence();
      C3H_PROF(4, first && c0 == 0);
      const int np = (min(nlist - c0, 64) + 1) >> 1;  // voxel pairs in this chunk
      const uint32_t* x0r = s_ch + X0 * kW117ChStride;
      const uint32_t* y0r = s_ch + Y0 * kW117ChStride;
      const uint32_t* x1r = s_ch + X1 * kW117ChStride;
      const uint32_t* y1r = s_ch + Y1 * kW117ChStride;
      for (int p = 0; p < np; p += 4) {  // 4 pairs (8 voxels) per 16-B read; the tail reads zeros
        const uint4 xa = *reinterpret_cast<const uint4*>(x0r + p);
        const uint4 ya = *reinterpret_cast<const uint4*>(y0r + p);
        const uint4 xb = *reinterpret_cast<const uint4*>(x1r + p);
        const uint4 yb = *reinterpret_cast<const uint4*>(y1r + p);
        acc0 = udot2(xa.x, ya.x, acc0);
        acc0 = udot2(xa.y, ya.y, acc0);
        acc0 = udot2(xa.z, ya.z, acc0);
        acc0 = udot2(xa.w, ya.w, acc0);
        acc1 = udot2(xb.x, yb.x, acc1);
        acc1 = udot2(xb.y, yb.y, acc1);
        acc1 = udot2(xb.z, yb.z, acc1);
        acc1 = udot2(xb.w, yb.w, acc1);
      }
      wave_lds_fence();  // the channel table is rewritten by the next chunk
    }
    C3H_PROF(5, first);
    // 5. epilogue: normalise (c3_hlac.cpp:233-250), exist gate, row list
    float* out = ffeat + gc.h * 117;
    out[lane] = (float)acc0 * norm117(lane);
    if (has1) out[lane + 64] = (float)acc1 * norm117(lane + 64);
    const uint32_t s0 = __shfl(acc0, 0, 64), s1 = __shfl(acc0, 1, 64);
    if (lane == 0) {
      fexist[gc.h] = exist_from((float)s0, (float)s1);
      if (frows) frows[wi] = (int32_t)gc.h;
    }
    C3H_PROF(6, first);
    first = false;
    if (!more) break;
  }
  C3H_PROF(7, true);
}

// everything a C3 launch needs (built on the host by build_c3_args, c3hlac.hip)
struct C3Args {
  OccArgs oa;
  KArgs ka;
  int g1, tgrid, nframes;      // occupancy / tile workgroups per frame
  size_t occ_lds, tile_lds;  // dynamic LDS bytes
  bool bits, ax, vec;        // occupancy variant
};

namespace {
__global__ __launch_bounds__(kBlock) void c3hlac_tile_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t tile_smem[];
  if (a.wave117) c3hlac_wave117_body(a, blockIdx.x, blockIdx.y, gridDim.x, tile_smem);
  else c3hlac_tile_body(a, blockIdx.x, blockIdx.y, gridDim.x, tile_smem);
}
}  // namespace

C3Args build_c3_args(const C3Launch& l);  // c3hlac.hip

}  // namespace c3h
