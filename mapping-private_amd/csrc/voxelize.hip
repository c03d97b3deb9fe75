// voxelize.hip -- LDS-privatised voxeliser for gfx950 (PCL VoxelGrid semantics).
//
// Replaces getVoxelGrid (c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:124-130 -> PCL
// VoxelGrid::filter, semantics restated in SURVEY.md App. B) and limitPoint
// (color_voxel_recognition/test/detect_object.cpp:68-87).
//
// Hot path: two launches, no hash table.
//   vox_accum   one workgroup per 4,096 consecutive points (a depth camera's pixel order
//               is spatially coherent: a voxel is hit by runs of neighbouring pixels):
//               coalesced 16-B loads; the cell's toroidal index t (VoxArgs); runs of equal
//               t in each 16-lane row merged by a DPP segmented scan; one LDS hash insert
//               per run (count | r, b | g sums, the closest point's distance to a cell face).
//               Flush, per (workgroup, voxel): two 64-bit adds into acc[t] (the first one
//               returning: the workgroup that sees count 0 is the voxel's first toucher and
//               lists it in its segment) and, only for points near a cell face, a min into
//               mg[t].  64-bit device atomics run at ~22 G/s chip-wide whatever their scope
//               or table size (tools/atomic_bench.hip, profiles/r5/), so the flush is priced
//               by their count: round 4's global hash claim (a returning CAS + two adds)
//               and round 5's owner word (a third atomic on every pair) both cost more.
//               The launch also clears the grid words the previous frame wrote (listed by
//               it) and writes bounds / counts to its own partial record.
//   vox_scatter every block reduces the partial records (bounds, totals), then converts
//               its segment's voxels -- linear index (cell - min_b) from t (modular
//               offsets, exact while the extent fits the toroidal dims), the canonical
//               colour mean kOcc | r<<16 | g<<8 | b with r = (int)(float(sum_r) * (1 /
//               float(count))) (Eigen 3.0's scalar quotient, see pcl_colour_word), the
//               centroid safety test below -- and returns acc[t] / mg[t] to zero / ~0.
//               The sums are loaded with the list entries, before the bounds reduction.
// A brick-partitioned variant with no per-voxel global atomic (one atomic per (workgroup,
// 8^3-cell brick) pair, a planning launch and a per-brick emit) was built and measured at
// 76 us per 1M-point frame against this design's 32 (profiles/r5/vox_brick/).
// Integer sums are exact and order-independent, so the grid is deterministic.
//
// Centroids.  C3-HLAC takes a voxel's subdivision (floor(c / voxel_size)) and neighbour
// base (the reference's PCL 1.0 getNeighborCentroidIndices: floor(c / leaf_size)) from its
// float centroid c = (fp32 sequential sum of its points in input order) * (1 / count), as
// PCL 1.0's VoxelGrid on Eigen 3.0 computes it (pinned by the reference's shape_data
// feature files, tests/test_shape_fixtures.py).  That can leave the voxel's own cell only when c lies within the sum's
// rounding of a cell boundary; vox_scatter flags a voxel when its closest point's margin
// is below (count + 4) * 2^-22 * (|cell| + 1) cells (4x the error bound of the mean, the
// multiply and the divide).  Only then (and for c3h_get_downsampled) the exact pass runs:
// points are bucketed per voxel (counting sort over the owning entries), each bucket sorted by
// point index and summed sequentially in fp32 -- bit-identical to the oracle -- and voxels
// whose centroid cells differ from their own cell are recorded (c3h_extract corrects
// their C3-HLAC contribution, c3hlac.hip offcell_delta_kernel).
#include <algorithm>
#include <climits>

#include <rocprim/device/device_radix_sort.hpp>

#include "c3h_internal.h"

namespace c3h {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kNoMargin = 0xffffffffu;  // above every float's bits: "no point yet"
constexpr uint32_t kNoT = 0xffffffffu;       // no toroidal index / no grid word
#ifndef C3H_VOX_CHUNK
#define C3H_VOX_CHUNK 4096
#endif
#ifndef C3H_VOX_THREADS
#define C3H_VOX_THREADS 1024  // accumulate workgroup: 16 waves (4 per SIMD) over one LDS table
#endif
constexpr int kVB = C3H_VOX_THREADS;
constexpr int kVoxChunk = C3H_VOX_CHUNK;      // points per workgroup (16 per thread; 4096 / 2048 slots measured
                                              // 40.9 us per 1M-point frame vs 41.9 at 2048 / 1024, 51 at 1024)
constexpr int kVoxPer = kVoxChunk / kVB;
#ifndef C3H_VOX_SLOTS
#define C3H_VOX_SLOTS 2048
#endif
#ifndef C3H_VOX_MERGE
#define C3H_VOX_MERGE 1  // the run merge (0: every point updates the LDS table itself)
#endif
// the owner's read and clear of a voxel's sums (one 16-B load and store; the adds are a
// previous launch's)
__device__ __forceinline__ ulonglong2 take_acc(ulonglong2* p) {
  const ulonglong2 v = *p;
  *p = make_ulonglong2(0ull, 0ull);
  return v;
}
#ifndef C3H_VOX_DIAG_NOFLUSH
#define C3H_VOX_DIAG_NOFLUSH 0
#endif
#ifndef C3H_VOX_ATOM_SCOPE
#define C3H_VOX_ATOM_SCOPE __HIP_MEMORY_SCOPE_AGENT
#endif
constexpr int kLSlots = C3H_VOX_SLOTS;        // LDS hash slots per workgroup
constexpr int kLProbe = 48;                   // LDS probes before a point goes straight to the global table
constexpr int kCellBias = 1 << 20;
// point margins (cells) at or above this are not recorded per voxel: the scatter's bound
// is below it except for very dense far voxels, which it then flags conservatively
constexpr uint32_t kMarginFlush = 0x3c800000u;  // 1/64

// PCL VoxelGrid's colour of a voxel (the reference's PCL 1.0 on Eigen 3.0): the channel
// sums divided by the point count, which Eigen 3.0 evaluates as sum * (1 / n) in float,
// truncated to int and repacked (kOcc marks the word occupied)
__device__ __forceinline__ uint32_t pcl_colour_word(unsigned long long sr, unsigned long long sg,
                                                    unsigned long long sb, uint32_t count) {
  const float rn = __fdiv_rn(1.0f, (float)count);
  const uint32_t r = (uint32_t)(int)__fmul_rn((float)sr, rn);
  const uint32_t g = (uint32_t)(int)__fmul_rn((float)sg, rn);
  const uint32_t b = (uint32_t)(int)__fmul_rn((float)sb, rn);
  return kOcc | (r << 16) | (g << 8) | b;
}

__device__ __forceinline__ bool point_valid(const float4& p, float z_limit) {
  return isfinite(p.x) && isfinite(p.y) && isfinite(p.z) && p.z < z_limit;
}

template <class T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = op(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ bool point_cell(float inv, const float4& p, int c[3], float* margin) {
  const float f[3] = {p.x * inv, p.y * inv, p.z * inv};
  float m = 1.0f;
  bool ok = true;
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {
    const float fl = floorf(f[ax]);  // PCL: static_cast<int> (floor (p * inverse_leaf_size))
    ok = ok && fl > (float)(-kCellBias) && fl < (float)(kCellBias - 1);
    c[ax] = ok ? (int)fl : 0;
    m = fminf(m, fminf(f[ax] - fl, fl + 1.0f - f[ax]));
  }
  *margin = fmaxf(m, 0.0f);
  return ok;
}

// toroidal index of an absolute cell (two's complement masks: cell mod 2^tb per axis)
__device__ __forceinline__ uint32_t tor_index(const int tb[3], const int c[3]) {
  return ((uint32_t)c[0] & ((1u << tb[0]) - 1)) | (((uint32_t)c[1] & ((1u << tb[1]) - 1)) << tb[0]) |
         (((uint32_t)c[2] & ((1u << tb[2]) - 1)) << (tb[0] + tb[1]));
}
// offsets of a toroidal index from min_b (exact while the extent fits 2^tb per axis)
__device__ __forceinline__ void tor_offsets(const int tb[3], uint32_t t, const int mn[3], uint32_t o[3]) {
  const uint32_t mx = (1u << tb[0]) - 1, my = (1u << tb[1]) - 1, mz = (1u << tb[2]) - 1;
  o[0] = ((t & mx) - (uint32_t)mn[0]) & mx;
  o[1] = (((t >> tb[0]) & my) - (uint32_t)mn[1]) & my;
  o[2] = (((t >> (tb[0] + tb[1])) & mz) - (uint32_t)mn[2]) & mz;
}

// per accum block: {min xyz, max xyz, valid points, list entries, error} at part[par][b]
constexpr int kPartW = 12;
enum { kPMin = 0, kPMax = 3, kPValid = 6, kPNew = 7, kPErr = 8 };
static_assert(kPNew == kVoxPartNew, "the extract's list stamp reads the entry counts");

__device__ __forceinline__ const int32_t* part_of(const VoxArgs& a, int par) {
  return a.part + (size_t)par * a.nblk_cap * kPartW;
}

// DPP row_shr:o (within 16-lane rows); lanes without a source read 0
template <int O>
__device__ __forceinline__ uint32_t vrow_shr(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 | O, 0xf, 0xf, true);
}

// diagnostics builds: per-block phase timestamps (C3H_PROF; thread 0 of each block)
#ifdef C3H_DIAG
#define C3H_VPROF(k) \
  if (a.prof && threadIdx.x == 0) a.prof[(size_t)blockIdx.x * 8 + (k)] = (long long)wall_clock64()
#else
#define C3H_VPROF(k)
#endif

__global__ __launch_bounds__(kVB) void vox_accum_kernel(VoxArgs a) {
  __shared__ uint32_t s_key[kLSlots];
  __shared__ unsigned long long s_A[kLSlots];  // count << 40 | sum r
  __shared__ unsigned long long s_B[kLSlots];  // sum b << 32 | sum g
  __shared__ uint32_t s_m[kLSlots];
  __shared__ uint32_t s_nnew;                  // list entries of this workgroup
  __shared__ int s_red[kVB / 64][8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, b = blockIdx.x + a.blk0;
  C3H_VPROF(0);
  if (b == 0 && tid == 0) {  // totals of an empty frame (the scatter publishes the others)
    for (int ax = 0; ax < 3; ++ax) {
      reinterpret_cast<int32_t*>(a.cnt)[kVcMin + ax] = INT_MAX;
      reinterpret_cast<int32_t*>(a.cnt)[kVcMax + ax] = INT_MIN;
    }
    a.cnt[kVcValid] = a.cnt[kVcValid + 1] = 0;
    a.cnt[kVcSlots + a.par] = 0;
    a.cnt[kVcFlag] = a.cnt[kVcErr] = a.cnt[kVcOver] = a.cnt[kVcOff] = 0;
  }
  // the previous frame's grid words (its segments b, b + grid, ...), cleared while this
  // block's point loads are in flight (this frame's scatter, a later launch, writes the grid)
  auto clear_prev = [&]() {
    if (!a.clear_grid) return;
    const int pp = a.par ^ 1;
    for (int pb = blockIdx.x; pb < a.nblk_prev; pb += gridDim.x) {  // (a launch with blk0 0)
      const int nn = part_of(a, pp)[(size_t)pb * kPartW + kPNew];
      const uint32_t* tl = a.lists + (size_t)(2 + pp) * a.lcap + (size_t)pb * kVoxChunk;
      for (int i = tid; i < nn; i += kVB) {
        const uint32_t wi = tl[i];
        if (wi != kNoT) a.grid[wi] = 0u;
      }
    }
  };
  if (b >= a.nblk) {  // clearing only (an empty frame still runs one block)
    clear_prev();
    return;
  }
  const int64_t base = b * (int64_t)kVoxChunk;
  float4 p[kVoxPer];
#pragma unroll
  for (int j = 0; j < kVoxPer; ++j) {
    const int64_t i = base + j * kVB + tid;
    if (i < a.n) {  // streamed once: non-temporal
      const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.pts) + i);
      p[j] = make_float4(v.x, v.y, v.z, v.w);
    } else {
      p[j] = make_float4(NAN, NAN, NAN, 0.0f);
    }
  }
  clear_prev();
  C3H_VPROF(1);
  for (int s = tid; s < kLSlots; s += kVB) {
    s_key[s] = kNoT;
    s_A[s] = 0;
    s_B[s] = 0;
    s_m[s] = kNoMargin;
  }
  if (tid == 0) s_nnew = 0;
  __syncthreads();
  C3H_VPROF(2);
  uint32_t* sl = a.lists + (size_t)a.par * a.lcap + (size_t)b * kVoxChunk;
  ulonglong2* __restrict__ acc = a.acc;
  uint32_t* __restrict__ mg = a.mg;
  // a (workgroup, voxel) pair that missed the LDS table: the first toucher (its returning
  // add saw count 0) lists the voxel; the margin goes to mg only when near a face
  auto add_global = [&](uint32_t t, unsigned long long va, unsigned long long vb, uint32_t m) {
    const unsigned long long old = __hip_atomic_fetch_add(&acc[t].x, va, __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE);
    if ((old >> 40) == 0) sl[atomicAdd(&s_nnew, 1u)] = t;
    __hip_atomic_fetch_add(&acc[t].y, vb, __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE);
    if (m != kNoMargin) __hip_atomic_fetch_min(mg + t, m, __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE);
  };
  int mn[3] = {INT_MAX, INT_MAX, INT_MAX}, mx[3] = {INT_MIN, INT_MIN, INT_MIN};
  int nv = 0;
  int err = 0;  // kVcErrRange
  const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);  // lanes <= this one
#pragma unroll
  for (int j = 0; j < kVoxPer; ++j) {
    int c[3] = {0, 0, 0};
    float margin = 1.0f;
    bool valid = point_valid(p[j], a.z_limit);
    if (valid && !point_cell(a.inv, p[j], c, &margin)) {
      err |= kVcErrRange;
      valid = false;
    }
    uint32_t t = kNoT, w0 = 0, w1 = 0, mb = kNoMargin;
    if (valid) {
      ++nv;
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        mn[ax] = min(mn[ax], c[ax]);
        mx[ax] = max(mx[ax], c[ax]);
      }
      t = tor_index(a.tb, c);
      const uint32_t rgb = __float_as_uint(p[j].w);
      w0 = ((rgb >> 16) & 0xffu) | (((rgb >> 8) & 0xffu) << 12) | (1u << 24);  // r | g << 12 | count << 24
      w1 = rgb & 0xffu;                                                         // b
      const uint32_t mbits = __float_as_uint(margin);
      mb = mbits < kMarginFlush ? mbits : kNoMargin;
    }
    // runs of equal keys inside each 16-lane row: a lane starts a run when it is invalid,
    // the row's first lane, or its key differs from the previous lane's; only a run's last
    // lane updates the LDS table (same-address LDS atomics serialise).  The DPP read runs
    // with every lane active: under a short-circuit mask a lane whose source lane is off
    // reads 0 and would join a run of key 0 (round 5 bug: cell 0's voxel took its
    // neighbour lane's point)
    const uint32_t tp = vrow_shr<1>(t);
    const bool head = !C3H_VOX_MERGE || !valid || (lane & 15) == 0 || tp != t;
    const uint64_t hm = __ballot(head);
    const int o0 = lane - (63 - __clzll(hm & le));  // lanes before this one in its run
    uint32_t s0, s1, sm;
    s0 = vrow_shr<1>(w0); s1 = vrow_shr<1>(w1); sm = vrow_shr<1>(mb);
    if (o0 >= 1) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<2>(w0); s1 = vrow_shr<2>(w1); sm = vrow_shr<2>(mb);
    if (o0 >= 2) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<4>(w0); s1 = vrow_shr<4>(w1); sm = vrow_shr<4>(mb);
    if (o0 >= 4) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<8>(w0); s1 = vrow_shr<8>(w1); sm = vrow_shr<8>(mb);
    if (o0 >= 8) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    const bool tail = valid && ((lane & 15) == 15 || ((hm >> (lane + 1)) & 1));
    if (!tail) continue;
    // the run's totals: count <= 16, channel sums <= 4080
    const unsigned long long A = ((unsigned long long)(w0 >> 24) << 40) | (w0 & 0xfffu);
    const unsigned long long B = ((unsigned long long)w1 << 32) | ((w0 >> 12) & 0xfffu);
    uint32_t h = (t * 0x9E3779B1u) >> (32 - __builtin_ctz(kLSlots));
    bool done = false;
    for (int probe = 0; probe < kLProbe; ++probe) {
      const uint32_t prev = atomicCAS(&s_key[h], kNoT, t);
      if (prev == kNoT || prev == t) {
        atomicAdd(&s_A[h], A);
        atomicAdd(&s_B[h], B);
        if (mb != kNoMargin) atomicMin(&s_m[h], mb);
        done = true;
        break;
      }
      h = (h + 1) & (kLSlots - 1);
    }
    if (!done) add_global(t, A, B, mb);  // LDS table full: straight to the global sums
  }
  __syncthreads();  // every point's LDS update is in
  C3H_VPROF(3);
  // flush: per (workgroup, voxel) two adds and, near a face only, the margin min (~2 global
  // atomics per pair: 64-bit device atomics run at ~22 G/s chip-wide, tools/atomic_bench.hip,
  // so their count sets the flush's cost).  The returning add detects the voxel's first
  // toucher, which lists it (one list entry per voxel); a thread's returning adds are all
  // issued before any result is used
  if (!C3H_VOX_DIAG_NOFLUSH) {
    constexpr int kFl = (kLSlots + kVB - 1) / kVB;
    uint32_t key[kFl];
    unsigned long long old[kFl];
#pragma unroll
    for (int k = 0; k < kFl; ++k) {
      const int s = tid + k * kVB;
      key[k] = s < kLSlots ? s_key[s] : kNoT;
      old[k] = key[k] != kNoT ? __hip_atomic_fetch_add(&acc[key[k]].x, s_A[s], __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE)
                              : 1ull << 40;
    }
#pragma unroll
    for (int k = 0; k < kFl; ++k) {
      const int s = tid + k * kVB;
      if (key[k] == kNoT) continue;
      __hip_atomic_fetch_add(&acc[key[k]].y, s_B[s], __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE);
      if (s_m[s] != kNoMargin) __hip_atomic_fetch_min(mg + key[k], s_m[s], __ATOMIC_RELAXED, C3H_VOX_ATOM_SCOPE);
      if ((old[k] >> 40) == 0) sl[atomicAdd(&s_nnew, 1u)] = key[k];
    }
  }
  // bounds, counts and the entry count go to this block's partial record: no same-address
  // atomics across blocks (they serialise at the memory side)
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {
    mn[ax] = wave_reduce(mn[ax], [](int x, int y) { return min(x, y); });
    mx[ax] = wave_reduce(mx[ax], [](int x, int y) { return max(x, y); });
  }
  nv = wave_reduce(nv, [](int x, int y) { return x + y; });
  const int e = wave_reduce(err, [](int x, int y) { return x | y; });
  if (lane == 0) {
    for (int ax = 0; ax < 3; ++ax) {
      s_red[w][ax] = mn[ax];
      s_red[w][3 + ax] = mx[ax];
    }
    s_red[w][6] = nv;
    s_red[w][7] = e;
  }
  __syncthreads();
  C3H_VPROF(4);
  int32_t* pr = a.part + ((size_t)a.par * a.nblk_cap + b) * kPartW;
  if (tid < 8) {
    int v = s_red[0][tid];
    for (int i = 1; i < kVB / 64; ++i) {
      const int u = s_red[i][tid];
      v = tid < 3 ? min(v, u) : (tid < 6 ? max(v, u) : (tid == 6 ? v + u : (v | u)));
    }
    pr[tid < 7 ? tid : kPErr] = v;
  }
  if (tid == 8) pr[kPNew] = (int)s_nnew;
  C3H_VPROF(5);
}

// every block reduces the accum blocks' partial records (a few KB, from L2); block 0
// publishes the totals for the host and the later kernels
struct VoxTotals {
  int mn[3], dv[3];
  int64_t nvox;
  bool any;
};

__device__ VoxTotals vox_reduce(const VoxArgs& a, bool publish) {
  __shared__ int s_r[kBlock / 64][10];
  const int32_t* pt = part_of(a, a.par);
  int mn[3] = {INT_MAX, INT_MAX, INT_MAX}, mx[3] = {INT_MIN, INT_MIN, INT_MIN};
  int nv = 0, er = 0;
  for (int b = threadIdx.x; b < a.nblk; b += kBlock) {
    const int32_t* r = pt + (size_t)b * kPartW;
    if (r[kPValid]) {
      for (int ax = 0; ax < 3; ++ax) {
        mn[ax] = min(mn[ax], r[kPMin + ax]);
        mx[ax] = max(mx[ax], r[kPMax + ax]);
      }
    }
    nv += r[kPValid];
    er |= r[kPErr];
  }
  for (int ax = 0; ax < 3; ++ax) {
    mn[ax] = wave_reduce(mn[ax], [](int x, int y) { return min(x, y); });
    mx[ax] = wave_reduce(mx[ax], [](int x, int y) { return max(x, y); });
  }
  nv = wave_reduce(nv, [](int x, int y) { return x + y; });
  er = wave_reduce(er, [](int x, int y) { return x | y; });
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int ax = 0; ax < 3; ++ax) {
      s_r[w][ax] = mn[ax];
      s_r[w][3 + ax] = mx[ax];
    }
    s_r[w][6] = nv;
    s_r[w][8] = er;
  }
  __syncthreads();
  VoxTotals t;
  int64_t nvox = 1;
  for (int ax = 0; ax < 3; ++ax) {
    int lo = s_r[0][ax], hi = s_r[0][3 + ax];
    for (int i = 1; i < kBlock / 64; ++i) {
      lo = min(lo, s_r[i][ax]);
      hi = max(hi, s_r[i][3 + ax]);
    }
    t.mn[ax] = lo;
    t.dv[ax] = hi - lo + 1;
    nvox *= t.dv[ax];
  }
  int tv = 0, te = 0;
  for (int i = 0; i < kBlock / 64; ++i) {
    tv += s_r[i][6];
    te |= s_r[i][8];
  }
  t.any = tv > 0;
  t.nvox = t.any ? nvox : 0;
  if (publish && threadIdx.x == 0) {
    int32_t* ci = reinterpret_cast<int32_t*>(a.cnt);
    for (int ax = 0; ax < 3; ++ax) {
      ci[kVcMin + ax] = t.mn[ax];
      ci[kVcMax + ax] = t.mn[ax] + t.dv[ax] - 1;
    }
    a.cnt[kVcValid] = (uint32_t)tv;
    a.cnt[kVcValid + 1] = 0;
    if (te) a.cnt[kVcErr] = (uint32_t)te;
  }
  return t;
}

__device__ __forceinline__ int seg_count(const VoxArgs& a, int b) {
  return part_of(a, a.par)[(size_t)b * kPartW + kPNew];
}

// one block per accum block: its segment's entries.  The first round of entries and their
// owner words are loaded before the totals are reduced (neither depends on the other)
__global__ __launch_bounds__(kBlock) void vox_scatter_kernel(VoxArgs a) {
  const int b = blockIdx.x;
  const int nn = seg_count(a, b);
  const size_t seg = (size_t)b * kVoxChunk;
  const uint32_t* sl = a.lists + (size_t)a.par * a.lcap + seg;
  uint32_t* tl = a.lists + (size_t)(2 + a.par) * a.lcap + seg;
  uint32_t* lc = a.lcnt + seg;
  const uint32_t q0 = (uint32_t)seg;
  constexpr int kPre = 2;  // entries per thread loaded ahead
  uint32_t pt[kPre];
  ulonglong2 pacc[kPre];  // the sums (the accumulate launch's adds are all in)
#pragma unroll
  for (int k = 0; k < kPre; ++k) {
    const int i = threadIdx.x + k * kBlock;
    pt[k] = i < nn ? sl[i] : 0u;
    pacc[k] = i < nn ? a.acc[pt[k]] : make_ulonglong2(0ull, 0ull);
  }
  const VoxTotals tot = vox_reduce(a, blockIdx.x == 0);
  if (!tot.any) return;
  // the extent beyond the toroidal dims (the host enlarges them and runs the frame again),
  // or beyond the grid buffer (the host grows it and runs this again): nothing is written
  bool wrap = false;
  for (int ax = 0; ax < 3; ++ax) wrap = wrap || tot.dv[ax] > (1 << a.tb[ax]);
  if (wrap) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.cnt + kVcErr, kVcErrWrap);
    return;
  }
  if (tot.nvox > a.grid_cap || tot.nvox > INT_MAX) {
    if (blockIdx.x == 0 && threadIdx.x == 0) a.cnt[kVcOver] = 1;
    return;
  }
  uint32_t flagged = 0, owned = 0, bad = 0;
  auto visit = [&](int i, uint32_t t, ulonglong2 v) {  // every listed voxel is listed once
    const uint32_t q = q0 + (uint32_t)i;
    a.acc[t] = make_ulonglong2(0ull, 0ull);
    const uint32_t m = a.mg[t];
    if (m != kNoMargin) a.mg[t] = kNoMargin;  // only the near-face voxels changed it
    uint32_t o[3];
    tor_offsets(a.tb, t, tot.mn, o);
    // bound check: a listed key is a cell of this frame's points, so its offsets lie inside
    // the frame's extent -- unless the accumulators held sums no point of this frame added
    // (kVcErrBad: nothing written, the call fails)
    if (o[0] >= (uint32_t)tot.dv[0] || o[1] >= (uint32_t)tot.dv[1] || o[2] >= (uint32_t)tot.dv[2] ||
        (v.x >> 40) == 0) {
      tl[i] = kNoT;
      lc[i] = 0u;
      ++bad;
      return;
    }
    ++owned;
    a.tpos[t] = q;
    const int64_t idx = o[0] + (int64_t)tot.dv[0] * (o[1] + (int64_t)tot.dv[1] * o[2]);
    const uint32_t count = (uint32_t)(v.x >> 40);
    a.grid[idx] = pcl_colour_word(v.x & 0xffffffffffull, v.y & 0xffffffffull, v.y >> 32, count);
    tl[i] = (uint32_t)idx;
    lc[i] = count;
    // margins >= kMarginFlush were not recorded: conservative when the bound exceeds it
    const int cmag = max(max(abs(tot.mn[0] + (int)o[0]), abs(tot.mn[1] + (int)o[1])), abs(tot.mn[2] + (int)o[2])) + 1;
    const float eps = (float)(count + 4) * (float)cmag * 0x1p-22f;
    if (__uint_as_float(m) < eps || eps >= __uint_as_float(kMarginFlush)) ++flagged;
  };
#pragma unroll
  for (int k = 0; k < kPre; ++k) {
    const int i = threadIdx.x + k * kBlock;
    if (i < nn) visit(i, pt[k], pacc[k]);
  }
  for (int i = threadIdx.x + kPre * kBlock; i < nn; i += kBlock) {
    const uint32_t t = sl[i];
    visit(i, t, a.acc[t]);
  }
  // one count add per block (same-address adds serialise at the memory side)
  __shared__ uint32_t s_cnt[2][kBlock / 64];
  flagged = wave_reduce(flagged, [](uint32_t u, uint32_t v) { return u + v; });
  owned = wave_reduce(owned, [](uint32_t u, uint32_t v) { return u + v; });
  bad = wave_reduce(bad, [](uint32_t u, uint32_t v) { return u | v; });
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_cnt[0][w] = flagged;
    s_cnt[1][w] = owned;
    if (bad) atomicOr(a.cnt + kVcErr, kVcErrBad);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint32_t v = 0;
    for (int i = 0; i < kBlock / 64; ++i) v += s_cnt[threadIdx.x][i];
    if (v) atomicAdd(a.cnt + (threadIdx.x == 0 ? kVcFlag : kVcSlots + a.par), v);
  }
}

__device__ __forceinline__ bool vox_bounds(const VoxArgs& a, int mn[3], int dv[3], int64_t* nvox) {
  const int32_t* ci = reinterpret_cast<const int32_t*>(a.cnt);
  int64_t n = 1;
  for (int ax = 0; ax < 3; ++ax) {
    mn[ax] = ci[kVcMin + ax];
    dv[ax] = ci[kVcMax + ax] - mn[ax] + 1;
    n *= dv[ax];
  }
  *nvox = n;
  return ci[kVcMax] >= ci[kVcMin];
}

// ---- exact centroids (flagged frames and c3h_get_downsampled) ----------------------
// positions p = b * kVoxChunk + i of the segmented entry list; entries that do not own
// their voxel and gaps (i >= the segment's count) hold count 0
__global__ __launch_bounds__(kBlock) void vox_counts_kernel(VoxArgs a, uint32_t* __restrict__ counts) {
  const int64_t np = (int64_t)a.nblk * kVoxChunk;
  for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < np; q += (int64_t)gridDim.x * kBlock) {
    const int b = (int)(q / kVoxChunk), i = (int)(q % kVoxChunk);
    counts[q] = i < seg_count(a, b) ? a.lcnt[q] : 0u;
  }
}

// Bound checks (round 6): the bucket of a voxel has exactly its accumulated count of slots.
// A point whose voxel's owning entry is not this frame's (tpos stale: the voxel was never
// listed) or whose bucket is already full (the count holds a point it does not own) is not
// filed, and the centroid pass skips a bucket with an unfilled slot -- the round-5 fault: a
// run-merge bug moved one point's count to cell 0's voxel, which left one slot of its bucket
// unwritten, and on a fresh context that slot's uninitialised index was read as a point.
__global__ __launch_bounds__(kBlock) void vox_bucket_kernel(VoxArgs a, const uint32_t* __restrict__ off,
                                                            const uint32_t* __restrict__ counts,
                                                            uint32_t* __restrict__ cur,
                                                            uint32_t* __restrict__ bucket) {
  const uint64_t np = (uint64_t)a.nblk * kVoxChunk;
  const uint32_t* sl = a.lists + (size_t)a.par * a.lcap;
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kBlock) {
    const float4 p = a.pts[i];
    if (!point_valid(p, a.z_limit)) continue;
    int c[3];
    float m;
    if (!point_cell(a.inv, p, c, &m)) continue;
    const uint32_t t = tor_index(a.tb, c);
    const uint32_t lp = a.tpos[t];
    // counts[lp] is 0 beyond the entry's segment count and for entries that own nothing
    if (lp >= np || sl[lp] != t || counts[lp] == 0) {
      bad = true;
      continue;
    }
    const uint32_t slot = atomicAdd(&cur[lp], 1u);
    if (slot >= counts[lp]) {
      bad = true;
      continue;
    }
    bucket[off[lp] + slot] = (uint32_t)i;
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(a.cnt + kVcErr, kVcErrBad);
}

// per voxel: its points in input order (shell sort of the bucket), the fp32 sequential
// sum and the IEEE mean (the oracle's orc_voxel_fill); off-cell voxels are recorded as
// {linear index, neighbour-base cell xyz, subdivision cell xyz} relative to min_b
__global__ __launch_bounds__(kBlock) void vox_centroid_kernel(VoxArgs a, const uint32_t* __restrict__ off,
                                                              const uint32_t* __restrict__ counts,
                                                              const uint32_t* __restrict__ cur,
                                                              uint32_t* __restrict__ bucket,
                                                              float4* __restrict__ cent,
                                                              int32_t* __restrict__ offcell) {
  int mn[3], dv[3];
  int64_t nvox;
  vox_bounds(a, mn, dv, &nvox);
  const int64_t np = (int64_t)a.nblk * kVoxChunk;
  const uint32_t* sl = a.lists + (size_t)a.par * a.lcap;
  const uint32_t* tl = a.lists + (size_t)(2 + a.par) * a.lcap;
  for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < np; q += (int64_t)gridDim.x * kBlock) {
    const int m = (int)counts[q];
    if (m == 0) continue;
    if (cur[q] != (uint32_t)m) {  // a slot not filed by this frame's points (vox_bucket_kernel)
      atomicOr(a.cnt + kVcErr, kVcErrBad);
      cent[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      continue;
    }
    uint32_t* bk = bucket + off[q];
    const int gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
    for (int gi = 0; gi < 8; ++gi) {
      const int gap = gaps[gi];
      for (int u = gap; u < m; ++u) {
        const uint32_t t = bk[u];
        int v = u;
        for (; v >= gap && bk[v - gap] > t; v -= gap) bk[v] = bk[v - gap];
        bk[v] = t;
      }
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    for (int u = 0; u < m; ++u) {
      const float4 p = a.pts[bk[u]];
      sx += p.x;
      sy += p.y;
      sz += p.z;
    }
    const float rn = __fdiv_rn(1.0f, (float)m);  // Eigen 3.0: centroid / n == centroid * (1 / n)
    const float c[3] = {__fmul_rn(sx, rn), __fmul_rn(sy, rn), __fmul_rn(sz, rn)};
    const uint32_t idx = tl[q];
    cent[q] = make_float4(c[0], c[1], c[2], __uint_as_float(a.grid[idx] & 0x00ffffffu));
    uint32_t o[3];
    tor_offsets(a.tb, sl[q], mn, o);
    int nb[3], sb[3];
    bool moved = false;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      const int own = mn[ax] + (int)o[ax];
      nb[ax] = (int)floorf(__fdiv_rn(c[ax], a.leaf));  // PCL 1.0 getNeighborCentroidIndices: floor(p / leaf)
      sb[ax] = nb[ax];                                  // c3_hlac.cpp:349-354: floor(p / voxel_size)
      moved = moved || nb[ax] != own || sb[ax] != own;
    }
    if (moved) {
      const uint32_t k = atomicAdd(a.cnt + kVcOff, 1u);
      int32_t* oc = offcell + 8 * (int64_t)k;
      oc[0] = (int32_t)idx;
      for (int ax = 0; ax < 3; ++ax) {
        oc[1 + ax] = nb[ax] - mn[ax];
        oc[4 + ax] = sb[ax] - mn[ax];
      }
      oc[7] = 0;
    }
  }
}

__global__ __launch_bounds__(kBlock) void vox_downsampled_kernel(VoxArgs a, const float4* __restrict__ cent,
                                                                 const uint32_t* __restrict__ counts,
                                                                 const int32_t* __restrict__ leaf,
                                                                 float4* __restrict__ out) {
  const int64_t np = (int64_t)a.nblk * kVoxChunk;
  const uint32_t* tl = a.lists + (size_t)(2 + a.par) * a.lcap;
  for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < np; q += (int64_t)gridDim.x * kBlock)
    if (counts[q]) out[leaf[tl[q]]] = cent[q];
}

// returns the accumulators a frame's accumulate pass touched to zero (a frame the scatter
// did not convert: its extent wrapped the toroidal dims and it went to the sorted path).
// Every non-zero record was first touched by one (block, voxel) pair, which listed it.
__global__ __launch_bounds__(kBlock) void vox_clear_kernel(VoxArgs a) {
  const int b = blockIdx.x;
  const int nn = seg_count(a, b);
  const uint32_t* sl = a.lists + (size_t)a.par * a.lcap + (size_t)b * kVoxChunk;
  for (int i = threadIdx.x; i < nn; i += kBlock) {
    const uint32_t t = sl[i];
    a.acc[t] = make_ulonglong2(0ull, 0ull);
    a.mg[t] = kNoMargin;
  }
}

// ---- wide frames: the sorted path ---------------------------------------------------
// A frame whose extent needs more than 2^kVoxTorMaxBits toroidal cells (24 B each) is
// voxelised by sorting instead: its valid points' linear voxel indices (cell - min_b, known
// from the first pass; < 2^31 by the host's check) as 32-bit keys, invalid points keyed
// nvox (after every voxel), a stable radix sort of (key, point index) pairs, and one thread
// per run of equal keys.  The stable sort keeps a voxel's points in input order, so the
// thread sums them exactly as the oracle does (fp32 sequential xyz, integer colour), and
// writes the grid word, the list entries, the exact centroid and the off-cell record: the
// state vox_scatter + the exact pass leave.  Memory O(points) whatever the extent.
__global__ __launch_bounds__(kBlock) void voxs_keys_kernel(VoxArgs a, int3 mn, int3 dv, uint32_t sentinel,
                                                           uint32_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * kBlock) {
    const float4 p = a.pts[i];
    int c[3];
    float m;
    uint32_t k = sentinel;
    if (point_valid(p, a.z_limit) && point_cell(a.inv, p, c, &m)) {
      const uint32_t o0 = (uint32_t)(c[0] - mn.x), o1 = (uint32_t)(c[1] - mn.y), o2 = (uint32_t)(c[2] - mn.z);
      if (o0 < (uint32_t)dv.x && o1 < (uint32_t)dv.y && o2 < (uint32_t)dv.z)  // bounds of the same points
        k = o0 + (uint32_t)dv.x * (o1 + (uint32_t)dv.y * o2);
    }
    keys[i] = k;
    idx[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(kBlock) void voxs_heads_kernel(const uint32_t* __restrict__ keys, int64_t nv,
                                                            uint32_t* __restrict__ head) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock)
    head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void voxs_emit_kernel(VoxArgs a, int3 mn, int3 dv, const uint32_t* __restrict__ keys,
                                                           const uint32_t* __restrict__ idx,
                                                           const uint32_t* __restrict__ head,
                                                           const int32_t* __restrict__ ord, int64_t nv,
                                                           uint32_t* __restrict__ counts, float4* __restrict__ cent,
                                                           int32_t* __restrict__ offcell) {
  uint32_t* sl = a.lists + (size_t)a.par * a.lcap;
  uint32_t* tl = a.lists + (size_t)(2 + a.par) * a.lcap;
  uint32_t nocc = 0;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock) {
    if (!head[i]) continue;
    const uint32_t key = keys[i];
    const uint32_t q = (uint32_t)ord[i];
    unsigned long long sr = 0, sg = 0, sb = 0;
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    uint32_t cnt = 0;
    for (int64_t j = i; j < nv && keys[j] == key; ++j, ++cnt) {
      const float4 p = a.pts[idx[j]];
      sx += p.x;
      sy += p.y;
      sz += p.z;
      const uint32_t rgb = __float_as_uint(p.w);
      sr += (rgb >> 16) & 0xffu;
      sg += (rgb >> 8) & 0xffu;
      sb += rgb & 0xffu;
    }
    const uint32_t word = pcl_colour_word(sr, sg, sb, cnt);
    a.grid[key] = word;
    sl[q] = key;
    tl[q] = key;
    a.lcnt[q] = cnt;
    counts[q] = cnt;
    ++nocc;
    const float rn = __fdiv_rn(1.0f, (float)cnt);  // Eigen 3.0: centroid / n == centroid * (1 / n)
    const float c[3] = {__fmul_rn(sx, rn), __fmul_rn(sy, rn), __fmul_rn(sz, rn)};
    cent[q] = make_float4(c[0], c[1], c[2], __uint_as_float(word & 0x00ffffffu));
    const int own[3] = {mn.x + (int)(key % (uint32_t)dv.x), mn.y + (int)(key / (uint32_t)dv.x % (uint32_t)dv.y),
                        mn.z + (int)(key / (uint32_t)dv.x / (uint32_t)dv.y)};
    const int mnv[3] = {mn.x, mn.y, mn.z};
    int nb[3];
    bool moved = false;
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
      nb[ax] = (int)floorf(__fdiv_rn(c[ax], a.leaf));  // as vox_centroid_kernel
      moved = moved || nb[ax] != own[ax];
    }
    if (moved) {
      const uint32_t k = atomicAdd(a.cnt + kVcOff, 1u);
      int32_t* oc = offcell + 8 * (int64_t)k;
      oc[0] = (int32_t)key;
      for (int ax = 0; ax < 3; ++ax) {
        oc[1 + ax] = nb[ax] - mnv[ax];
        oc[4 + ax] = nb[ax] - mnv[ax];
      }
      oc[7] = 0;
    }
  }
  nocc = wave_reduce(nocc, [](uint32_t u, uint32_t v) { return u + v; });
  if ((threadIdx.x & 63) == 0 && nocc) atomicAdd(a.cnt + kVcSlots + a.par, nocc);
}

// the segment counts of the positions 0 .. nocc - 1 (list segments of kVoxChunk), for the
// readers that walk the lists by segment (the next frame's grid clear, the counts pass)
__global__ __launch_bounds__(kBlock) void voxs_parts_kernel(VoxArgs a) {
  const int64_t nocc = a.cnt[kVcSlots + a.par];
  int32_t* pr = a.part + (size_t)a.par * a.nblk_cap * kPartW;
  for (int b = blockIdx.x * kBlock + threadIdx.x; b < a.nblk; b += gridDim.x * kBlock) {
    const int64_t r = nocc - (int64_t)b * kVoxChunk;
    pr[(size_t)b * kPartW + kPNew] = (int32_t)(r < 0 ? 0 : (r > kVoxChunk ? kVoxChunk : r));
  }
}

// ---- exclusive scans (leaf layout, bucket offsets) --------------------------------
constexpr int kScanItems = 4;  // items per thread
constexpr int kScanBlock = kBlock * kScanItems;

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
  for (int w = 0; w < kBlock / 64; ++w) {
    if (w < wid) wbase += lds[w];
    tot += lds[w];
  }
  *total = tot;
  __syncthreads();
  return wbase + x - v;
}

// item value: grid word occupancy (leaf layout) or a count array
template <bool kOccupancy>
__device__ __forceinline__ uint32_t scan_item(const uint32_t* src, int64_t i, int64_t n) {
  if (i >= n) return 0;
  return kOccupancy ? (src[i] ? 1u : 0u) : src[i];
}

template <bool kOccupancy>
__global__ __launch_bounds__(kBlock) void scan_count_kernel(const uint32_t* __restrict__ src, int64_t n,
                                                            uint32_t* __restrict__ sums) {
  __shared__ uint32_t lds[kBlock / 64];
  const int64_t base = blockIdx.x * (int64_t)kScanBlock + threadIdx.x * kScanItems;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) c += scan_item<kOccupancy>(src, base + j, n);
  uint32_t tot;
  block_exclusive_scan(c, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_sums_kernel(uint32_t* __restrict__ sums, int64_t nblocks) {
  __shared__ uint32_t lds[kBlock / 64];
  uint32_t carry = 0;
  for (int64_t b0 = 0; b0 < nblocks; b0 += kBlock) {
    const int64_t i = b0 + threadIdx.x;
    const uint32_t v = i < nblocks ? sums[i] : 0;
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan(v, lds, &tot);
    if (i < nblocks) sums[i] = carry + ex;
    carry += tot;
  }
}

// kOccupancy: leaf layout (rank or -1 per voxel); else exclusive offsets of the counts
template <bool kOccupancy>
__global__ __launch_bounds__(kBlock) void scan_write_kernel(const uint32_t* __restrict__ src, int64_t n,
                                                            const uint32_t* __restrict__ sums,
                                                            int32_t* __restrict__ out) {
  __shared__ uint32_t lds[kBlock / 64];
  const int64_t base = blockIdx.x * (int64_t)kScanBlock + threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = scan_item<kOccupancy>(src, base + j, n);
    c += v[j];
  }
  uint32_t tot;
  uint32_t rank = sums[blockIdx.x] + block_exclusive_scan(c, lds, &tot);
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j >= n) break;
    out[base + j] = kOccupancy ? (v[j] ? (int32_t)rank : -1) : (int32_t)rank;
    rank += v[j];
  }
}

int grid_for(int64_t n, int cap = 4096) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// ---- batched voxeliser (c3h_run_point_frames) ----------------------------------------
// Two launches per batch of frames, no host round trip:
//   voxb_accum   block b = (frame f, chunk of kBChunk consecutive points): first it clears
//                the canvas words the previous batch on this buffer set wrote through its
//                own segment b (read before this block rewrites the segment's record).
//                Points (limitPoint + VoxelGrid quantisation, as vox_accum) are keyed by
//                the cell's toroidal index (x, y, z mod powers of two >= the canvas).  A
//                depth camera's consecutive pixels hit the same voxel in runs: within each
//                16-lane row of a wave the runs are summed by a segmented DPP scan and only
//                a run's last lane inserts into the LDS hash (one CAS + two adds for ~5
//                points).  The flush adds each (block, voxel) total into the frame's
//                toroidal accumulator (one 16-B record) with one returning atomic (count 0
//                before = first touch: the entry goes to the block's segment of the voxel
//                list) and one plain one.
//   voxb_reduce  one block per frame: its blocks' partial records -> its VoxelGrid
//                geometry, getSubdivNum and the gate's position limits.
//   voxb_scatter block b turns its segment's entries into canvas words -- canvas index =
//                cell - min_b, with cell - min_b = (t - min_b) mod 2^tb per axis, exact
//                whenever the frame's extent fits the canvas -- clears the accumulator
//                records and lists the words for the next batch's clear.
#ifndef C3H_VB_CHUNK
#define C3H_VB_CHUNK 16384  // a depth camera's rows: 16k pixels per block, each voxel flushed by 1.16 blocks
                            // at 256^3 (4k: 1.71), 1.40 at 128^3 (4k: 2.67)
#endif
#ifndef C3H_VB_THREADS
#define C3H_VB_THREADS 512  // 8 waves over a 2,048-slot table (1,024 threads: 8.0 vs 6.5 us per 128^3 frame)
#endif
#ifndef C3H_VB_SLOTS
#define C3H_VB_SLOTS 2048
#endif
constexpr int kBChunk = C3H_VB_CHUNK;
constexpr int kBT = C3H_VB_THREADS;
constexpr int kBPer = kBChunk / kBT;
#ifndef C3H_VB_ROUND
#define C3H_VB_ROUND 8
#endif
constexpr int kBRound = kBPer < C3H_VB_ROUND ? kBPer : C3H_VB_ROUND;  // loads in flight per thread
static_assert(kBPer % kBRound == 0, "rounds");
constexpr int kBSlots = C3H_VB_SLOTS;
static_assert(kBChunk % kBT == 0 && (kBSlots & (kBSlots - 1)) == 0, "batch voxeliser shape");
#ifndef C3H_VB_DIAG
#define C3H_VB_DIAG 0  // diagnostics builds only: 1 = no global flush, 2 = no LDS insert either
#endif
#ifndef C3H_VB_ATOM_SCOPE
#define C3H_VB_ATOM_SCOPE __HIP_MEMORY_SCOPE_AGENT  // diagnostics: workgroup scope times L2-local atomics
#endif
#ifndef C3H_VB_MERGE
#define C3H_VB_MERGE 1  // the run merge (0: every point inserts into the LDS hash itself)
#endif

__device__ __forceinline__ int vb_frame(const int* blk0, int nf, int b) {
  int lo = 0, hi = nf;  // blk0[lo] <= b < blk0[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (blk0[mid] <= b) lo = mid;
    else hi = mid;
  }
  return lo;
}


__global__ __launch_bounds__(kBT) void voxb_accum_kernel(VoxBatchArgs a) {
  __shared__ uint32_t s_key[kBSlots];
  __shared__ unsigned long long s_A[kBSlots];  // count << 40 | sum r
  __shared__ unsigned long long s_B[kBSlots];  // sum b << 32 | sum g
  __shared__ uint32_t s_m[kBSlots];
  __shared__ uint32_t s_nnew;
  __shared__ int s_red[kBT / 64][8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  int32_t* pr = a.part + (size_t)b * kPartW;
  if (b < a.prev_total) {  // the previous batch's canvas words of segment b
    const int fp = vb_frame(a.prev_blk0, a.prev_nf, b);
    const int nn = pr[kPNew];
    uint32_t* g = a.grid[fp];
    const uint32_t* wl = a.wlist + (size_t)b * kBChunk;
    for (int i = tid; i < nn; i += kBT) g[wl[i]] = 0u;
  }
  if (b >= a.total) return;  // clearing only
  const int f = vb_frame(a.blk0, a.nf, b);
  const int64_t base = (int64_t)(b - a.blk0[f]) * kBChunk;
  const float4* __restrict__ pts = a.pts[f];
  const int64_t n = a.n[f];
  const uint32_t mx_ = (1u << a.tb[0]) - 1, my_ = (1u << a.tb[1]) - 1, mz_ = (1u << a.tb[2]) - 1;
  const int sy = a.tb[0], sz = a.tb[0] + a.tb[1];
  ulonglong2* __restrict__ acc = a.acc + f * a.s_acc;
  uint32_t* __restrict__ Mg = a.accM + f * a.s_acc;
  uint32_t* __restrict__ vl = a.vlist + (size_t)b * kBChunk;
  for (int s = tid; s < kBSlots; s += kBT) {
    s_key[s] = kNoT;
    s_A[s] = 0;
    s_B[s] = 0;
    s_m[s] = kNoMargin;
  }
  if (tid == 0) s_nnew = 0;
  __syncthreads();
  int mn[3] = {INT_MAX, INT_MAX, INT_MAX}, mx[3] = {INT_MIN, INT_MIN, INT_MIN};
  int nv = 0;
  bool err = false;
  // a (block, voxel) pair that misses the LDS table: the first toucher (the returning add
  // saw count 0) lists the voxel; its margin goes to Mg only when near a face
  auto add_global = [&](uint32_t t, unsigned long long va, unsigned long long vb, uint32_t m) {
    const unsigned long long old = __hip_atomic_fetch_add(&acc[t].x, va, __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE);
    if ((old >> 40) == 0) vl[atomicAdd(&s_nnew, 1u)] = t;
    __hip_atomic_fetch_add(&acc[t].y, vb, __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE);
    if (m < kMarginFlush) __hip_atomic_fetch_min(Mg + t, m, __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE);
  };
  const uint64_t le = (lane == 63) ? ~0ull : ((2ull << lane) - 1);  // lanes <= this one
  for (int r0 = 0; r0 < kBPer; r0 += kBRound) {
  float4 p[kBRound];
#pragma unroll
  for (int j = 0; j < kBRound; ++j) {  // a round of loads in flight together
    const int64_t i = base + (int64_t)(r0 + j) * kBT + tid;
    if (i < n) {
      const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(pts) + i);
      p[j] = make_float4(v.x, v.y, v.z, v.w);
    } else {
      p[j] = make_float4(NAN, NAN, NAN, 0.0f);
    }
  }
#pragma unroll
  for (int j = 0; j < kBRound; ++j) {
    int c[3];
    float margin;
    bool valid = point_valid(p[j], a.z_limit);
    if (valid && !point_cell(a.inv, p[j], c, &margin)) {
      err = true;
      valid = false;
    }
    uint32_t t = kNoT, w0 = 0, w1 = 0, mb = kNoMargin;
    if (valid) {
      ++nv;
#pragma unroll
      for (int ax = 0; ax < 3; ++ax) {
        mn[ax] = min(mn[ax], c[ax]);
        mx[ax] = max(mx[ax], c[ax]);
      }
      t = ((uint32_t)c[0] & mx_) | (((uint32_t)c[1] & my_) << sy) | (((uint32_t)c[2] & mz_) << sz);
      const uint32_t rgb = __float_as_uint(p[j].w);
      w0 = ((rgb >> 16) & 0xffu) | (((rgb >> 8) & 0xffu) << 12) | (1u << 24);  // r | g << 12 | count << 24
      w1 = rgb & 0xffu;                                                         // b
      const uint32_t mbits = __float_as_uint(margin);
      mb = mbits < kMarginFlush ? mbits : kNoMargin;
    }
    // runs of equal keys inside each 16-lane row: a lane starts a run when it is invalid,
    // the row's first lane, or its key differs from the previous lane's
    const uint32_t tp = vrow_shr<1>(t);
    const bool head = !C3H_VB_MERGE || !valid || (lane & 15) == 0 || tp != t;
    const uint64_t hm = __ballot(head);
    const int hpos = 63 - __clzll(hm & le);  // this lane's run start
    const int o0 = lane - hpos;              // lanes before this one in its run
    uint32_t s0, s1, sm;
    s0 = vrow_shr<1>(w0); s1 = vrow_shr<1>(w1); sm = vrow_shr<1>(mb);
    if (o0 >= 1) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<2>(w0); s1 = vrow_shr<2>(w1); sm = vrow_shr<2>(mb);
    if (o0 >= 2) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<4>(w0); s1 = vrow_shr<4>(w1); sm = vrow_shr<4>(mb);
    if (o0 >= 4) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    s0 = vrow_shr<8>(w0); s1 = vrow_shr<8>(w1); sm = vrow_shr<8>(mb);
    if (o0 >= 8) { w0 += s0; w1 += s1; mb = min(mb, sm); }
    const bool tail = C3H_VB_DIAG < 2 && valid && ((lane & 15) == 15 || ((hm >> (lane + 1)) & 1));
    if (tail) {  // the run's totals: count <= 16, channel sums <= 4080
      const unsigned long long A = ((unsigned long long)(w0 >> 24) << 40) | (w0 & 0xfffu);
      const unsigned long long Bv = ((unsigned long long)w1 << 32) | ((w0 >> 12) & 0xfffu);
      uint32_t h = (t * 0x9E3779B1u) >> (32 - __builtin_ctz(kBSlots));
      bool done = false;
      for (int probe = 0; probe < kLProbe; ++probe) {
        const uint32_t prev = atomicCAS(&s_key[h], kNoT, t);
        if (prev == kNoT || prev == t) {
          atomicAdd(&s_A[h], A);
          atomicAdd(&s_B[h], Bv);
          if (mb != kNoMargin) atomicMin(&s_m[h], mb);
          done = true;
          break;
        }
        h = (h + 1) & (kBSlots - 1);
      }
      if (!done) add_global(t, A, Bv, mb);  // LDS table full
    }
  }
  }
  __syncthreads();
  // flush: per (block, voxel) two adds and, near a face only, the margin min (~2 global
  // atomics per pair; round 5's owner word -- a third atomic, min(margin << 32 | entry id),
  // every pair -- measured slower: 6.1 vs 5.6 us per 128^3 frame, profiles/r5/).  The
  // returning add detects the voxel's first toucher, which lists it; a thread's slots'
  // returning adds are all issued before any result is used
  if (C3H_VB_DIAG == 0) {
    constexpr int kFl = (kBSlots + kBT - 1) / kBT;
    uint32_t key[kFl];
    unsigned long long old[kFl];
#pragma unroll
    for (int k = 0; k < kFl; ++k) {
      const int s = tid + k * kBT;
      key[k] = s < kBSlots ? s_key[s] : kNoT;
      old[k] = key[k] != kNoT ? __hip_atomic_fetch_add(&acc[key[k]].x, s_A[s], __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE)
                              : 1ull << 40;
    }
#pragma unroll
    for (int k = 0; k < kFl; ++k) {
      const int s = tid + k * kBT;
      if (key[k] == kNoT) continue;
      __hip_atomic_fetch_add(&acc[key[k]].y, s_B[s], __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE);
      if (s_m[s] < kMarginFlush) __hip_atomic_fetch_min(Mg + key[k], s_m[s], __ATOMIC_RELAXED, C3H_VB_ATOM_SCOPE);
      if ((old[k] >> 40) == 0) vl[atomicAdd(&s_nnew, 1u)] = key[k];
    }
  }
#pragma unroll
  for (int ax = 0; ax < 3; ++ax) {
    mn[ax] = wave_reduce(mn[ax], [](int x, int y) { return min(x, y); });
    mx[ax] = wave_reduce(mx[ax], [](int x, int y) { return max(x, y); });
  }
  nv = wave_reduce(nv, [](int x, int y) { return x + y; });
  const int e = wave_reduce(err ? 1 : 0, [](int x, int y) { return x | y; });
  if (lane == 0) {
    for (int ax = 0; ax < 3; ++ax) {
      s_red[w][ax] = mn[ax];
      s_red[w][3 + ax] = mx[ax];
    }
    s_red[w][6] = nv;
    s_red[w][7] = e;
  }
  __syncthreads();
  if (tid < 8) {
    int v = s_red[0][tid];
    for (int i = 1; i < kBT / 64; ++i) {
      const int u = s_red[i][tid];
      v = tid < 3 ? min(v, u) : (tid < 6 ? max(v, u) : (tid == 6 ? v + u : (v | u)));
    }
    pr[tid < 7 ? tid : kPErr] = v;
  }
  if (tid == 8) pr[kPNew] = (int)s_nnew;
}

// one block per frame: its accumulate blocks' records -> the frame's VoxelGrid geometry,
// getSubdivNum and the gate's position limits (a separate launch: a last-block hand-off
// inside voxb_accum kept every block resident until its flush atomics had drained)
__global__ __launch_bounds__(kBlock) void voxb_reduce_kernel(VoxBatchArgs a) {
  __shared__ int s_red[kBlock / 64][8];
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int lo[3] = {INT_MAX, INT_MAX, INT_MAX}, hi[3] = {INT_MIN, INT_MIN, INT_MIN};
  int tv = 0, tn = 0, te = 0;
  for (int qb = a.blk0[f] + tid; qb < a.blk0[f + 1]; qb += kBlock) {
    const int32_t* r = a.part + (size_t)qb * kPartW;
    const int rv = r[kPValid];
    if (rv) {
      for (int ax = 0; ax < 3; ++ax) {
        lo[ax] = min(lo[ax], r[kPMin + ax]);
        hi[ax] = max(hi[ax], r[kPMax + ax]);
      }
    }
    tv += rv;
    tn += r[kPNew];
    te |= r[kPErr];
  }
  for (int ax = 0; ax < 3; ++ax) {
    lo[ax] = wave_reduce(lo[ax], [](int x, int y) { return min(x, y); });
    hi[ax] = wave_reduce(hi[ax], [](int x, int y) { return max(x, y); });
  }
  tv = wave_reduce(tv, [](int x, int y) { return x + y; });
  tn = wave_reduce(tn, [](int x, int y) { return x + y; });
  te = wave_reduce(te, [](int x, int y) { return x | y; });
  if (lane == 0) {
    for (int ax = 0; ax < 3; ++ax) {
      s_red[w][ax] = lo[ax];
      s_red[w][3 + ax] = hi[ax];
    }
    s_red[w][6] = tv;
    s_red[w][7] = tn | (te ? INT_MIN : 0);
  }
  __syncthreads();
  if (tid != 0) return;
  int dv[3];
  bool err = false;
  tv = tn = 0;
  for (int ax = 0; ax < 3; ++ax) {
    int l = INT_MAX, h = INT_MIN;
    for (int i = 0; i < kBlock / 64; ++i) {
      l = min(l, s_red[i][ax]);
      h = max(h, s_red[i][3 + ax]);
    }
    lo[ax] = l;
    dv[ax] = h - l + 1;
  }
  for (int i = 0; i < kBlock / 64; ++i) {
    tv += s_red[i][6];
    tn += s_red[i][7] & INT_MAX;
    err = err || s_red[i][7] < 0;
  }
  const bool over = tv > 0 && (dv[0] > a.C[0] || dv[1] > a.C[1] || dv[2] > a.C[2]);
  int sb[3] = {0, 0, 0};
  if (tv > 0) {
    if (a.subdiv > 0) {  // setVoxelFilter (c3_hlac.cpp:204-231), float arithmetic as there
      if (dv[0] > a.off[0] && dv[1] > a.off[1] && dv[2] > a.off[2])
        for (int ax = 0; ax < 3; ++ax) sb[ax] = (int)ceilf((float)(dv[ax] - a.off[ax]) * a.inv_s);
    } else {
      sb[0] = sb[1] = sb[2] = 1;
    }
  }
  VoxFrameRec& rec = a.info[f];
  for (int ax = 0; ax < 3; ++ax) {
    rec.min_b[ax] = tv > 0 ? lo[ax] : 0;
    rec.max_b[ax] = tv > 0 ? lo[ax] + dv[ax] - 1 : -1;
    rec.sb[ax] = sb[ax];
    a.lim[4 * f + ax] = (over || err) ? 0 : sb[ax];
  }
  a.lim[4 * f + 3] = 0;
  rec.n_valid = (uint32_t)tv;
  rec.n_occ = (uint32_t)tn;  // listed voxels (one entry per voxel: its first toucher)
  rec.flagged = 0;  // the scatter adds its flags
  rec.err = (err ? 1u : 0u) | (over ? 2u : 0u);
  rec.moved = 0;
  if (a.xcnt)
    for (int k = 0; k < 4; ++k) a.xcnt[4 * f + k] = 0u;
}

#ifndef C3H_VB_STAMP_DEDUP
#define C3H_VB_STAMP_DEDUP 1  // the scatter's tile stamps deduplicated per workgroup in LDS
#endif
__global__ __launch_bounds__(kBlock) void voxb_scatter_kernel(VoxBatchArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const int f = vb_frame(a.blk0, a.nf, b);
  const VoxFrameRec& rec = a.info[f];  // published by the last accumulate block of the frame
  if (rec.n_valid == 0) return;
  const int lo[3] = {rec.min_b[0], rec.min_b[1], rec.min_b[2]};
  const int Cx = a.C[0], Cy = a.C[1];
  const uint32_t mx_ = (1u << a.tb[0]) - 1, my_ = (1u << a.tb[1]) - 1, mz_ = (1u << a.tb[2]) - 1;
  const int sy = a.tb[0], sz = a.tb[0] + a.tb[1];
  const int nseg = a.part[(size_t)b * kPartW + kPNew];
  const uint32_t* vl = a.vlist + (size_t)b * kBChunk;
  uint32_t* wl = a.wlist + (size_t)b * kBChunk;
  ulonglong2* __restrict__ acc = a.acc + f * a.s_acc;
  uint32_t* __restrict__ Mg = a.accM + f * a.s_acc;
  uint32_t* __restrict__ grid = a.grid[f];
  // the tick's tile stamps (occupancy_bits_body's rule: a centre voxel of subdivision
  // t = mx[x] + ns0 (my[y] + ns1 mz[z]) stamps t; the first stamper lists it)
  const int16_t* __restrict__ ax = a.axmap;
  uint32_t* __restrict__ flags = a.stamp ? a.tf + f * a.s_tf + 4 : nullptr;
  uint32_t* cnt = a.stamp ? a.tf + f * a.s_tf + 2 + (a.epoch & 1) : nullptr;
  int32_t* __restrict__ work = a.stamp ? a.work + f * a.s_work : nullptr;
  const int lane = tid & 63;
  // tiles this workgroup stamped already: one global exchange per (workgroup, tile)
  extern __shared__ uint32_t vb_stamped[];
  if (a.stamp) {
    for (int i = tid; i < (a.ntiles + 31) / 32; i += kBlock) vb_stamped[i] = 0u;
    __syncthreads();
  }
  uint32_t flagged = 0;
  for (int i0 = 0; i0 < nseg; i0 += kBlock) {  // wave-uniform trip count (the stamp ballots)
    const int i = i0 + tid;
    int tile = -1;
    if (i < nseg) {  // every listed voxel is listed once (by its first toucher)
      const uint32_t t = vl[i];
      const ulonglong2 v = take_acc(&acc[t]);
      const uint32_t m = Mg[t];
      if (m != kNoMargin) Mg[t] = kNoMargin;  // only the rare near-face voxels changed it
      // offsets from min_b: the toroidal coordinates minus min_b, modulo 2^tb
      const uint32_t cx = ((t & mx_) - (uint32_t)lo[0]) & mx_;
      const uint32_t cy = (((t >> sy) & my_) - (uint32_t)lo[1]) & my_;
      const uint32_t cz = (((t >> sz) & mz_) - (uint32_t)lo[2]) & mz_;
      // an extent beyond the canvas (flagged by the reduction) may land past it: clamp
      const uint32_t kx = min(cx, (uint32_t)Cx - 1), ky = min(cy, (uint32_t)Cy - 1), kz = min(cz, (uint32_t)a.C[2] - 1);
      const uint32_t idx = kx + (uint32_t)Cx * (ky + (uint32_t)Cy * kz);
      const uint32_t count = (uint32_t)(v.x >> 40);
      grid[idx] = pcl_colour_word(v.x & 0xffffffffffull, v.y & 0xffffffffull, v.y >> 32, count);
      wl[i] = idx;
      if (a.stamp) {
        const int sx = ax[kx], sy_ = ax[Cx + ky], sz_ = ax[Cx + Cy + kz];
        if (sx >= 0 && sy_ >= 0 && sz_ >= 0) tile = sx + a.ns0 * (sy_ + a.ns1 * sz_);
      }
      // the exact centroid test of vox_scatter_kernel on the absolute cell
      const int ax_ = lo[0] + (int)cx, ay_ = lo[1] + (int)cy, az_ = lo[2] + (int)cz;
      const int cmag = max(max(abs(ax_), abs(ay_)), abs(az_)) + 1;
      const float eps = (float)(count + 4) * (float)cmag * 0x1p-22f;
      if (__uint_as_float(m) < eps || eps >= __uint_as_float(kMarginFlush)) {
        ++flagged;
        if (a.flags) {  // to the exact pass: its points are bucketed and summed in input order
          uint32_t* xc = a.xcnt + 4 * f;
          const uint32_t k = atomicAdd(xc, 1u);
          const uint32_t o = atomicAdd(xc + 1, count);
          if (k < (uint32_t)kVbFlagCap && o + count <= (uint32_t)kVbBucketCap)
            a.flags[(size_t)f * kVbFlagCap + k] = VoxFlag{t, idx, count, o, 0u, 0u};
          else
            atomicOr(&a.info[f].err, 4u);
        }
      }
    }
    if (a.stamp) {  // uniform
      // neighbouring entries were first touched by neighbouring points: mostly one tile
      const int tp = __shfl_up(tile, 1, 64);
      bool cand = tile >= 0 && !(lane > 0 && tp == tile);
      if (C3H_VB_STAMP_DEDUP && cand) {
        const uint32_t bit = 1u << (tile & 31);
        cand = (atomicOr(&vb_stamped[tile >> 5], bit) & bit) == 0u;
      } else if (cand) {  // (diagnostics: a plain read of the stamp instead)
        cand = flags[tile] != a.epoch;
      }
      const bool fresh = cand && atomicExch(&flags[tile], a.epoch) != a.epoch;
      const unsigned long long bm = __ballot(fresh);
      if (bm) {
        uint32_t b0 = 0;
        if (lane == 0) b0 = atomicAdd(cnt, (uint32_t)__popcll(bm));
        b0 = __shfl(b0, 0, 64);
        if (fresh) work[b0 + __popcll(bm & ((1ull << lane) - 1))] = tile;
      }
    }
  }
  flagged = wave_reduce(flagged, [](uint32_t u, uint32_t v) { return u + v; });
  if ((tid & 63) == 0 && flagged) atomicAdd(&a.info[f].flagged, flagged);
}

// ---- exact centroids of the flagged voxels (round 4) ---------------------------------
// voxb_bucket: kBucketSplit blocks per block b of the accumulate grid re-read its points
// (a quarter each, loaded together; frames without flagged voxels return at once) and file
// every point of a flagged voxel (an LDS hash of the frame's flagged keys) into that
// voxel's bucket.
constexpr int kVbFlagSlots = 2 * kVbFlagCap;
constexpr int kBucketSplit = 4;  // blocks per accumulate chunk (each re-reads a quarter of its points)
static_assert(kBPer % kBucketSplit == 0, "bucket split");
static_assert((kVbFlagSlots & (kVbFlagSlots - 1)) == 0, "flag hash");
// A bounded grid (kBucketGrid blocks: one dispatch round) walks the (chunk, quarter) items:
// frames without flagged voxels -- all of the synthetic points-in frames -- cost a counter
// read per item instead of a dispatched 48 KB-LDS block each (round 6: 15.6k empty blocks
// per 64-frame batch took ~20 us of the voxeliser's critical path)
constexpr int kBucketGrid = 768;
__global__ __launch_bounds__(kBT) void voxb_bucket_kernel(VoxBatchArgs a, int nitems) {
  __shared__ uint32_t s_key[kVbFlagSlots];
  __shared__ uint16_t s_rec[kVbFlagSlots];
  const int tid = threadIdx.x;
  // a batch without a flagged voxel in any frame (all synthetic points-in batches): one
  // load per frame, every block out at once
  __shared__ int s_any;
  if (tid < 64) {
    const bool fl = tid < a.nf && a.xcnt[4 * tid] != 0u;
    const unsigned long long m = __ballot(fl);
    if (tid == 0) s_any = m != 0ull;
  }
  __syncthreads();
  if (!s_any) return;
  int f_tab = -1;  // the frame whose flagged keys s_key holds
  for (int w = blockIdx.x; w < nitems; w += gridDim.x) {  // uniform per block
    const int b = w / kBucketSplit, qy = w - b * kBucketSplit;
    const int f = vb_frame(a.blk0, a.nf, b);
    const uint32_t nflag = a.xcnt[4 * f];
    if (nflag == 0 || a.info[f].err) continue;  // uniform
    const int nrec = (int)min(nflag, (uint32_t)kVbFlagCap);
    VoxFlag* fl = a.flags + (size_t)f * kVbFlagCap;
    uint32_t* bk = a.bucket + (size_t)f * kVbBucketCap;
    if (f != f_tab) {
      __syncthreads();  // the previous frame's lookups are done
      for (int s = tid; s < kVbFlagSlots; s += kBT) s_key[s] = kNoT;
      __syncthreads();
      for (int r = tid; r < nrec; r += kBT) {
        const uint32_t t = fl[r].t;
        uint32_t h = (t * 0x9E3779B1u) >> (32 - __builtin_ctz(kVbFlagSlots));
        while (atomicCAS(&s_key[h], kNoT, t) != kNoT) h = (h + 1) & (kVbFlagSlots - 1);
        s_rec[h] = (uint16_t)r;
      }
      __syncthreads();
      f_tab = f;
    }
    const int64_t base = (int64_t)(b - a.blk0[f]) * kBChunk;
    const float4* __restrict__ pts = a.pts[f];
    const int64_t n = a.n[f];
    const uint32_t mx_ = (1u << a.tb[0]) - 1, my_ = (1u << a.tb[1]) - 1, mz_ = (1u << a.tb[2]) - 1;
    const int sy = a.tb[0], sz = a.tb[0] + a.tb[1];
    // this item's share of the chunk: kBPer / kBucketSplit points per thread, loaded together
    constexpr int kPer = kBPer / kBucketSplit;
    float4 p[kPer];
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t i = base + (int64_t)(qy * kPer + q) * kBT + tid;
      p[q] = i < n ? pts[i] : make_float4(NAN, NAN, NAN, 0.0f);
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int64_t i = base + (int64_t)(qy * kPer + q) * kBT + tid;
      int c[3];
      float margin;
      if (!point_valid(p[q], a.z_limit) || !point_cell(a.inv, p[q], c, &margin)) continue;
      const uint32_t t = ((uint32_t)c[0] & mx_) | (((uint32_t)c[1] & my_) << sy) | (((uint32_t)c[2] & mz_) << sz);
      uint32_t h = (t * 0x9E3779B1u) >> (32 - __builtin_ctz(kVbFlagSlots));
      for (;;) {
        const uint32_t k = s_key[h];
        if (k == kNoT) break;
        if (k == t) {
          VoxFlag& r = fl[s_rec[h]];
          bk[r.off + atomicAdd(&r.cur, 1u)] = (uint32_t)i;
          break;
        }
        h = (h + 1) & (kVbFlagSlots - 1);
      }
    }
  }
}

// voxb_exact: kExactSplit blocks per frame, a thread per flagged voxel: its points in input
// order (the bucket copied to the thread's LDS slice, 8 loads in flight, and insertion-
// sorted there when it holds <= 64 points; a shell sort in place otherwise), the fp32 sequential sum times 1/n (PCL 1.0 on
// Eigen 3.0, as the single-frame path and the oracle; the point loads issued 8 ahead of the
// adds, which stay in order), the centroid cell floor(c / leaf); a voxel whose centroid
// cell is not its own cell goes to the frame's moved list (the fixup after the tile role).
// A centroid cell past the frame's last subdivision (where the reference reads beyond its
// histograms) sends the frame to the single-frame path.  (Round 4 ran one block per frame
// with the sort in global memory: 136 us per 32-frame batch on the voxeliser's stream.)
constexpr int kExactSplit = 16;
constexpr int kExactLds = 64;  // bucket entries per thread sorted in LDS (64 KB; the real Kinect
                               // views' near-face voxels hold <= 66 points, 99 % <= 51)
__global__ __launch_bounds__(kBlock) void voxb_exact_kernel(VoxBatchArgs a) {
  __shared__ uint32_t s_bk[kBlock * kExactLds];
  const int f = blockIdx.x, tid = threadIdx.x;
  VoxFrameRec& rec = a.info[f];
  const uint32_t nflag = a.xcnt[4 * f];
  if (nflag == 0 || rec.err) return;
  const int nrec = (int)min(nflag, (uint32_t)kVbFlagCap);
  const VoxFlag* fl = a.flags + (size_t)f * kVbFlagCap;
  uint32_t* bks = a.bucket + (size_t)f * kVbBucketCap;
  const float4* __restrict__ pts = a.pts[f];
  const int Cx = a.C[0], Cy = a.C[1];
  uint32_t* mine = s_bk + tid;  // this thread's slice, strided by kBlock (bank-conflict free)
  for (int r = blockIdx.y * kBlock + tid; r < nrec; r += kBlock * gridDim.y) {
    const VoxFlag e = fl[r];
    const int m = (int)e.count;
    uint32_t* bk = bks + e.off;
    const bool small = m <= kExactLds;
    if (small) {
      for (int u0 = 0; u0 < m; u0 += 8) {  // the bucket into LDS, 8 loads in flight
        uint32_t t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) t[q] = u0 + q < m ? bk[u0 + q] : 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (u0 + q < m) mine[(u0 + q) * kBlock] = t[q];
      }
      for (int u = 1; u < m; ++u) {  // insertion sort in LDS
        const uint32_t t = mine[u * kBlock];
        int v = u;
        for (; v > 0 && mine[(v - 1) * kBlock] > t; --v) mine[v * kBlock] = mine[(v - 1) * kBlock];
        mine[v * kBlock] = t;
      }
    } else {
      const int gaps[8] = {701, 301, 132, 57, 23, 10, 4, 1};
      for (int gi = 0; gi < 8; ++gi) {
        const int gap = gaps[gi];
        for (int u = gap; u < m; ++u) {
          const uint32_t t = bk[u];
          int v = u;
          for (; v >= gap && bk[v - gap] > t; v -= gap) bk[v] = bk[v - gap];
          bk[v] = t;
        }
      }
    }
    float sx = 0.0f, sy = 0.0f, sz = 0.0f;
    for (int u0 = 0; u0 < m; u0 += 8) {
      float4 p[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int u = u0 + q;
        p[q] = u < m ? pts[small ? mine[u * kBlock] : bk[u]] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if (u0 + q < m) {
          sx += p[q].x;
          sy += p[q].y;
          sz += p[q].z;
        }
      }
    }
    const float rn = __fdiv_rn(1.0f, (float)m);
    const float c[3] = {__fmul_rn(sx, rn), __fmul_rn(sy, rn), __fmul_rn(sz, rn)};
    const int own[3] = {(int)(e.idx % (uint32_t)Cx), (int)((e.idx / (uint32_t)Cx) % (uint32_t)Cy),
                        (int)(e.idx / ((uint32_t)Cx * (uint32_t)Cy))};
    int bc[3];
    bool moved = false;
    for (int ax = 0; ax < 3; ++ax) {
      bc[ax] = (int)floorf(__fdiv_rn(c[ax], a.leaf)) - rec.min_b[ax];  // canvas coordinates
      moved = moved || bc[ax] != own[ax];
    }
    if (!moved) continue;
    // a centroid cell past the canvas (a frame whose extent fills an axis, a boundary voxel
    // whose centroid rounds up past it): the fixup's canvas maps have no entry there (its
    // centre subdivision would be dropped), while the reference may still count the voxel
    // in the last subdivision -- the frame takes the single-frame path.  (Below the canvas,
    // bc = -1, the reference's tmp < 0 is no centre either: the fixup agrees.)
    if (bc[0] >= Cx || bc[1] >= Cy || bc[2] >= a.C[2]) {
      atomicOr(&rec.err, 8u);
      continue;
    }
    if (a.subdiv > 0) {  // computeC3HLAC's subdivision of the centroid (c3_hlac.cpp:349-362)
      bool centre = true, past = false;
      for (int ax = 0; ax < 3; ++ax) {
        const int tmp = bc[ax] - a.off[ax];
        centre = centre && tmp >= 0;
        past = past || (tmp >= 0 && (int)floorf((float)tmp * a.inv_s) >= rec.sb[ax]);
      }
      if (centre && past) {
        atomicOr(&rec.err, 8u);
        continue;
      }
    }
    const uint32_t k = atomicAdd(a.xcnt + 4 * f + 2, 1u);
    if (k < (uint32_t)kVbMovedCap)
      a.moved[(size_t)f * kVbMovedCap + k] = VoxMoved{e.idx, {bc[0], bc[1], bc[2]}};
    else
      atomicOr(&rec.err, 4u);
    atomicAdd(&rec.moved, 1u);
  }
}

}  // namespace

int vb_chunk() { return kBChunk; }

hipError_t launch_vox_batch(const VoxBatchArgs& a, hipStream_t s) {
  const hipError_t e = launch_vox_batch_accum(a, s);
  return e != hipSuccess ? e : launch_vox_batch_post(a, s);
}

hipError_t launch_vox_batch_accum(const VoxBatchArgs& a, hipStream_t s) {
  const int g = std::max(a.total, a.prev_total);
  if (g > 0) voxb_accum_kernel<<<(unsigned)g, kBT, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_vox_batch_post(const VoxBatchArgs& a, hipStream_t s) {
  if (a.total > 0) {
    voxb_reduce_kernel<<<(unsigned)a.nf, kBlock, 0, s>>>(a);
    voxb_scatter_kernel<<<(unsigned)a.total, kBlock, a.stamp ? 4 * (size_t)((a.ntiles + 31) / 32) : 0, s>>>(a);
    if (a.flags) {
      const int items = a.total * kBucketSplit;
      voxb_bucket_kernel<<<(unsigned)std::min(items, kBucketGrid), kBT, 0, s>>>(a, items);
      voxb_exact_kernel<<<dim3((unsigned)a.nf, kExactSplit), kBlock, 0, s>>>(a);
    }
  }
  return hipGetLastError();
}

int64_t scan_blocks(int64_t n) { return (n + kScanBlock - 1) / kScanBlock; }
int64_t leaf_layout_blocks(int64_t nvox) { return scan_blocks(nvox); }

hipError_t launch_voxelize(const VoxArgs& a, hipStream_t s) {
  // at least one accum block: it also clears the previous frame and resets the totals
  vox_accum_kernel<<<(unsigned)std::max(a.nblk, 1), kVB, 0, s>>>(a);
  if (a.nblk > 0) vox_scatter_kernel<<<(unsigned)a.nblk, kBlock, 0, s>>>(a);
  return hipGetLastError();
}


hipError_t launch_vox_accum(const VoxArgs& a, int nblocks, hipStream_t s) {
  if (nblocks > 0) vox_accum_kernel<<<(unsigned)nblocks, kVB, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_vox_scatter(const VoxArgs& a, hipStream_t s) {
  if (a.nblk > 0) vox_scatter_kernel<<<(unsigned)a.nblk, kBlock, 0, s>>>(a);
  return hipGetLastError();
}

int64_t vox_blocks(int64_t n) { return (n + kVoxChunk - 1) / kVoxChunk; }
int64_t vox_positions(int64_t n) { return vox_blocks(n) * kVoxChunk; }
int vox_part_words() { return kPartW; }

hipError_t launch_vox_centroids(const VoxArgs& a, uint32_t* counts, uint32_t* offs, uint32_t* cur,
                                uint32_t* block_sums, uint32_t* bucket, float4* cent, int32_t* offcell,
                                hipStream_t s) {
  const int64_t np = (int64_t)a.nblk * kVoxChunk;
  if (np <= 0) return hipSuccess;
  vox_counts_kernel<<<grid_for(np), kBlock, 0, s>>>(a, counts);
  const int64_t nb = scan_blocks(np);
  scan_count_kernel<false><<<(unsigned)nb, kBlock, 0, s>>>(counts, np, block_sums);
  scan_sums_kernel<<<1, kBlock, 0, s>>>(block_sums, nb);
  scan_write_kernel<false><<<(unsigned)nb, kBlock, 0, s>>>(counts, np, block_sums, reinterpret_cast<int32_t*>(offs));
  hipError_t e = hipMemsetAsync(cur, 0, (size_t)np * 4, s);
  if (e != hipSuccess) return e;
  vox_bucket_kernel<<<grid_for(a.n, 8192), kBlock, 0, s>>>(a, offs, counts, cur, bucket);
  vox_centroid_kernel<<<grid_for(np), kBlock, 0, s>>>(a, offs, counts, cur, bucket, cent, offcell);
  return hipGetLastError();
}

hipError_t launch_vox_clear(const VoxArgs& a, hipStream_t s) {
  if (a.nblk > 0) vox_clear_kernel<<<(unsigned)a.nblk, kBlock, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_vox_sorted(const VoxArgs& a, const int mn[3], const int dv[3], int64_t nv, VoxSortBufs& b,
                             uint32_t* counts, float4* cent, int32_t* offcell, hipStream_t s) {
  const int64_t nvox = (int64_t)dv[0] * dv[1] * dv[2];
  int bits = 1;  // the keys' width: voxel indices and the sentinel nvox
  while (bits < 32 && ((int64_t)1 << bits) <= nvox) ++bits;
  const size_t n = (size_t)std::max<int64_t>(a.n, 1);
  if (!b.tmp)  // size query
    return rocprim::radix_sort_pairs(nullptr, b.tmp_bytes, b.keys, b.keys2, b.idx, b.idx2, n, 0, bits, s);
  if (a.n <= 0 || nv <= 0) return hipSuccess;
  const int3 m3 = make_int3(mn[0], mn[1], mn[2]), d3 = make_int3(dv[0], dv[1], dv[2]);
  voxs_keys_kernel<<<grid_for(a.n, 8192), kBlock, 0, s>>>(a, m3, d3, (uint32_t)nvox, b.keys, b.idx);
  hipError_t e = rocprim::radix_sort_pairs(b.tmp, b.tmp_bytes, b.keys, b.keys2, b.idx, b.idx2, (size_t)a.n, 0, bits, s);
  if (e != hipSuccess) return e;
  voxs_heads_kernel<<<grid_for(nv, 8192), kBlock, 0, s>>>(b.keys2, nv, b.head);
  const int64_t nb = scan_blocks(nv);
  scan_count_kernel<false><<<(unsigned)nb, kBlock, 0, s>>>(b.head, nv, b.block_sums);
  scan_sums_kernel<<<1, kBlock, 0, s>>>(b.block_sums, nb);
  scan_write_kernel<false><<<(unsigned)nb, kBlock, 0, s>>>(b.head, nv, b.block_sums, b.ord);
  e = hipMemsetAsync(counts, 0, (size_t)a.nblk * kVoxChunk * 4, s);
  if (e != hipSuccess) return e;
  voxs_emit_kernel<<<grid_for(nv, 8192), kBlock, 0, s>>>(a, m3, d3, b.keys2, b.idx2, b.head, b.ord, nv, counts, cent,
                                                          offcell);
  voxs_parts_kernel<<<(unsigned)((a.nblk + kBlock - 1) / kBlock), kBlock, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_vox_downsampled(const VoxArgs& a, const float4* cent, const uint32_t* counts, const int32_t* leaf,
                                  float* out, hipStream_t s) {
  const int64_t np = (int64_t)a.nblk * kVoxChunk;
  if (np <= 0) return hipSuccess;
  vox_downsampled_kernel<<<grid_for(np), kBlock, 0, s>>>(a, cent, counts, leaf, reinterpret_cast<float4*>(out));
  return hipGetLastError();
}

hipError_t launch_leaf_layout(const uint32_t* grid, int64_t nvox, int32_t* leaf,
                              uint32_t* block_sums, int64_t nblocks, hipStream_t s) {
  scan_count_kernel<true><<<(unsigned)nblocks, kBlock, 0, s>>>(grid, nvox, block_sums);
  scan_sums_kernel<<<1, kBlock, 0, s>>>(block_sums, nblocks);
  scan_write_kernel<true><<<(unsigned)nblocks, kBlock, 0, s>>>(grid, nvox, block_sums, leaf);
  return hipGetLastError();
}

}  // namespace c3h
