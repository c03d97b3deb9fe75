// voxelize.hip -- hash-and-scatter voxeliser for gfx950 (PCL VoxelGrid semantics).
//
// Replaces getVoxelGrid (c3_hlac/include/c3_hlac/c3_hlac_tools.hpp:124-130 -> PCL
// VoxelGrid::filter, semantics restated in SURVEY.md App. B) and limitPoint
// (color_voxel_recognition/test/detect_object.cpp:68-87).
//
// Pass 1 (minmax): one coalesced 16-B read per point; finite && z < z_limit filter;
//   wave/block reduction of the bounds, one atomic per block.
// Pass 2 (accum): voxel index = floor(p * inv_leaf) - min_b (float multiply + floor,
//   exactly PCL's), inserted into an open-addressing hash table sized >= 2x the valid
//   points; integer atomics accumulate count and r/g/b sums (exact), float atomics the
//   xyz sums (only used for the optional downsampled cloud).
// Pass 3 (scatter): one word per occupied voxel into the dense packed grid:
//   kOcc | r<<16 | g<<8 | b with r = (int)(float(sum_r) / float(count)) (IEEE divide,
//   the canonical PCL >= 1.2 colour rule).
#include "c3h_internal.h"

namespace c3h {
namespace {

__device__ __forceinline__ uint32_t enc_f(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
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

__global__ __launch_bounds__(kBlock) void minmax_kernel(const float4* __restrict__ pts,
                                                        int64_t n, float z_limit,
                                                        uint32_t* __restrict__ out) {
  uint32_t mn[3] = {0xffffffffu, 0xffffffffu, 0xffffffffu}, mx[3] = {0, 0, 0};
  uint32_t cnt = 0;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const float4 p = pts[i];
    if (!point_valid(p, z_limit)) continue;
    ++cnt;
    const uint32_t e[3] = {enc_f(p.x), enc_f(p.y), enc_f(p.z)};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      mn[a] = min(mn[a], e[a]);
      mx[a] = max(mx[a], e[a]);
    }
  }
  auto umin = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
  auto umax = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  auto uadd = [](uint32_t a, uint32_t b) { return a + b; };
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    mn[a] = wave_reduce(mn[a], umin);
    mx[a] = wave_reduce(mx[a], umax);
  }
  cnt = wave_reduce(cnt, uadd);
  // block reduction in LDS, then one set of atomics per block (same-address atomics
  // from every wave serialise at the memory side)
  __shared__ uint32_t red[kBlock / 64][7];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int a = 0; a < 3; ++a) {
      red[w][a] = mn[a];
      red[w][3 + a] = mx[a];
    }
    red[w][6] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < kBlock / 64; ++i) {
      for (int a = 0; a < 3; ++a) {
        red[0][a] = umin(red[0][a], red[i][a]);
        red[0][3 + a] = umax(red[0][3 + a], red[i][3 + a]);
      }
      red[0][6] += red[i][6];
    }
    for (int a = 0; a < 3; ++a) {
      atomicMin(&out[a], red[0][a]);
      atomicMax(&out[3 + a], red[0][3 + a]);
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(out + 6), (unsigned long long)red[0][6]);
  }
}

__device__ __forceinline__ uint32_t hash_key(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  k *= 0x846ca68bu;
  k ^= k >> 16;
  return k;
}

__global__ __launch_bounds__(kBlock) void accum_kernel(
    const float4* __restrict__ pts, int64_t n, float z_limit, float inv, int mbx, int mby,
    int mbz, int dx, int dy, uint32_t* __restrict__ keys, uint32_t* __restrict__ cnt,
    uint32_t* __restrict__ sr, uint32_t* __restrict__ sg, uint32_t* __restrict__ sb,
    float* __restrict__ sx, float* __restrict__ sy, float* __restrict__ sz, uint64_t mask,
    uint32_t* __restrict__ overflow) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const float4 p = pts[i];
    if (!point_valid(p, z_limit)) continue;
    // PCL: static_cast<int>(floor(p * inverse_leaf_size) - static_cast<float>(min_b))
    const int ix = (int)(floorf(p.x * inv) - (float)mbx);
    const int iy = (int)(floorf(p.y * inv) - (float)mby);
    const int iz = (int)(floorf(p.z * inv) - (float)mbz);
    const uint32_t key = (uint32_t)ix + (uint32_t)iy * (uint32_t)dx + (uint32_t)iz * (uint32_t)dx * (uint32_t)dy;
    uint64_t h = hash_key(key) & mask;
    uint64_t probes = 0;
    for (;;) {
      const uint32_t prev = atomicCAS(&keys[h], kEmptyKey, key);
      if (prev == kEmptyKey || prev == key) break;
      h = (h + 1) & mask;
      if (++probes > mask) {
        atomicOr(overflow, 1u);
        break;
      }
    }
    if (probes > mask) continue;
    const uint32_t rgb = __float_as_uint(p.w);
    atomicAdd(&cnt[h], 1u);
    atomicAdd(&sr[h], (rgb >> 16) & 0xffu);
    atomicAdd(&sg[h], (rgb >> 8) & 0xffu);
    atomicAdd(&sb[h], rgb & 0xffu);
    if (sx) {
      atomicAdd(&sx[h], p.x);
      atomicAdd(&sy[h], p.y);
      atomicAdd(&sz[h], p.z);
    }
  }
}

__global__ __launch_bounds__(kBlock) void scatter_kernel(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
    const uint32_t* __restrict__ sr, const uint32_t* __restrict__ sg,
    const uint32_t* __restrict__ sb, uint64_t table_size, uint32_t* __restrict__ grid,
    uint32_t* __restrict__ n_occ) {
  uint32_t local = 0;
  for (uint64_t s = blockIdx.x * (uint64_t)kBlock + threadIdx.x; s < table_size;
       s += (uint64_t)gridDim.x * kBlock) {
    const uint32_t key = keys[s];
    if (key == kEmptyKey) continue;
    const float c = (float)cnt[s];
    const uint32_t r = (uint32_t)(int)__fdiv_rn((float)sr[s], c);
    const uint32_t g = (uint32_t)(int)__fdiv_rn((float)sg[s], c);
    const uint32_t b = (uint32_t)(int)__fdiv_rn((float)sb[s], c);
    grid[key] = kOcc | (r << 16) | (g << 8) | b;
    ++local;
  }
  auto uadd = [](uint32_t a, uint32_t b) { return a + b; };
  local = wave_reduce(local, uadd);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(n_occ, local);
}

// ---- leaf layout: exclusive scan of occupancy over the grid (not on the timed path)
constexpr int kScanItems = 4;  // voxels per thread
constexpr int kScanBlock = kBlock * kScanItems;

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds,
                                                         uint32_t* total) {
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

__global__ __launch_bounds__(kBlock) void occ_count_kernel(const uint32_t* __restrict__ grid,
                                                           int64_t nvox,
                                                           uint32_t* __restrict__ sums) {
  __shared__ uint32_t lds[kBlock / 64];
  const int64_t base = blockIdx.x * (int64_t)kScanBlock + threadIdx.x * kScanItems;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j)
    if (base + j < nvox && grid[base + j]) ++c;
  uint32_t tot;
  block_exclusive_scan(c, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_sums_kernel(uint32_t* __restrict__ sums,
                                                           int64_t nblocks) {
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

__global__ __launch_bounds__(kBlock) void leaf_write_kernel(const uint32_t* __restrict__ grid,
                                                            int64_t nvox,
                                                            const uint32_t* __restrict__ sums,
                                                            int32_t* __restrict__ leaf) {
  __shared__ uint32_t lds[kBlock / 64];
  const int64_t base = blockIdx.x * (int64_t)kScanBlock + threadIdx.x * kScanItems;
  uint32_t occ[kScanItems];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    occ[j] = (base + j < nvox && grid[base + j]) ? 1u : 0u;
    c += occ[j];
  }
  uint32_t tot;
  uint32_t rank = sums[blockIdx.x] + block_exclusive_scan(c, lds, &tot);
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j >= nvox) break;
    leaf[base + j] = occ[j] ? (int32_t)rank : -1;
    rank += occ[j];
  }
}

__global__ __launch_bounds__(kBlock) void downsampled_kernel(
    const int32_t* __restrict__ leaf, const uint32_t* __restrict__ grid, int64_t nvox,
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ cnt,
    const float* __restrict__ sx, const float* __restrict__ sy, const float* __restrict__ sz,
    uint64_t mask, float* __restrict__ out) {
  for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nvox;
       v += (int64_t)gridDim.x * kBlock) {
    const int32_t rk = leaf[v];
    if (rk < 0) continue;
    const uint32_t key = (uint32_t)v;
    uint64_t h = hash_key(key) & mask;
    for (uint64_t probes = 0; probes <= mask; ++probes) {
      if (keys[h] == key) break;
      h = (h + 1) & mask;
    }
    const float c = (float)cnt[h];
    float4 o;
    o.x = __fdiv_rn(sx[h], c);
    o.y = __fdiv_rn(sy[h], c);
    o.z = __fdiv_rn(sz[h], c);
    o.w = __uint_as_float(grid[v] & 0x00ffffffu);
    reinterpret_cast<float4*>(out)[rk] = o;
  }
}

int grid_for(int64_t n, int cap = 4096) {
  int64_t g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

}  // namespace

hipError_t launch_minmax(const float4* pts, int64_t n, float z_limit, uint32_t* out,
                         hipStream_t s) {
  minmax_kernel<<<grid_for(n, 512), kBlock, 0, s>>>(pts, n, z_limit, out);
  return hipGetLastError();
}

hipError_t launch_voxel_accum(const float4* pts, int64_t n, float z_limit, float inv,
                              const int32_t min_b[3], const int32_t div_b[3], uint32_t* keys,
                              uint32_t* cnt, uint32_t* sr, uint32_t* sg, uint32_t* sb,
                              float* sx, float* sy, float* sz, uint64_t table_size,
                              uint32_t* overflow, hipStream_t s) {
  accum_kernel<<<grid_for(n, 8192), kBlock, 0, s>>>(pts, n, z_limit, inv, min_b[0], min_b[1],
                                                     min_b[2], div_b[0], div_b[1], keys, cnt,
                                                     sr, sg, sb, sx, sy, sz, table_size - 1,
                                                     overflow);
  return hipGetLastError();
}

hipError_t launch_voxel_scatter(const uint32_t* keys, const uint32_t* cnt, const uint32_t* sr,
                                const uint32_t* sg, const uint32_t* sb, uint64_t table_size,
                                uint32_t* grid, uint32_t* n_occ, hipStream_t s) {
  scatter_kernel<<<grid_for((int64_t)table_size), kBlock, 0, s>>>(keys, cnt, sr, sg, sb,
                                                                  table_size, grid, n_occ);
  return hipGetLastError();
}

hipError_t launch_leaf_layout(const uint32_t* grid, int64_t nvox, int32_t* leaf,
                              uint32_t* block_sums, int64_t nblocks, hipStream_t s) {
  occ_count_kernel<<<(unsigned)nblocks, kBlock, 0, s>>>(grid, nvox, block_sums);
  scan_sums_kernel<<<1, kBlock, 0, s>>>(block_sums, nblocks);
  leaf_write_kernel<<<(unsigned)nblocks, kBlock, 0, s>>>(grid, nvox, block_sums, leaf);
  return hipGetLastError();
}

int64_t leaf_layout_blocks(int64_t nvox) { return (nvox + kScanBlock - 1) / kScanBlock; }

hipError_t launch_downsampled(const int32_t* leaf, const uint32_t* grid, int64_t nvox,
                              const int32_t div_b[3], const uint32_t* keys, const uint32_t* cnt,
                              const float* sx, const float* sy, const float* sz,
                              uint64_t table_size, float* out, hipStream_t s) {
  (void)div_b;
  downsampled_kernel<<<grid_for(nvox, 8192), kBlock, 0, s>>>(leaf, grid, nvox, keys, cnt, sx,
                                                             sy, sz, table_size - 1, out);
  return hipGetLastError();
}

}  // namespace c3h
