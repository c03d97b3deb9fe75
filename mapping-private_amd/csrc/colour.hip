// colour.hip -- automatic colour threshold: the per-channel 256-bin
// histograms of the occupied voxels' colours that calc_scene_auto_threshold.cpp:84-109
// accumulates over the downsampled scene clouds, and its between-class-variance argmax
// (:111-146) on the host.
//
// The voxel colours are the packed grid's words (1 << 24 | r << 16 | g << 8 | b, the
// canonical PCL centroid colour; 0 = empty), so the histogram is one HBM stream of the grid
// (4 B/voxel): 16-B non-temporal loads, 8 per lane in flight, one LDS histogram copy per
// wave (3 x 256 u32; LDS atomics of different waves never contend), merged into 768 u64
// global counters once per workgroup.  Counts are exact integers.
#include <algorithm>

#include "c3h_internal.h"

namespace c3h {
namespace {

constexpr int kHistUnroll = 8;
constexpr int kHistWaves = kBlock / 64;

__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t w) {
  if (w) {  // an occupied voxel: +1 in each channel's bin (result unused: ds_add, no wait)
    atomicAdd(&h[(w >> 16) & 0xffu], 1u);
    atomicAdd(&h[256 + ((w >> 8) & 0xffu)], 1u);
    atomicAdd(&h[512 + (w & 0xffu)], 1u);
  }
}

__global__ __launch_bounds__(kBlock) void colour_hist_kernel(const uint32_t* __restrict__ grid, int64_t nvox,
                                                             unsigned long long* __restrict__ out) {
  __shared__ uint32_t s_h[kHistWaves * 768];
  const int tid = threadIdx.x;
  for (int i = tid; i < kHistWaves * 768; i += kBlock) s_h[i] = 0u;
  __syncthreads();
  uint32_t* h = s_h + (tid >> 6) * 768;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const int64_t n4 = nvox >> 2;
  const v4u* g4 = reinterpret_cast<const v4u*>(grid);
  constexpr int kChunk = kBlock * kHistUnroll;
  for (int64_t c0 = blockIdx.x * (int64_t)kChunk; c0 < n4; c0 += (int64_t)gridDim.x * kChunk) {
    v4u w[kHistUnroll];
#pragma unroll
    for (int j = 0; j < kHistUnroll; ++j) {  // all loads first; clamped address + select
      const int64_t i = c0 + j * kBlock + tid;
      const v4u t = __builtin_nontemporal_load(g4 + (i < n4 ? i : n4 - 1));
      w[j] = i < n4 ? t : v4u{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < kHistUnroll; ++j) {
      if ((w[j].x | w[j].y | w[j].z | w[j].w) == 0u) continue;
      hist_add(h, w[j].x);
      hist_add(h, w[j].y);
      hist_add(h, w[j].z);
      hist_add(h, w[j].w);
    }
  }
  if (blockIdx.x == 0)  // the nvox % 4 tail
    for (int64_t i = (n4 << 2) + tid; i < nvox; i += kBlock) hist_add(h, grid[i]);
  __syncthreads();
  for (int i = tid; i < 768; i += kBlock) {
    uint32_t s = 0;
#pragma unroll
    for (int w = 0; w < kHistWaves; ++w) s += s_h[w * 768 + i];
    if (s) atomicAdd(&out[i], (unsigned long long)s);
  }
}

}  // namespace

hipError_t launch_colour_hist(const uint32_t* grid, int64_t nvox, unsigned long long* out, hipStream_t s) {
  if (nvox <= 0) return hipSuccess;
  int dev = 0, ncu = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t chunks = ((nvox >> 2) + kBlock * kHistUnroll - 1) / (kBlock * kHistUnroll);
  const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(chunks, (int64_t)ncu * 4));
  colour_hist_kernel<<<g, kBlock, 0, s>>>(grid, nvox, out);
  return hipGetLastError();
}

}  // namespace c3h
