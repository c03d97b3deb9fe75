// Diagnostics: HBM read-stream rates for access shapes like c3_occupancy_kernel's
// (16-B loads, U loads in flight per lane, chunked grid-stride), on a 537 MB buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int U, bool NT>
__global__ __launch_bounds__(256) void rd(const uint4* __restrict__ g, int64_t n4, uint32_t* out) {
  uint32_t acc = 0;
  const int64_t chunk = 256 * U;
  for (int64_t c0 = blockIdx.x * chunk; c0 < n4; c0 += (int64_t)gridDim.x * chunk) {
    uint4 w[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int64_t i = c0 + j * 256 + threadIdx.x;
      typedef unsigned int v4u __attribute__((ext_vector_type(4)));
      if (NT) {
        v4u t = i < n4 ? __builtin_nontemporal_load(reinterpret_cast<const v4u*>(g) + i) : v4u{0, 0, 0, 0};
        w[j] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        w[j] = i < n4 ? g[i] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) acc |= w[j].x | w[j].y | w[j].z | w[j].w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int U, bool NT>
float run(const uint4* g, int64_t n4, uint32_t* out, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) rd<U, NT><<<grid, 256>>>(g, n4, out);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) rd<U, NT><<<grid, 256>>>(g, n4, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const int64_t bytes = 8ll * 67108864;  // 8 frames of 256^3 x 4 B
  uint4* g;
  uint32_t* out;
  if (hipMalloc(&g, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(g, 0, bytes);
  const int64_t n4 = bytes / 16;
  const int grids[] = {256, 512, 1024, 2048, 4096, 8192};
  for (int grid : grids) {
    printf("grid %5d  U16 %.2f TB/s  U8 %.2f  U4 %.2f  U16nt %.2f  U8nt %.2f\n", grid,
           bytes / run<16, false>(g, n4, out, grid) / 1e9, bytes / run<8, false>(g, n4, out, grid) / 1e9,
           bytes / run<4, false>(g, n4, out, grid) / 1e9, bytes / run<16, true>(g, n4, out, grid) / 1e9,
           bytes / run<8, true>(g, n4, out, grid) / 1e9);
  }
  return 0;
}
