// diagnostics: throughput of 64-bit global atomics on MI355X, the voxelisers' flush pattern
// (entries spread over a large toroidal table, 3 atomics per entry: two adds + a min).
// Device scope (agent) vs L2-local (workgroup scope on an XCD-private copy of the table,
// indexed by the executing XCD's id), non-returning.  Build: hipcc --offload-arch=gfx950 -O3
// tools/atomic_bench.hip -o tools/atomic_bench  (run on the GPU box; prints one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                             \
    }                                                                       \
  } while (0)

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
  return v & 7u;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// mode 0: agent scope on one table; mode 1: workgroup scope on the XCD's own copy;
// mode 2: agent scope, the sums and the owner word interleaved in one 32-B record per cell
// (one line per entry instead of two)
template <int kMode>
__global__ __launch_bounds__(256) void flush_kernel(unsigned long long* acc, unsigned long long* mo, uint32_t mask,
                                                    size_t copy_stride, int entries_per_thread, uint32_t seed) {
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  size_t base = 0;
  if (kMode == 1) base = (size_t)xcc_id() * copy_stride;
  for (int k = 0; k < entries_per_thread; ++k) {
    const uint32_t t = mix(g * 977u + k * 131071u + seed) & mask;
    unsigned long long* a = acc + base + 2 * (size_t)t;
    unsigned long long* m = mo + base / 2 + t;
    if (kMode == 2) {
      unsigned long long* r = acc + 4 * (size_t)t;
      __hip_atomic_fetch_add(r, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(r + 1, 3ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_min(r + 2, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (kMode == 0) {
      __hip_atomic_fetch_add(a, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(a + 1, 3ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_min(m, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      __hip_atomic_fetch_add(a, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_add(a + 1, 3ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_min(m, (unsigned long long)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

// same-address returning adds: `per_block` lanes of every workgroup add 1 to one counter
// (the voxeliser's per-brick list index) and store what they got
__global__ __launch_bounds__(256) void same_addr_kernel(unsigned* ctr, unsigned* out, int per_block) {
  if ((int)threadIdx.x < per_block) out[blockIdx.x * per_block + threadIdx.x] = atomicAdd(ctr, 1u);
}

int main() {
  const int tb = 24;  // 2^24 cells: the 256^3 frame's toroidal table
  const size_t cells = (size_t)1 << tb;
  unsigned long long *acc, *mo;
  CHK(hipMalloc(&acc, 8 * cells * 2 * 8));  // 8 copies of {x, y}
  CHK(hipMalloc(&mo, 8 * cells * 8));
  CHK(hipMemset(acc, 0, 8 * cells * 2 * 8));
  CHK(hipMemset(mo, 0xff, 8 * cells * 8));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  printf("{");
  const int entries[] = {96 * 1024, 384 * 1024};
  bool first = true;
  for (int tbm : {24, 20, 17}) {  // table sizes: 384 MB, 24 MB, 3 MB (acc + owner words)
  const uint32_t mask = (1u << tbm) - 1;
  for (int ne : entries) {
    for (int mode = 0; mode < 3; ++mode) {
      const int ept = 4;
      const int blocks = (ne / ept + 255) / 256;
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        CHK(hipEventRecord(e0));
        if (mode == 0)
          flush_kernel<0><<<blocks, 256>>>(acc, mo, mask, cells * 2, ept, rep);
        else if (mode == 2)
          flush_kernel<2><<<blocks, 256>>>(acc, mo, mask, cells * 2, ept, rep);
        else
          flush_kernel<1><<<blocks, 256>>>(acc, mo, mask, cells * 2, ept, rep);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("%s\"tb%d_%s_%dk_us\": %.2f", first ? "" : ", ", tbm, mode == 2 ? "agent_32B_record" : (mode ? "l2_xcd_copy" : "agent"), ne / 1024, best * 1e3);
      first = false;
    }
  }
  }
  for (int blocks : {245, 490}) {
    for (int per : {12, 40}) {
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        CHK(hipMemset(mo, 0, 4));
        CHK(hipEventRecord(e0));
        same_addr_kernel<<<blocks, 256>>>(reinterpret_cast<unsigned*>(mo), reinterpret_cast<unsigned*>(acc), per);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf(", \"same_addr_%dx%d_us\": %.2f", blocks, per, best * 1e3);
    }
  }
  printf("}\n");
  CHK(hipFree(acc));
  CHK(hipFree(mo));
  return 0;
}
