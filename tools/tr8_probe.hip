// Probe of ds_read_b64_tr_b8 (gfx950) lane/byte semantics: LDS byte i holds i & 255; lane l
// supplies byte address A(l); prints each lane's 8 result bytes.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
typedef int v2i __attribute__((ext_vector_type(2)));
__global__ void k(const int* addr, uint32_t* out) {
  __shared__ uint8_t lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (uint8_t)i;
  __syncthreads();
  const int a = addr[threadIdx.x];
  v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((__attribute__((address_space(3))) v2i*)(lds + a));
  out[2 * threadIdx.x] = r.x;
  out[2 * threadIdx.x + 1] = r.y;
}
int main() {
  for (int mode = 0; mode < 2; ++mode) {
    int h[64];
    // mode 0: lane l -> bytes 8l; mode 1: lane l -> 16 (l >> 1) + 8 (l & 1) within the group,
    // groups at 128-byte steps (a 16-byte-record layout: lane 2q + p -> record q, half p)
    for (int l = 0; l < 64; ++l) h[l] = mode == 0 ? 8 * l : 128 * (l >> 4) + 16 * ((l & 15) >> 1) + 8 * (l & 1);
    int* da;
    uint32_t* dout;
    if (hipMalloc(&da, 256) || hipMalloc(&dout, 512)) return 1;
    if (hipMemcpy(da, h, 256, hipMemcpyHostToDevice)) return 1;
    k<<<1, 64>>>(da, dout);
    uint32_t o[128];
    if (hipMemcpy(o, dout, 512, hipMemcpyDeviceToHost)) return 1;
    printf("mode %d\n", mode);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d:", l);
      for (int b = 0; b < 8; ++b) printf(" %3u", (o[2 * l + b / 4] >> (8 * (b % 4))) & 0xffu);
      printf("\n");
    }
  }
  return 0;
}
