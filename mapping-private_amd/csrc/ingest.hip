// ingest.hip -- sensor_msgs/PointCloud2 -> the c3h_voxelize point layout on the device
// (pcl::fromROSMsg(*msg, cloud) of color_voxel_recognition/test/detect_object.cpp:142 for
// pcl::PointXYZRGB: fields matched by name, every point of the height x width message
// kept, NaN points included -- limitPoint drops them afterwards).
#include "c3h_internal.h"

namespace c3h {

__device__ __forceinline__ uint32_t pc2_word(const uint8_t* __restrict__ p, int big) {
  const uint32_t b0 = p[0], b1 = p[1], b2 = p[2], b3 = p[3];
  return big ? (b0 << 24 | b1 << 16 | b2 << 8 | b3) : (b3 << 24 | b2 << 16 | b1 << 8 | b0);
}

// one point per thread; field bytes are read one by one (offsets / steps need not be
// 4-byte aligned), rgb absent (offset < 0) reads as 0
__global__ void pc2_convert_kernel(const uint8_t* __restrict__ data, uint32_t width, int64_t n,
                                   uint32_t point_step, uint32_t row_step, int4 off, int big,
                                   float4* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / width, col = i - row * width;
    const uint8_t* p = data + row * (int64_t)row_step + col * (int64_t)point_step;
    float4 v;
    v.x = __uint_as_float(pc2_word(p + off.x, big));
    v.y = __uint_as_float(pc2_word(p + off.y, big));
    v.z = __uint_as_float(pc2_word(p + off.z, big));
    v.w = __uint_as_float(off.w >= 0 ? pc2_word(p + off.w, big) : 0u);
    out[i] = v;
  }
}

hipError_t launch_pc2_convert(const void* data, uint32_t height, uint32_t width, uint32_t point_step,
                              uint32_t row_step, const int32_t off[4], int big, float* out, hipStream_t s) {
  const int64_t n = (int64_t)height * width;
  if (n == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 16384);
  pc2_convert_kernel<<<(unsigned)blocks, 256, 0, s>>>(static_cast<const uint8_t*>(data), width, n, point_step,
                                                       row_step, make_int4(off[0], off[1], off[2], off[3]), big,
                                                       reinterpret_cast<float4*>(out));
  return hipGetLastError();
}

}  // namespace c3h
