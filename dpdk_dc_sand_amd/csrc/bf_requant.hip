// 8-bit requantiser: q = clamp(rne(y * scale), -127, 127).  The reference has no requantiser;
// this is the contract the fused beamformer's int8 output also follows (oracle.requantise).
#include "bf_common.hpp"

namespace bf {

__device__ __forceinline__ int8_t requant1(float v, float scale) {
  float r = __builtin_rintf(v * scale);
  r = fminf(fmaxf(r, -127.0f), 127.0f);
  return static_cast<int8_t>(static_cast<int>(r));
}

__global__ __launch_bounds__(256) void requant_kernel(const float* __restrict__ y, int8_t* __restrict__ q, size_t n,
                                                      float scale) {
  const size_t n4 = n / 4;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(y)[i];
    char4 o;
    o.x = requant1(v.x, scale);
    o.y = requant1(v.y, scale);
    o.z = requant1(v.z, scale);
    o.w = requant1(v.w, scale);
    reinterpret_cast<char4*>(q)[i] = o;
  }
  if (blockIdx.x == 0) {
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) q[i] = requant1(y[i], scale);
  }
}

}  // namespace bf

extern "C" int bf_requant(const float* y, int8_t* q, size_t n, float scale, void* stream) {
  BF_REQUIRE(y && q, "bf_requant: null pointer");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(y) & 15) == 0 && (reinterpret_cast<uintptr_t>(q) & 3) == 0,
             "bf_requant: misaligned buffer");
  if (n == 0) return BF_OK;
  size_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(bf::requant_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, bf::as_stream(stream),
                     y, q, n, scale);
  BF_LAUNCHED("requant_kernel");
}
