// The box's HBM stream ceiling as a small stand-alone library (build/libbf_stream.so, `make stream`): bench.py's
// `ceiling` blocks time the fused kernels' read/write byte mix through these plain streams, so the bench no longer
// needs the whole diagnostic build (build/libbf_diag.so) on the GPU box.  Measurement only, never the product.
#include "../dpdk_dc_sand_amd/csrc/diag/stream_kernels.hpp"

// code: 1 plain 16-byte loads/stores, 101 non-temporal stores, 102 non-temporal loads, 103 both (grid-stride over
// max(in, out) pieces); 200 / 201 the 4:1 read:write mix (out_bytes = in_bytes / 4) with / without non-temporal
// stores.  Returns the hipError_t of the launch (0 = launched).
extern "C" int bf_stream_ceiling(const void* in, void* out, size_t in_bytes, size_t out_bytes, int grid, int code,
                                 void* stream) {
  auto in4 = reinterpret_cast<const uint4*>(in);
  auto out4 = reinterpret_cast<uint4*>(out);
  auto st = reinterpret_cast<hipStream_t>(stream);
  using namespace bf::stream;
  switch (code) {
    case 1:
      hipLaunchKernelGGL((stream_kernel<1, false, false>), dim3(grid), dim3(256), 0, st, in4, out4, in_bytes / 16,
                         out_bytes / 16);
      break;
    case 101:
      hipLaunchKernelGGL((stream_kernel<1, false, true>), dim3(grid), dim3(256), 0, st, in4, out4, in_bytes / 16,
                         out_bytes / 16);
      break;
    case 102:
      hipLaunchKernelGGL((stream_kernel<1, true, false>), dim3(grid), dim3(256), 0, st, in4, out4, in_bytes / 16,
                         out_bytes / 16);
      break;
    case 103:
      hipLaunchKernelGGL((stream_kernel<1, true, true>), dim3(grid), dim3(256), 0, st, in4, out4, in_bytes / 16,
                         out_bytes / 16);
      break;
    case 200:
    case 201:
      if (out_bytes * 4 != in_bytes) return static_cast<int>(hipErrorInvalidValue);
      if (code == 200)
        hipLaunchKernelGGL((stream_mix_kernel<true>), dim3(grid), dim3(256), 0, st, in4, out4, out_bytes / 16);
      else
        hipLaunchKernelGGL((stream_mix_kernel<false>), dim3(grid), dim3(256), 0, st, in4, out4, out_bytes / 16);
      break;
    default:
      return static_cast<int>(hipErrorInvalidValue);
  }
  return static_cast<int>(hipGetLastError());
}
