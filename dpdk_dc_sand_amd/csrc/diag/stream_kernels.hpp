// The HBM stream-ceiling kernels: plain streams over a read/write byte mix, the achievable ceiling a fused kernel's
// traffic is compared with.  Included by the diagnostic build (fused_diag.inc) and by the small measurement library
// bench.py loads for its `ceiling` blocks (tools/stream_ceiling.hip -> build/libbf_stream.so).  Not product code.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace bf {
namespace stream {
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Streams in_bytes in and out_bytes out with 16-byte lanes, `unroll` loads in flight per lane before the stores:
// the achievable HBM ceiling for the fused kernel's traffic mix.
template <int U, bool NtLoad = false, bool NtStore = false>
__global__ __launch_bounds__(256) void stream_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n_in,
                                                     size_t n_out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t n = n_in > n_out ? n_in : n_out;
  for (size_t i0 = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i0 < n; i0 += stride * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + u * stride;
      if (i < n_in) {
        if constexpr (NtLoad) {
          const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + i));
          v[u] = make_uint4(t[0], t[1], t[2], t[3]);
        } else {
          v[u] = in[i];
        }
      } else {
        v[u] = make_uint4(static_cast<uint32_t>(i), 1, 2, 3);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + u * stride;
      if (i < n_out) {
        if constexpr (NtStore) {
          __builtin_nontemporal_store(u32x4{v[u].x, v[u].y, v[u].z, v[u].w}, reinterpret_cast<u32x4*>(out + i));
        } else {
          out[i] = v[u];
        }
      }
    }
  }
}
// The int8 path's traffic mix as a stream: 4 bytes read per byte written, uniformly over time (out[i] = xor of
// four in-streams), non-temporal loads (and stores when NtStore).
template <bool NtStore>
__global__ __launch_bounds__(256) void stream_mix_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                         size_t n_out) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n_out; i += stride) {
    u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + i));
#pragma unroll
    for (int u = 1; u < 4; ++u) a ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + i + u * n_out));
    if constexpr (NtStore)
      __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(out + i));
    else
      *reinterpret_cast<u32x4*>(out + i) = a;
  }
}
}  // namespace stream
}  // namespace bf
