// Probe: does an LDS-DMA (buffer_load_dwordx4 ... lds via the builtin) land at LDS byte offsets above 64 KiB on
// gfx950?  One workgroup with a 128 KiB LDS array DMAs 1 KiB pieces of a known pattern to offsets 0, 60, 64, 80 and
// 120 KiB and copies the whole array back; the host checks every piece landed where it was sent and nowhere else.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __attribute__((address_space(3))) void* lds_void_ptr;
__shared__ __attribute__((aligned(16))) int4 big[128 * 1024 / 16];

__global__ __launch_bounds__(64) void probe(const int* src, int* out) {
  const int lane = threadIdx.x;
  for (int i = lane; i < 128 * 1024 / 16; i += 64) big[i] = int4{-1, -1, -1, -1};
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
  const int offs_kib[5] = {0, 60, 64, 80, 120};
  for (int p = 0; p < 5; ++p)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_ptr)(big + offs_kib[p] * 64), 16, 16 * lane, 1024 * p, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = lane; i < 128 * 1024 / 16; i += 64) reinterpret_cast<int4*>(out)[i] = big[i];
}

int main() {
  std::vector<int> h(5 * 256);
  for (int i = 0; i < 5 * 256; ++i) h[i] = 1000000 * (i / 256 + 1) + i % 256;
  int *d, *o;
  hipMalloc(&d, h.size() * 4);
  hipMalloc(&o, 128 * 1024);
  hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
  std::vector<int> r(32 * 1024);
  hipMemcpy(r.data(), o, 128 * 1024, hipMemcpyDeviceToHost);
  const int offs[5] = {0, 60, 64, 80, 120};
  int bad = 0, stray = 0;
  std::vector<char> expect(128, 0);
  for (int p = 0; p < 5; ++p) {
    expect[offs[p]] = 1;
    for (int w = 0; w < 256; ++w)
      if (r[offs[p] * 256 + w] != h[p * 256 + w]) ++bad;
  }
  for (int k = 0; k < 128; ++k)
    if (!expect[k])
      for (int w = 0; w < 256; ++w)
        if (r[k * 256 + w] != -1) ++stray;
  printf("lds_dma_high: %d wrong words in the 5 pieces, %d words changed elsewhere -> %s\n", bad, stray,
         bad == 0 && stray == 0 ? "LDS-DMA reaches offsets >= 64 KiB" : "FAIL");
  return bad || stray;
}
