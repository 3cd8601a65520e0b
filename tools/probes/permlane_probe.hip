// Probe: lane semantics of v_permlane32_swap / v_permlane16_swap on gfx950 (prints src lane ids after the swap).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  auto a = __builtin_amdgcn_permlane32_swap(l, 100 + l, false, false);
  auto b = __builtin_amdgcn_permlane16_swap(l, 100 + l, false, false);
  out[l] = a[0]; out[64 + l] = a[1]; out[128 + l] = b[0]; out[192 + l] = b[1];
}
int main() {
  unsigned* d; hipMalloc(&d, 256 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[256]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[4] = {"p32[0]", "p32[1]", "p16[0]", "p16[1]"};
  for (int r = 0; r < 4; ++r) {
    printf("%s:", nm[r]);
    for (int g = 0; g < 4; ++g) printf(" rows%d:%u..%u", g, h[64 * r + 16 * g], h[64 * r + 16 * g + 15]);
    printf("\n");
  }
  return 0;
}
