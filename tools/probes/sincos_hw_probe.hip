// Probe: accuracy of the hardware v_sin_f32 / v_cos_f32 (input in revolutions) for the f32 wide kernel's phasors,
// against the float64 sin/cos of the same angle, and of the current steering_coeff_fast path.  The argument is
// reduced in float64 first (u = rot / 2pi - rint(rot / 2pi), |u| <= 1/2), rounded once to float32.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/sincos_hw_probe.hip -o build/sincos_hw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__device__ __forceinline__ unsigned long long mix(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ void probe(unsigned long long n, double* out) {
  double emax_hw = 0, emax_hw_red = 0, esum = 0;
  for (unsigned long long i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    // steering phases |rot| up to ~2e3 rad (delays up to hundreds of samples)
    const double rot = (static_cast<double>(mix(i) >> 11) * 0x1p-53 - 0.5) * 4000.0;
    const double u64 = rot * 0.15915494309189535;
    const double ur = u64 - rint(u64);
    const float u = static_cast<float>(ur);
    const float s = __builtin_amdgcn_sinf(u), c = __builtin_amdgcn_cosf(u);
    const double se = sin(rot), ce = cos(rot);
    const double e = fmax(fabs(s - se), fabs(c - ce));
    // the same hardware instructions on the exactly reduced float32 angle (excludes the argument rounding)
    const double se2 = sin(6.283185307179586 * static_cast<double>(u)), ce2 = cos(6.283185307179586 * static_cast<double>(u));
    const double e2 = fmax(fabs(s - se2), fabs(c - ce2));
    emax_hw = fmax(emax_hw, e);
    emax_hw_red = fmax(emax_hw_red, e2);
    esum += e;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    emax_hw = fmax(emax_hw, __shfl_xor(emax_hw, o));
    emax_hw_red = fmax(emax_hw_red, __shfl_xor(emax_hw_red, o));
    esum += __shfl_xor(esum, o);
  }
  if ((threadIdx.x & 63) == 0) {
    const unsigned w = blockIdx.x * 4 + threadIdx.x / 64;
    out[3 * w] = emax_hw;
    out[3 * w + 1] = emax_hw_red;
    out[3 * w + 2] = esum;
  }
}

int main() {
  const int grid = 1024;
  const unsigned long long n = 1ull << 28;
  double* d;
  hipMalloc(&d, grid * 4 * 3 * sizeof(double));
  hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, n, d);
  static double h[1024 * 4 * 3];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  double m1 = 0, m2 = 0, sum = 0;
  for (int w = 0; w < grid * 4; ++w) {
    m1 = fmax(m1, h[3 * w]);
    m2 = fmax(m2, h[3 * w + 1]);
    sum += h[3 * w + 2];
  }
  printf("v_sin/v_cos_f32 on float64-reduced revolutions, %llu angles |rot| < 2000 rad:\n", n);
  printf("  max |err| vs float64 sin/cos(rot): %.3e (= %.2f x 2^-24); mean %.3e\n", m1, m1 / 0x1p-24, sum / n);
  printf("  max |err| of the instruction alone (vs sin/cos(2 pi u_f32)): %.3e (= %.2f x 2^-24)\n", m2, m2 / 0x1p-24);
  return 0;
}
