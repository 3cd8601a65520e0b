// Steering-phase evaluation shared by the coefficient generators and the fused beamformer.
#pragma once

#include <hip/hip_runtime.h>

namespace bf {

// rot = tau*ch*(-pi)/(Ctot*Ts) + phi - tau*(Ctot/2)*(-pi)/(Ctot*Ts), in float64 and in the reference's
// left-to-right order (unit_test/coeff_generator_cpu.py:145-164, beamforming/coeff_generator.py:55-65; numpy 1.x
// promotes every step to float64).  FMA contraction is disabled so every step rounds exactly like the host.
// Time extension: tau += tau_rate*dt and phi += phi_rate*dt first; at dt == 0 the
// result is bit-identical to the reference.
__device__ __forceinline__ double steering_rotation(float4 dv, double ch, double ctot, double ts, double dt) {
#pragma clang fp contract(off)
  double tau = static_cast<double>(dv.x);
  double phi = static_cast<double>(dv.z);
  if (dt != 0.0) {
    tau = tau + static_cast<double>(dv.y) * dt;
    phi = phi + static_cast<double>(dv.w) * dt;
  }
  const double neg_pi = -3.141592653589793;  // -np.math.pi
  const double denom = ctot * ts;            // n_channels * sample_period
  const double initial = tau * ch * neg_pi / denom + phi;
  const double centre = tau * (ctot / 2.0) * neg_pi / denom;
  return initial - centre;
}

// cos/sin in float64 (libm semantics, as math.cos / math.sin on the host), rounded to float32 on store.
__device__ __forceinline__ void steering_coeff(float4 dv, double ch, double ctot, double ts, double dt,
                                               float* re, float* im) {
  const double rot = steering_rotation(dv, ch, ctot, ts, dt);
  double s, c;
  sincos(rot, &s, &c);
  *re = static_cast<float>(c);
  *im = static_cast<float>(s);
}

// Fast steering phasor (fused kernels' default): rot = phi' + tau' * (ch - Ctot/2) * K with K = -pi/(Ctot*Ts)
// precomputed on the host, all in float64 (no divisions, no cancellation), reduced to [-pi, pi] in float64,
// then a float32 sincos of the reduced angle with a first-order correction for its float32 rounding:
// |error| ~ 1 ulp of float32 against the exact phasor (the exact mode above is bit-exact to the reference).
__device__ __forceinline__ void steering_coeff_fast(float4 dv, double chc, double k, double dt, float* re, float* im) {
  double tau = static_cast<double>(dv.x);
  double phi = static_cast<double>(dv.z);
  if (dt != 0.0) {
    tau = fma(static_cast<double>(dv.y), dt, tau);
    phi = fma(static_cast<double>(dv.w), dt, phi);
  }
  const double rot = fma(tau * chc, k, phi);
  const double n = rint(rot * 0.15915494309189535);     // 1 / (2 pi)
  double r = fma(-n, 6.283185307179586, rot);           // 2 pi (hi)
  r = fma(-n, 2.4492935982947064e-16, r);               // 2 pi (lo)
  const float rf = static_cast<float>(r);
  const float dr = static_cast<float>(r - static_cast<double>(rf));
  float s, c;
  sincosf(rf, &s, &c);
  *re = fmaf(-s, dr, c);
  *im = fmaf(c, dr, s);
}

}  // namespace bf
