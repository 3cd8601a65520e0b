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

}  // namespace bf
