// Steering-phase evaluation shared by the coefficient generators and the fused beamformer.
#pragma once

#include <hip/hip_runtime.h>

namespace bf {

// Per-launch constants of the exact phase: denom = Ctot*Ts (one rounding, as n_channels * sample_period on the
// host), its correctly rounded reciprocal, and Ctot/2.  Built once per thread; all inputs are uniform.
struct PhaseK {
  double half_ctot, denom, inv;
};

__device__ __forceinline__ PhaseK make_phase(double ctot, double ts) {
  PhaseK k;
  k.half_ctot = ctot / 2.0;
  k.denom = ctot * ts;
  k.inv = 1.0 / k.denom;
  return k;
}

// a / denom, correctly rounded, without a division: q0 = RN(a * RN(1/denom)) is within an ulp, the residual
// fma(-q0, denom, a) is exact, and one Markstein step fma(r, inv, q0) rounds to RN(a / denom) (0 differences
// in 2.8e8 steering quotients, tools/probes/div_check.c).  r == 0 means q0 is exact: keep it (and its sign of 0).
__device__ __forceinline__ double div_denom(double a, const PhaseK& k) {
  const double q0 = a * k.inv;
  const double r = fma(-q0, k.denom, a);
  return r == 0.0 ? q0 : fma(r, k.inv, q0);
}

// rot = tau*ch*(-pi)/(Ctot*Ts) + phi - tau*(Ctot/2)*(-pi)/(Ctot*Ts), in float64 and in the reference's
// left-to-right order (unit_test/coeff_generator_cpu.py:145-164, beamforming/coeff_generator.py:55-65; numpy 1.x
// promotes every step to float64).  FMA contraction is disabled so every step rounds exactly like the host.
// Time extension: tau += tau_rate*dt and phi += phi_rate*dt first; at dt == 0 the
// result is bit-identical to the reference.
__device__ __forceinline__ double steering_rotation(float4 dv, double ch, const PhaseK& k, double dt) {
#pragma clang fp contract(off)
  double tau = static_cast<double>(dv.x);
  double phi = static_cast<double>(dv.z);
  if (dt != 0.0) {
    tau = tau + static_cast<double>(dv.y) * dt;
    phi = phi + static_cast<double>(dv.w) * dt;
  }
  const double neg_pi = -3.141592653589793;  // -np.math.pi
  const double initial = div_denom(tau * ch * neg_pi, k) + phi;
  const double centre = div_denom(tau * k.half_ctot * neg_pi, k);
  return initial - centre;
}

// float64 sin and cos for |x| < ~1e5: Cody-Waite reduction by pi/2 (three-part constant, fma) and the fdlibm
// minimax kernels on [-pi/4, pi/4].  Within 1 ulp of libm; the float32 roundings of cos and sin matched libm's
// on all 7e7 probe arguments (tools/probes/sincos_check.c), at about a fifth of the generic sincos' cost (no
// Payne-Hanek path, no double-double reduction).  Steering phases are |rot| < ~1e3.
__device__ __forceinline__ void sincos_pio2(double x, double* s, double* c) {
#pragma clang fp contract(off)
  const double n = rint(x * 0.63661977236758138);  // 2 / pi
  double r = fma(-n, 1.5707963267948966e+00, x);
  r = fma(-n, 6.123233995736766e-17, r);
  r = fma(-n, -1.4973849048591698e-33, r);
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                      2.75573137070700676789e-06), -1.98412698298579493134e-04),
                        8.33333333332248946124e-03);
  const double sn = fma(r * z, fma(z, ps, -1.66666666666666324348e-01), r);
  const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                  -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                    -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cs = w + (((1.0 - w) - hz) + z * pc);
  const int q = static_cast<int>(static_cast<long long>(n) & 3);
  const double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}

// cos/sin in float64 (libm semantics, as math.cos / math.sin on the host), rounded to float32 on store.
__device__ __forceinline__ void steering_coeff(float4 dv, double ch, const PhaseK& k, double dt, float* re,
                                               float* im) {
  const double rot = steering_rotation(dv, ch, k, dt);
  double s, c;
  sincos_pio2(rot, &s, &c);
  *re = static_cast<float>(c);
  *im = static_cast<float>(s);
}

// Fast steering phasor (fused kernels' default): rot = phi' + tau' * (ch - Ctot/2) * K with K = -pi/(Ctot*Ts)
// precomputed on the host, in float64 (no divisions); reduced by pi/2 in float64 (Cody-Waite, two terms); then
// float32 minimax polynomials (Cephes sinf/cosf coefficients) on the reduced angle rf in [-pi/4, pi/4], a
// first-order correction for rf's float32 rounding dr = r - rf, and the quadrant swap.  <= 1.32 ulp of float32 (mean
// |error| 2e-8) against the exact phasor over 2e7 probe angles (tools/probes/sincosf_check.c), about a third of the
// instructions of the generic sincosf (which redoes a general range reduction).
__device__ __forceinline__ void steering_coeff_fast(float4 dv, double chc, double k, double dt, float* re, float* im) {
  double tau = static_cast<double>(dv.x);
  double phi = static_cast<double>(dv.z);
  if (dt != 0.0) {
    tau = fma(static_cast<double>(dv.y), dt, tau);
    phi = fma(static_cast<double>(dv.w), dt, phi);
  }
  const double rot = fma(tau * chc, k, phi);
  const double n = rint(rot * 0.63661977236758138);  // 2 / pi
  double r = fma(-n, 1.5707963267948966e+00, rot);
  r = fma(-n, 6.123233995736766e-17, r);
  const float rf = static_cast<float>(r);
  const float dr = static_cast<float>(r - static_cast<double>(rf));
  const float z = rf * rf;
  const float ps = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * rf, rf);
  const float pc = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f),
                             z * z, -0.5f * z), 1.0f, 1.0f);
  const float s1 = fmaf(pc, dr, ps), c1 = fmaf(-ps, dr, pc);  // sin, cos of r = rf + dr
  const int q = static_cast<int>(static_cast<long long>(n) & 3);
  const float s0 = (q & 1) ? c1 : s1, c0 = (q & 1) ? s1 : c1;
  *re = ((q + 1) & 2) ? -c0 : c0;
  *im = (q & 2) ? -s0 : s0;
}

}  // namespace bf
