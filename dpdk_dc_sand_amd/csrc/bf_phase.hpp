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
// Returns the float64 rotation (callers that need a validity range check it).
__device__ __forceinline__ double steering_coeff_fast(float4 dv, double chc, double k, double dt, float* re,
                                                      float* im) {
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
  // quadrant by one saturating v_cvt_i32_f64 (the 64-bit conversion costs four float64 instructions); exact for
  // |n| < 2^31, i.e. |rot| < 3.4e9 rad, far beyond where a float64 rotation still carries phase information
  const int q = __double2int_rn(n) & 3;
  const float s0 = (q & 1) ? c1 : s1, c0 = (q & 1) ? s1 : c1;
  *re = ((q + 1) & 2) ? -c0 : c0;
  *im = (q & 2) ? -s0 : s0;
  return rot;
}

// Hardware phasor (measurement): the float64 rotation reduced to revolutions in float64 (u = rot / 2 pi - rint(.),
// |u| <= 1/2), rounded once to float32, then v_sin_f32 / v_cos_f32 (which take revolutions).  The argument rounding
// is <= 2^-26 rev (~2^-23.3 in the phasor); the instructions' own error is measured by
// tools/probes/sincos_hw_probe.hip.
__device__ __forceinline__ void steering_coeff_hw(float4 dv, double chc, double k, double dt, float* re, float* im) {
  const double tau = fma(static_cast<double>(dv.y), dt, static_cast<double>(dv.x));
  const double phi = fma(static_cast<double>(dv.w), dt, static_cast<double>(dv.z));
  const double u = fma(tau * chc, k, phi) * 0.15915494309189535;  // 1 / (2 pi)
  const float uf = static_cast<float>(u - rint(u));
  *re = __builtin_amdgcn_cosf(uf);
  *im = __builtin_amdgcn_sinf(uf);
}

// ---- Q14 phasors of the integer (int8-beam) path ----------------------------------------------------------------
// Contract (oracle fused_beamform_int8): W = (rint(2^14 re), rint(2^14 im)) of the EXACT phasor (steering_coeff,
// then the optional gain), ties to even.  q14_fast evaluates cos/sin of the reduced angle to ~1e-11 instead:
// float64 rotation without divisions, two-term Cody-Waite reduction, the fdlibm kernels truncated to five terms
// in plain float64 Horner form (float64 FMA issues at the float32 rate on CDNA4, so no float32 tails and no
// conversions), |v - cos(rot_exact)| <= 7.5e-12 (tools/probes/q14_fast_check.c: 2e7 arguments, delays up to 2e5
// samples) < kQ14Eps.  The exact float32 phasor component is then RN32(v -+ eps) -- one of two adjacent floats --
// and when both give the same Q14 value (after the gain, as the contract applies it) that value IS the contract's.
// Both Q14 decisions are taken on cos r and sin r of the reduced angle; the quadrant swap and signs are applied to
// the integers afterwards (Q(-v) = -Q(v): RN32, the gain product and rint are all odd).  Otherwise (1.6e-5 of the
// components), or for a NaN / out-of-range argument, q14_fast returns false and the caller re-evaluates that
// coefficient exactly: bit-exact at little more than the cost of a float32 phasor.
constexpr double kQ14Eps = 5e-10;
constexpr float kQ14MaxMag = 2e5f;  // |tau'| (ch + Ctot/2) |K| + |phi'| bound of the error analysis above

// gq = gain * 2^14 (2^14 without gains): RN32(a * g) * 2^14 == RN32(a * gq) (a power-of-two scale commutes with
// rounding), so the contract's gain product and the Q14 scaling are one multiply.
__device__ __forceinline__ int q14_pair(double v, float gq, bool* ok) {
  const float a = static_cast<float>(v - kQ14Eps), b = static_cast<float>(v + kQ14Eps);
  const float qa = __builtin_rintf(__fmul_rn(a, gq)), qb = __builtin_rintf(__fmul_rn(b, gq));
  *ok = *ok && qa == qb;
  return static_cast<int>(qa);
}

// Unit gain: Q = rint(2^14 * RN32(v)).  The Q14 boundaries (2k + 1) / 2^15 are float32 numbers, so RN32 keeps v on
// its side of every boundary unless v lies within half a float32 ulp (<= 2^-24 for |v| <= 1) of it: with t = 2^14 v,
// Q = rint(t) whenever |t - rint(t)| < 1/2 - 2^14 (eps + 2^-24) (4 float64 operations).  Only the ~0.2 % of values
// nearer a boundary take q14_pair's two-sided test (which still decides almost all of them: Q(RN32(v -+ eps)) agree).
constexpr double kQ14UnitMargin = 0.5 - 16384.0 * (kQ14Eps + 0x1p-24);
__device__ __forceinline__ int q14_pair_unit(double v, bool* ok) {
  const double t = v * 16384.0;
  const double n = rint(t);
  if (fabs(t - n) < kQ14UnitMargin) return static_cast<int>(n);
  return q14_pair(v, 16384.0f, ok);
}

// q14_pair_unit on t = 2^14 v given directly (a recurrence kept in the 2^14-scaled domain: no rescale per value).
// (A float32 first test -- RN32(t) within 2^-10 of t -- measured slower, 74.5 vs 62 us for the config-4 generator:
// the ~0.4 % of values it leaves undecided put ~1 in 4 waves through both tests, profiles/r4_m_*.)
__device__ __forceinline__ int q14_pair_unit_scaled(double t, bool* ok) {
  const double n = rint(t);
  if (fabs(t - n) < kQ14UnitMargin) return static_cast<int>(n);
  return q14_pair(t * 0x1p-14, 16384.0f, ok);
}

// The truncated fdlibm coefficients (cos C5..C1, -1/2; sin S5..S1) as device memory, not literals: loaded once into
// SGRPs by s_load, each Horner step is then one VOP3 v_fma_f64 with an SGPR operand, where literal constants made
// the compiler rematerialise every addend with two v_mov_b32 per step (21 of ~96 VALU per phasor).
__constant__ double kQ14Poly[11] = {2.08757232129817482790e-09,  -2.75573143513906633035e-07, 2.48015872894767294178e-05,
                                    -1.38888888888741095749e-03, 4.16666666666666019037e-02,  -2.50507602534068634195e-08,
                                    2.75573137070700676789e-06,  -1.98412698298579493134e-04, 8.33333333332248946124e-03,
                                    -1.66666666666666324348e-01, 0.63661977236758138};

// uk = (ch + Ctot/2) * |K| (uniform per item), for the range check.  The rates are applied unconditionally: at
// dt == 0 they add exact zeros (a non-finite rate makes the range check fail, and the exact path ignores rates).
__device__ __forceinline__ bool q14_fast(float4 dv, double chc, double k, double dt, float uk, float gq, int* wc,
                                         int* ws) {
  const double tau = fma(static_cast<double>(dv.y), dt, static_cast<double>(dv.x));
  const double phi = fma(static_cast<double>(dv.w), dt, static_cast<double>(dv.z));
  const double* c = kQ14Poly;
  const double rot = fma(tau * chc, k, phi);
  const double n = rint(rot * c[10]);  // 2 / pi
  double r = fma(-n, 1.5707963267948966e+00, rot);
  r = fma(-n, 6.123233995736766e-17, r);
  const double z = r * r;
  const double cz = fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, c[0], c[1]), c[2]), c[3]), c[4]), -0.5), 1.0);
  const double sz = fma(r * z, fma(z, fma(z, fma(z, fma(z, c[5], c[6]), c[7]), c[8]), c[9]), r);
  const float mag = fabsf(static_cast<float>(tau)) * uk + fabsf(static_cast<float>(phi));
  bool ok = mag < kQ14MaxMag;  // false for NaN too
  const int qc = q14_pair(cz, gq, &ok), qs = q14_pair(sz, gq, &ok);
  const int q = __double2int_rn(n) & 3;  // saturating conversion; any garbage is flagged by the range check
  const int s0 = (q & 1) ? qc : qs, c0 = (q & 1) ? qs : qc;
  *wc = ((q + 1) & 2) ? -c0 : c0;
  *ws = (q & 2) ? -s0 : s0;
  return ok;
}

// The exact evaluation (the contract itself): float64 phase in the reference's order, float32 rounding, gain.
__device__ __forceinline__ void q14_exact(float4 dv, double ch, double ctot, double ts, double dt, const float* gain,
                                          float g, int* wc, int* ws) {
  float re, im;
  steering_coeff(dv, ch, make_phase(ctot, ts), dt, &re, &im);
  if (gain) {
    re = __fmul_rn(re, g);
    im = __fmul_rn(im, g);
  }
  *wc = static_cast<int>(__builtin_rintf(re * 16384.0f));
  *ws = static_cast<int>(__builtin_rintf(im * 16384.0f));
}

// N coefficients per lane: fast for all, then an exact pass per flagged coefficient (a wave runs as many exact
// passes as its most-flagged lane has flags: usually none).  valid[j] false -> W = 0.  FastFirst = false is the
// exact-only form (diagnostics / ablation).  Serial = true evaluates the N fast phasors one after another
// (a scheduling barrier between them): less instruction-level parallelism, but the float64 temporaries of only one
// phasor are live, which is what lets a kernel whose voltage loads are in flight meanwhile fit more waves.
// Branchless = true evaluates every fast phasor (invalid ones on their clamped, finite inputs) and zeroes the
// invalid results afterwards: no per-coefficient branch, so the N float64 Horner chains interleave (a lone wave per
// SIMD is otherwise latency-bound on them).
template <int N, bool FastFirst = true, bool Serial = false, bool Branchless = false>
__device__ __forceinline__ void q14_coeffs(const float4 (&dv)[N], const float (&g)[N], const bool (&valid)[N],
                                           double ch, double ctot, double ts, double k, double dt, const float* gain,
                                           int (&wc)[N], int (&ws)[N]) {
  const double chc = ch - ctot / 2.0;
  const float uk = static_cast<float>((ch + ctot / 2.0) * fabs(k));
  unsigned flagged = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    wc[j] = ws[j] = 0;
    if constexpr (Branchless && FastFirst) {
      int c, s;
      const bool ok = q14_fast(dv[j], chc, k, dt, uk, g[j] * 16384.0f, &c, &s);
      wc[j] = valid[j] ? c : 0;
      ws[j] = valid[j] ? s : 0;
      flagged |= (valid[j] && !ok) ? 1u << j : 0u;
      continue;
    }
    if (!valid[j]) continue;
    if constexpr (FastFirst) {
      if (!q14_fast(dv[j], chc, k, dt, uk, g[j] * 16384.0f, &wc[j], &ws[j])) flagged |= 1u << j;
    } else {
      flagged |= 1u << j;
    }
    if constexpr (Serial) __builtin_amdgcn_sched_barrier(0);
  }
  while (flagged) {
    const int j = __builtin_ctz(flagged);
    flagged &= flagged - 1;
    float4 d = dv[0];
    float gj = g[0];
#pragma unroll
    for (int jj = 1; jj < N; ++jj) {  // register selects (no dynamic indexing: that would go to scratch)
      const bool hit = j == jj;
      d.x = hit ? dv[jj].x : d.x;
      d.y = hit ? dv[jj].y : d.y;
      d.z = hit ? dv[jj].z : d.z;
      d.w = hit ? dv[jj].w : d.w;
      gj = hit ? g[jj] : gj;
    }
    int c, s;
    q14_exact(d, ch, ctot, ts, dt, gain, gj, &c, &s);
#pragma unroll
    for (int jj = 0; jj < N; ++jj) {
      wc[jj] = j == jj ? c : wc[jj];
      ws[jj] = j == jj ? s : ws[jj];
    }
  }
}

}  // namespace bf
