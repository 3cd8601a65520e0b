// Host probe for the integer path's fast Q14 phasor (bf_phase.hpp q14_fast): float64 rotation without divisions,
// Cody-Waite reduction, truncated fdlibm cos/sin kernels in float64.  Measures
// max |fast - cos(rot_exact)| (rot_exact = steering_rotation's reference-order float64 phase, libm cos/sin), and
// checks the decision rule: a = RN32(v - eps), b = RN32(v + eps); unflagged iff rint(2^14 a) == rint(2^14 b),
// which must then equal rint(2^14 RN32(cos(rot_exact))).
//   gcc -O2 -o /tmp/q14 tools/probes/q14_fast_check.c -lm && /tmp/q14 [n]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static double urand(void) {  // xorshift64*, [0, 1)
  s_state ^= s_state >> 12; s_state ^= s_state << 25; s_state ^= s_state >> 27;
  return (double)((s_state * 2685821657736338717ull) >> 11) * 0x1p-53;
}

#pragma STDC FP_CONTRACT OFF
static double rot_exact(float tau_f, float rate_f, float phi_f, float prate_f, double ch, double ctot, double ts,
                        double dt) {
  double tau = tau_f, phi = phi_f;
  if (dt != 0.0) { tau = tau + (double)rate_f * dt; phi = phi + (double)prate_f * dt; }
  const double npi = -3.141592653589793, denom = ctot * ts;
  const double initial = (tau * ch * npi) / denom + phi;
  const double centre = (tau * (ctot / 2.0) * npi) / denom;
  return initial - centre;
}

// the fast phasor, returning float64 cos/sin approximations (the device code's operation order): float64 rotation
// without divisions, two-term Cody-Waite reduction, truncated fdlibm kernels (sin: S1..S5, cos: C1..C5) in plain
// float64 Horner form (bf_phase.hpp q14_fast)
static void fast_phasor(float tau_f, float rate_f, float phi_f, float prate_f, double chc, double k, double dt,
                        double* c, double* s) {
  const double tau = fma((double)rate_f, dt, (double)tau_f), phi = fma((double)prate_f, dt, (double)phi_f);
  const double rot = fma(tau * chc, k, phi);
  const double n = rint(rot * 0.63661977236758138);
  double r = fma(-n, 1.5707963267948966e+00, rot);
  r = fma(-n, 6.123233995736766e-17, r);
  const double z = r * r;
  const double cz = fma(z, fma(z, fma(z, fma(z, fma(z, fma(z, 2.08757232129817482790e-09, -2.75573143513906633035e-07),
                                                    2.48015872894767294178e-05), -1.38888888888741095749e-03),
                                      4.16666666666666019037e-02), -0.5), 1.0);
  const double sp = fma(z, fma(z, fma(z, fma(z, -2.50507602534068634195e-08, 2.75573137070700676789e-06),
                                      -1.98412698298579493134e-04), 8.33333333332248946124e-03),
                        -1.66666666666666324348e-01);
  const double sz = fma(r * z, sp, r);
  const int q = (int)n & 3;
  const double s0 = (q & 1) ? cz : sz, c0 = (q & 1) ? sz : cz;
  *c = ((q + 1) & 2) ? -c0 : c0;
  *s = (q & 2) ? -s0 : s0;
}

static int q14(float v) { return (int)rintf(v * 16384.0f); }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  const double Ts = 1.0 / 1712e6, eps = 5e-10;
  double maxerr = 0.0;
  long flagged = 0, wrong = 0, big = 0;
  for (long i = 0; i < n; ++i) {
    const double ctot = (i & 1) ? 32768.0 : 4096.0;
    const float tau = (float)(urand() * 10 * Ts * ((i & 6) == 6 ? 100.0 : 1.0));
    const float rate = (float)((urand() * 2 - 1) * 1e-9), phi = (float)((urand() * 2 - 1) * M_PI);
    const float prate = (float)(urand() * 2 - 1);
    const double ch = floor(urand() * ctot), dt = (i & 8) ? urand() * 1e-2 : 0.0;
    const double rex = rot_exact(tau, rate, phi, prate, ch, ctot, Ts, dt);
    double c, s;
    fast_phasor(tau, rate, phi, prate, ch - ctot / 2.0, -3.141592653589793 / (ctot * Ts), dt, &c, &s);
    const double ce = cos(rex), se = sin(rex);
    const double e = fmax(fabs(c - ce), fabs(s - se));
    if (e > maxerr) maxerr = e;
    if (e > eps) ++big;
    const double v[2] = {c, s}, ex[2] = {ce, se};
    for (int j = 0; j < 2; ++j) {
      const int qa = q14((float)(v[j] - eps)), qb = q14((float)(v[j] + eps));
      if (qa != qb) { ++flagged; continue; }
      if (qa != q14((float)ex[j])) ++wrong;
    }
  }
  printf("n=%ld max|fast-exact|=%.3e (eps %.1e, %ld above) flagged %.3e per component, wrong unflagged %ld\n", n,
         maxerr, eps, big, (double)flagged / (2.0 * n), wrong);
  return wrong != 0 || big != 0;
}
