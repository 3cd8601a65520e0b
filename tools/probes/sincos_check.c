// Host probe for bf_phase.hpp sincos_pio2: float64 sin/cos by a three-part Cody-Waite reduction by pi/2 and the
// fdlibm minimax kernels, as the exact coefficient path evaluates them.  The coefficient contract stores
// RN32(cos(rot)) and RN32(sin(rot)) with libm's cos/sin (coeff_generator_cpu.py:166-186 via math.cos / math.sin).
// Counts arguments where the float32 roundings differ from libm's, and the largest float64 difference in ulps, over
// random steering phases |rot| < 1e3 (the range the kernels use) plus phases near multiples of pi/4.
// Exits 1 on any float32 difference.
//   gcc -O2 -ffp-contract=off -o /tmp/sc tools/probes/sincos_check.c -lm && /tmp/sc [n]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#pragma STDC FP_CONTRACT OFF

static uint64_t s_state = 0x9E3779B97F4A7C15ull;
static double urand(void) {  // xorshift64*, [0, 1)
  s_state ^= s_state >> 12; s_state ^= s_state << 25; s_state ^= s_state >> 27;
  return (double)((s_state * 2685821657736338717ull) >> 11) * 0x1p-53;
}

static void sincos_pio2(double x, double* s, double* c) {
  const double n = rint(x * 0.63661977236758138);
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
  const int q = (int)((long long)n & 3);
  const double s0 = (q & 1) ? cs : sn, c0 = (q & 1) ? sn : cs;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}

static double ulps(double a, double b) {  // |a - b| in units of b's ulp
  return a == b ? 0.0 : fabs(a - b) / (nextafter(fabs(b), INFINITY) - fabs(b));
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  long bad32 = 0;
  double maxulp = 0.0;
  for (long i = 0; i < n; ++i) {
    double x;
    if (i & 1)
      x = (urand() * 2 - 1) * ((i & 2) ? 1e3 : 40.0);
    else  // near k * pi/4, where the quadrant logic and the reduction are tested hardest
      x = floor((urand() * 2 - 1) * 1200.0) * 0.78539816339744830962 + (urand() * 2 - 1) * 1e-6;
    double s, c;
    sincos_pio2(x, &s, &c);
    const double se = sin(x), ce = cos(x);
    if ((float)s != (float)se || (float)c != (float)ce) {
      if (bad32 < 10) printf("float32 differs at x=%.17g: sin %.17g vs %.17g, cos %.17g vs %.17g\n", x, s, se, c, ce);
      ++bad32;
    }
    const double u = fmax(ulps(s, se), ulps(c, ce));
    if (u > maxulp) maxulp = u;
  }
  printf("n=%ld arguments, float32 roundings differing from libm: %ld, max float64 difference %.2f ulp\n", n, bad32,
         maxulp);
  return bad32 ? 1 : 0;
}
