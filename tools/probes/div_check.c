// Host probe for bf_phase.hpp div_denom: a / denom without a division, as the exact steering phase evaluates its two
// quotients by Ctot*Ts (coeff_generator_cpu.py:145-164 order).  q0 = RN(a * RN(1/denom)); r = fma(-q0, denom, a)
// (exact); q = r == 0 ? q0 : fma(r, inv, q0).  Counts the quotients where q differs from the IEEE division a / denom
// over random steering numerators (tau * ch * -pi and tau * (Ctot/2) * -pi, tau up to 1e3 samples, all channels of
// 1024..32768-channel bands, Ts = 1/1712e6 and random periods).  Exits 1 on any difference.
//   gcc -O2 -ffp-contract=off -o /tmp/div tools/probes/div_check.c -lm && /tmp/div [n]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#pragma STDC FP_CONTRACT OFF

static uint64_t s_state = 0x2545F4914F6CDD1Dull;
static double urand(void) {  // xorshift64*, [0, 1)
  s_state ^= s_state >> 12; s_state ^= s_state << 25; s_state ^= s_state >> 27;
  return (double)((s_state * 2685821657736338717ull) >> 11) * 0x1p-53;
}

static double div_denom(double a, double denom, double inv) {
  const double q0 = a * inv;
  const double r = fma(-q0, denom, a);
  return r == 0.0 ? q0 : fma(r, inv, q0);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  const double ctots[4] = {1024.0, 4096.0, 8192.0, 32768.0};
  long diff = 0;
  for (long i = 0; i < n; ++i) {
    const double ctot = ctots[i & 3];
    const double ts = (i & 4) ? 1.0 / 1712e6 : (0.5 + urand()) * 1e-9;
    const double denom = ctot * ts, inv = 1.0 / denom;
    const float tau_f = (float)(urand() * ts * ((i & 8) ? 1000.0 : 10.0));  // delay_vals are float32
    const double tau = tau_f;
    const double ch = floor(urand() * ctot * 8.0);  // absolute channel, up to 8 X-engines
    const double npi = -3.141592653589793;
    const double a = (i & 16) ? tau * ch * npi : tau * (ctot / 2.0) * npi;
    if (div_denom(a, denom, inv) != a / denom) {
      if (diff < 10) printf("differs: a=%.17g denom=%.17g\n", a, denom);
      ++diff;
    }
  }
  printf("n=%ld quotients, %ld differ from the IEEE division\n", n, diff);
  return diff ? 1 : 0;
}
