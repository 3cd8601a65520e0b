// Q14 steering-coefficient generator of the integer (int8-beam) path: the wavefront-parallel phasor kernel.
//
// The reference generates its steering coefficients in a kernel of its own (beamformer/beamforming/
// coeff_generator.py:12-103 writes a (B, P, C, 2A, 2M) float table; the C++ study's calculate_beamweights_*
// kernels, beamformer_coefficient_generator/BeamformerKernels.cu:7-189, one sincos per coefficient).  Here the int8
// path's coefficients -- W = rne(2^14 * RN32(g * RN32(cos rot))) and the same for sin (oracle quantise_coeffs of
// fused_tables), rot = the reference's float64 phase -- are written compactly, one uint32 (Wc | Ws << 16) per
// (b, c, m, a): 4 bytes where the reference writes 16 per coefficient and per (b, p).
//
// Cost.  With one delay model for every channel (delay_channels == 1) the phase is linear in the channel,
// rot(ch) = phi' + tau' (ch - Ctot/2) K, so a thread owns one (a, m) and walks a run of kRun consecutive channels:
// the phasor of the run's first channel from the float64 sincos (fdlibm kernels, <= 1 ulp), then one float64
// complex multiply by e^{i tau' K} per channel (<= 64 roundings: < 1e-13 drift, re-anchored every run).  Each
// component's Q14 value is decided on that float64 value +- kQ14Eps (bf_phase.hpp q14_pair: both sides give the
// same Q14 value, so it is the contract's; the recurrence's error is four orders below the guard); a component
// without a decision (~1e-5 of them), or a phase beyond the guard's validated range, is evaluated exactly
// (q14_exact: the float64 phase in the reference's operation order).  ~30 VALU per coefficient against ~80 for a
// fresh fast phasor.  Per-channel delay models (delay_channels == C) evaluate every channel with q14_fast.
//
// Layouts.  kLayoutNatural: (B, C, M, A) words (bf_q14_coeffs, include/bf.h).  kLayoutW32: the item layout the
// table-driven 32-beam int8 kernel stages into LDS (bf_wide_i8.hip): per (b, c, 32-beam slab) 1024 Sp words, word
// w = ((u >> 8) * 2 + (i >> 2)) * 1024 + (u & 255) * 4 + (i & 3) for unit u = (g << 5) | ml (beam ml of the slab,
// slot-antenna group g of 8) and slot antenna i of the group -- one 16-byte load per lane per half unit there, and
// 256 contiguous bytes per wave-store here.
#include <algorithm>
#include <cstdlib>

#include "bf_fused.hpp"

namespace bf {

namespace {

constexpr int kQ14Run = 64;  // channels per thread (re-anchored per run)
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));

struct Q14TableArgs {
  const float4* dv;
  const float* gain;
  uint32_t* out;
  int delay_channels, B, C, A, M, Sp, nslabs, layout, run, unit_fast, Cn;  // Cn: channels written (a chunk)
  long long base_ch;
  double ctot, ts, k, t0, batch_dt;
};

// Slot antenna sa of the w32 kernel's LDS image -> antenna (w8_step_base: the last step pulled back to [A - 32, A));
// false for a row an earlier step already covers or a padded step.
__device__ __forceinline__ bool w32_slot_antenna(int sa, int A, int* a) {
  const int st = sa >> 5;
  *a = min(32 * st, A - 32) + (sa & 31);
  return *a >= 32 * st && *a < A;
}

// Mode (diagnostics only): 1 the unit-gain walk without its stores (one store per thread if a sum is impossible),
// 2 the stores without the walk (each word its channel index).
template <bool Gain, int Mode = 0>
__global__ __launch_bounds__(256) void q14_table_kernel(Q14TableArgs P) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * P.run;
  const int w = blockIdx.x * 256 + threadIdx.x;  // word within a (b, c[, slab]) block
  int a, m, slab = 0;
  bool valid;
  size_t words, base;  // words per channel block; the block of (b, c0)
  if (P.layout == kLayoutNatural) {
    words = static_cast<size_t>(P.M) * P.A;
    if (w >= static_cast<int>(words)) return;
    m = w / P.A;
    a = w - m * P.A;
    valid = true;
    base = (static_cast<size_t>(b) * P.C + c0) * words + w;
  } else {
    const int per_slab = 1024 * P.Sp;
    slab = w / per_slab;
    if (slab >= P.nslabs) return;
    const int r = w - slab * per_slab;
    const int u = ((r >> 11) << 8) | ((r >> 2) & 255), i = (((r >> 10) & 1) << 2) | (r & 3);
    const int ml = u & 31, g = u >> 5;
    m = slab * 32 + ml;
    valid = w32_slot_antenna(8 * g + i, P.A, &a) && m < P.M;
    words = static_cast<size_t>(per_slab) * P.nslabs;
    base = (static_cast<size_t>(b) * P.C + c0) * words + w;
  }
  const int nrun = min(P.run, P.Cn - c0);
  uint32_t* o = P.out + base;
  if (!valid) {
    for (int j = 0; j < nrun; ++j) o[static_cast<size_t>(j) * words] = 0u;
    return;
  }
  const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
  const float g = Gain ? P.gain[static_cast<size_t>(m) * P.A + a] : 1.0f;
  const float gq = g * 16384.0f;
  const double half = P.ctot / 2.0;
  if (P.delay_channels != 1) {  // a model per channel: a fast phasor per channel, exact where undecided
    for (int j = 0; j < nrun; ++j) {
      const int c = c0 + j;
      const float4 d = P.dv[(static_cast<size_t>(c) * P.M + m) * P.A + a];
      const double ch = static_cast<double>(P.base_ch + c);
      const float uk = static_cast<float>((ch + half) * fabs(P.k));
      int wc, ws;
      if (!q14_fast(d, ch - half, P.k, dt, uk, gq, &wc, &ws)) q14_exact(d, ch, P.ctot, P.ts, dt, P.gain, g, &wc, &ws);
      o[static_cast<size_t>(j) * words] = (static_cast<uint32_t>(wc) & 0xffffu) | (static_cast<uint32_t>(ws) << 16);
    }
    return;
  }
  const float4 d = P.dv[static_cast<size_t>(m) * P.A + a];
  const double tau = fma(static_cast<double>(d.y), dt, static_cast<double>(d.x));
  const double phi = fma(static_cast<double>(d.w), dt, static_cast<double>(d.z));
  // the guard's validated range (bf_phase.hpp kQ14MaxMag), at the run's largest |channel| (NaN fails it too)
  const double ch_last = static_cast<double>(P.base_ch + c0 + nrun - 1);
  const float mag = fabsf(static_cast<float>(tau)) * static_cast<float>((ch_last + half) * fabs(P.k)) +
                    fabsf(static_cast<float>(phi));
  const bool in_range = mag < kQ14MaxMag;
  // The recurrence runs on 2^14 x the phasor (a power-of-two scale commutes with every rounding, so each value is
  // exactly 2^14 times the unscaled recurrence's): the unit-gain decision then starts from t = 2^14 v itself.
  double re = 16384.0, im = 0.0, cd = 1.0, sd = 0.0;
  if (in_range) {
    const double ch0 = static_cast<double>(P.base_ch + c0);
    sincos_pio2(fma(tau * (ch0 - half), P.k, phi), &im, &re);  // the anchor: rot(c0), as q14_fast forms it
    sincos_pio2(tau * P.k, &sd, &cd);                          // one channel's rotation
    re *= 16384.0;
    im *= 16384.0;
  }
  // The undecided channels (~1e-5 of the values, or all of them beyond the guard's range) are only flagged in the
  // walk and re-evaluated exactly after it: no divergent branch inside the recurrence loop (same speed as the
  // in-walk form, 68.3 vs 67.3 us same process, profiles/r4_o_generator_fixup_ab.txt).  Round 6: the walk is the
  // generator's cost (without its stores 59.9 of 65.6 us; the stores alone 38.9, profiles/r6_f_*), so per channel:
  // the flag is wave-wide (a ballot into a scalar mask, no 64-bit VALU shifts; every lane of a flagged channel is
  // re-evaluated exactly, which rewrites the decided lanes' words with the same contract values), the unit-gain
  // decision rounds by the float64 magic number (t + 1.5 * 2^52 holds rne(t) in its low word: no float64 -> int
  // conversion), the word is one v_perm, and the stores go through a buffer resource with the channel's offset in
  // the scalar soffset (no per-lane 64-bit address update).
  const __amdgpu_buffer_rsrc_t ors = __builtin_amdgcn_make_buffer_rsrc(
      P.out + (base - static_cast<size_t>(w)), 0, 0x7fffffff, 0x00020000);
  const uint32_t lane_off = static_cast<uint32_t>(w) * 4u;
  const uint32_t ch_off = static_cast<uint32_t>(words) * 4u;  // bytes per channel block
  auto put = [&](int j, uint32_t word) {
    __builtin_amdgcn_raw_buffer_store_b32(word, ors, lane_off, static_cast<uint32_t>(j) * ch_off, 0);
  };
  auto pack = [](int wc, int ws) {  // (Wc & 0xffff) | Ws << 16
    return __builtin_amdgcn_perm(static_cast<uint32_t>(ws), static_cast<uint32_t>(wc), 0x05040100u);
  };
  if constexpr (Mode == 2) {
    for (int j = 0; j < nrun; ++j) put(j, static_cast<uint32_t>(j));
    return;
  }
  unsigned long long fix = 0;  // wave-uniform: bit j set when some lane left channel c0 + j undecided (nrun <= 64)
  uint32_t acc = 0;
  constexpr double kMagic = 0x1.8p52;
  // a lane beyond the guard's range: every channel of the wave is evaluated exactly after the walk
  if (__builtin_amdgcn_ballot_w64(!in_range)) fix = nrun >= 64 ? ~0ull : (1ull << nrun) - 1;
  auto emit = [&](int j, uint32_t word) {  // store (or, diagnostics, fold) the word; step the recurrence
    if constexpr (Mode == 1)
      acc += word;
    else
      put(j, word);
    const double r2 = fma(re, cd, -im * sd);
    im = fma(re, sd, im * cd);
    re = r2;
  };
  if (Gain || !P.unit_fast) {  // (uniform, hoisted out of the walk)
    for (int j = 0; j < nrun; ++j) {
      bool ok = true;
      const uint32_t word = pack(q14_pair(re * 0x1p-14, gq, &ok), q14_pair(im * 0x1p-14, gq, &ok));
      if (__builtin_amdgcn_ballot_w64(ok) != __builtin_amdgcn_read_exec()) fix |= 1ull << j;
      emit(j, word);
    }
  } else {
    // t = 2^14 v: Q = rne(t) wherever t is farther than the margin from a half-integer (q14_pair_unit_scaled).  The
    // ~0.2 % of components nearer a boundary (some lane in ~1 of 4 wave-channels) take q14_pair's two-sided test
    // under ONE wave-uniform branch, and only that branch tracks undecided lanes: the common path is the recurrence,
    // four float64 margin operations per component, a v_perm and the store (round 6: the walk's scalar work --
    // two exec-mask branches and the per-channel flag update -- was ~18 SALU per channel against ~22 VALU,
    // profiles/r6_l_cfg4_gen_pmc.txt).
    for (int j = 0; j < nrun; ++j) {
      const double mc = re + kMagic, ms = im + kMagic;
      int wc = static_cast<int>(static_cast<uint32_t>(__builtin_bit_cast(unsigned long long, mc)));
      int ws = static_cast<int>(static_cast<uint32_t>(__builtin_bit_cast(unsigned long long, ms)));
      const bool uc = !(fabs(re - (mc - kMagic)) < kQ14UnitMargin);
      const bool us = !(fabs(im - (ms - kMagic)) < kQ14UnitMargin);
      if (__builtin_amdgcn_ballot_w64(uc || us)) {
        bool ok = true;
        if (uc) wc = q14_pair(re * 0x1p-14, 16384.0f, &ok);
        if (us) ws = q14_pair(im * 0x1p-14, 16384.0f, &ok);
        if (__builtin_amdgcn_ballot_w64(ok) != __builtin_amdgcn_read_exec()) fix |= 1ull << j;
      }
      emit(j, pack(wc, ws));
    }
  }
  if constexpr (Mode == 1) {
    if (acc == 0x9e3779b9u) *o = acc;
    return;
  }
  while (fix) {  // (each lane rewrites its own word: program order makes the exact value the final one)
    const int j = __builtin_ctzll(fix);
    fix &= fix - 1;
    int wc, ws;
    q14_exact(d, static_cast<double>(P.base_ch + c0 + j), P.ctot, P.ts, dt, P.gain, g, &wc, &ws);
    put(j, pack(wc, ws));
  }
}

#ifdef BF_DIAG
#include "diag/q14_image.inc"  // the halved-image generator (diagnostic build only)
#endif

}  // namespace

int launch_q14_table(const FusedArgs& P, uint32_t* out, int layout, hipStream_t st) {
  Q14TableArgs Q{};
  Q.dv = P.dv;
  Q.gain = P.gain;
  Q.out = out;
  Q.delay_channels = P.delay_channels;
  Q.B = P.B, Q.C = P.C, Q.A = P.A, Q.M = P.M;
  Q.Cn = P.c_count ? P.c_count : P.C;
  Q.Sp = w32_table_steps(P.A);
  Q.nslabs = (P.M + 31) / 32;
  Q.layout = layout;
  Q.base_ch = P.base_ch;
  Q.ctot = P.ctot, Q.ts = P.ts, Q.k = P.k, Q.t0 = P.t0, Q.batch_dt = P.batch_dt;
  const long long words = layout == kLayoutNatural ? static_cast<long long>(P.M) * P.A
                                                   : 1024LL * Q.Sp * Q.nslabs;
  // measurement: channels per recurrence run (16 / 32 / 64 / 128 / 256: 97 / 88 / 78-80 / 78 / 81 us at config 4;
  // four words per thread with 16-byte stores, plain or non-temporal: 87-90 us -- profiles/r3_o_generator_sweep.txt)
  const char* rn = diag_env("BF_Q14_RUN");
  Q.run = rn ? std::max(1, atoi(rn)) : kQ14Run;
  const char* uf = diag_env("BF_Q14_UNIT");  // measurement: 0 = the two-sided decision for unit gains too
  Q.unit_fast = !(uf && uf[0] == '0');
#ifdef BF_DIAG
  if (layout == kLayoutW32H) {  // one 1024-thread workgroup per (b, run, slab, 16-beam tile)
    Q.run = std::min(Q.run, kQ14Run);
    const long long gy = (Q.Cn + Q.run - 1) / Q.run;
    BF_REQUIRE(Q.Sp <= 8 && gy < 65536 && P.B < 65536 && Q.nslabs < 32768, "q14 image: shape too large");
    const dim3 grid(static_cast<unsigned>(2 * Q.nslabs), static_cast<unsigned>(gy), P.B);
    if (P.delay_channels != 1 && P.gain)
      hipLaunchKernelGGL((q14_image_kernel<true, true>), grid, dim3(1024), 0, st, Q);
    else if (P.delay_channels != 1)
      hipLaunchKernelGGL((q14_image_kernel<false, true>), grid, dim3(1024), 0, st, Q);
    else if (P.gain)
      hipLaunchKernelGGL((q14_image_kernel<true, false>), grid, dim3(1024), 0, st, Q);
    else
      hipLaunchKernelGGL((q14_image_kernel<false, false>), grid, dim3(1024), 0, st, Q);
    BF_LAUNCHED("q14_image_kernel");
  }
#else
  BF_REQUIRE(layout != kLayoutW32H, "q14 table: the halved-image layout is in the diagnostic build only");
#endif
  Q.run = std::min(Q.run, 64);  // (the deferred-fixup mask of q14_table_kernel holds 64 channels)
#ifdef BF_DIAG
  const char* gm = diag_env("BF_Q14_MODE");
  if (gm && (atoi(gm) == 1 || atoi(gm) == 2)) {  // measurement: the walk without stores (1) / stores only (2)
    const long long gx0 = (words + 255) / 256, gy0 = (Q.Cn + Q.run - 1) / Q.run;
    const dim3 grid(static_cast<unsigned>(gx0), static_cast<unsigned>(gy0), P.B);
    if (atoi(gm) == 1)
      hipLaunchKernelGGL((q14_table_kernel<false, 1>), grid, dim3(256), 0, st, Q);
    else
      hipLaunchKernelGGL((q14_table_kernel<false, 2>), grid, dim3(256), 0, st, Q);
    BF_LAUNCHED("q14_table_kernel");
  }
#endif
  const long long gx = (words + 255) / 256, gy = (Q.Cn + Q.run - 1) / Q.run;
  BF_REQUIRE(gx < (1LL << 31) && gy < 65536 && P.B < 65536, "q14 table: grid too large");
  if (P.gain)
    hipLaunchKernelGGL(q14_table_kernel<true>, dim3(static_cast<unsigned>(gx), static_cast<unsigned>(gy), P.B),
                       dim3(256), 0, st, Q);
  else
    hipLaunchKernelGGL(q14_table_kernel<false>, dim3(static_cast<unsigned>(gx), static_cast<unsigned>(gy), P.B),
                       dim3(256), 0, st, Q);
  BF_LAUNCHED("q14_table_kernel");
}

}  // namespace bf

extern "C" int bf_q14_coeffs(const float* delay_vals, int delay_channels, const float* gains, uint32_t* out, int B,
                             int C, int A, int M, int Ctot, int xeng_id, double sample_period, double t0,
                             double batch_dt, void* stream) {
  BF_REQUIRE(delay_vals && out, "bf_q14_coeffs: null pointer");
  BF_REQUIRE(B > 0 && C > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_q14_coeffs: bad shape B=%d C=%d A=%d M=%d Ctot=%d", B, C, A, M, Ctot);
  BF_REQUIRE(delay_channels == 1 || delay_channels == C, "bf_q14_coeffs: delay_channels must be 1 or C");
  BF_REQUIRE(static_cast<long long>(M) * A < (1LL << 31) && C < (1 << 30), "bf_q14_coeffs: shape too large");
  BF_REQUIRE(sample_period > 0.0, "bf_q14_coeffs: sample_period must be > 0");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 3) == 0,
             "bf_q14_coeffs: misaligned buffer");
  bf::FusedArgs P{};
  P.dv = reinterpret_cast<const float4*>(delay_vals);
  P.gain = gains;
  P.delay_channels = delay_channels;
  P.B = B, P.C = C, P.A = A, P.M = M;
  P.base_ch = static_cast<long long>(C) * xeng_id;
  P.ctot = static_cast<double>(Ctot);
  P.ts = sample_period;
  P.k = -3.141592653589793 / (static_cast<double>(Ctot) * sample_period);
  P.t0 = t0;
  P.batch_dt = batch_dt;
  return bf::launch_q14_table(P, out, bf::kLayoutNatural, bf::as_stream(stream));
}
