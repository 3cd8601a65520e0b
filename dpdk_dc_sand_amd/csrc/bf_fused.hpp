// Shared declarations of the fused beamform kernels (bf_fused.hip: item / pipe / generic / int8 kernels;
// bf_wide.hip: the wide kernel for many antennas x beams).
#pragma once

#include "bf_mfma.hpp"
#include "bf_phase.hpp"

namespace bf {

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));

struct FusedArgs {
  const uint8_t* raw;
  const float4* dv;
  const float* gain;  // optional (M, A) real per-input beam weights (?beam-weights), folded into the phasors
  const uint32_t* table;  // optional workspace for the int8 wide path's Q14 table (kLayoutW32, bf_q14table.hip)
  size_t table_bytes;
  void* y;
  int delay_channels, B, C, T, A, M, S, NT, nslabs, xcd_order;
  int path, order;  // BF_FUSED_PATH_* and BF_FUSED_ORDER_* bits of the launch flags (0 = automatic)
  int c_count;      // table-driven int8 path: channels this launch processes (0 = C; strides always use C)
  long long base_ch;
  double ctot, ts, k, t0, batch_dt;
  float out_scale;
  int knob;    // measurement knobs of the diagnostic build (0 in the product)
  int ch_run;  // persistent kernels: consecutive channels per workgroup (set by their launcher)
};

// Per-(a, m) real beam weight applied to the float32 phasor (one rounding per component, as the oracle).
__device__ __forceinline__ void apply_gain(float g, float* re, float* im) {
  *re = __fmul_rn(*re, g);
  *im = __fmul_rn(*im, g);
}


// ---- integer (int8-output) path helpers: v_mfma_i32_16x16x64_i8 fragments, Q14 limb LDS image, row transpose
constexpr uint32_t kSelP0 = 0x05040100u;  // v_perm: [S1.b0, S1.b1, S0.b0, S0.b1]
constexpr uint32_t kSelP1 = 0x07060302u;  // v_perm: [S1.b2, S1.b3, S0.b2, S0.b3]
typedef int i32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4_t mfma_i8(i32x4_t a, i32x4_t b, i32x4_t c) {
  return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

// LDS image: [s][tau][limb][lane] x 16 bytes, then 16*NTS int32 column sums.
__device__ __forceinline__ int coef8_byte(int k, int cl, int nts, int limb) {
  const int s = k >> 6, h = (k >> 4) & 3, j = k & 15, tau = cl >> 4, row = cl & 15;
  return ((((s * nts + tau) * 2 + limb) * 64) + row + 16 * h) * 16 + j;
}

// The integer contract's requantisation q = clamp(rne(f32(y) * s), +-127), as the low byte of a float's bits:
// v = RN(RN(f32(y) * s) + 1.5 * 2^23) carries rne(f32(y) * s) in its low mantissa bits whenever |f32(y) * s| < 2^22
// (the add lands in [2^23, 2^24), where the float spacing is 1, and the magic constant is even, so the add rounds
// half to even), and v_med3 against 1.5 * 2^23 +- 127 clamps every larger value to the right end.  The low byte of
// the clamped bits is then q in two's complement: 3 VALU + a quarter of a pack per value, instead of
// rint + clamp + float->int + shift/or (7).
// The two roundings are the contract: RN(y * s) first, then the magic add.  __fmul_rn / __fadd_rn alone do not stop
// hipcc from contracting them into one v_fma (v_fmaak_f32: a single rounding of y * s + magic, which differs where
// y * s lies within half a float32 ulp of a half-integer), so contraction is switched off here.  Pow2 = true: the
// caller guarantees s is a power of two, so y * s is exact and the single FMA is the same value (one VALU less).
template <bool Pow2 = false>
__device__ __forceinline__ uint32_t requant_bits(int y, float s) {
  constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23
  float v;
  if constexpr (Pow2) {
    v = __builtin_fmaf(static_cast<float>(y), s, kMagic);
  } else {
#pragma clang fp contract(off)
    v = static_cast<float>(y) * s + kMagic;
  }
  return __float_as_uint(__builtin_amdgcn_fmed3f(v, kMagic - 127.0f, kMagic + 127.0f));
}

// Whether s is a power of two (a normal float with an all-zero mantissa): requant_bits<true> is then exact.
inline bool scale_is_pow2(float s) {
  uint32_t u;
  memcpy(&u, &s, 4);
  const uint32_t e = (u >> 23) & 255;
  return (u & 0x7fffffu) == 0 && e > 0 && e < 255;
}

// [a.b0, b.b0, c.b0, d.b0]: three v_perm_b32
__device__ __forceinline__ uint32_t pack_low_bytes(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t ab = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);
  const uint32_t cd = __builtin_amdgcn_perm(d, c, 0x0c0c0400u);
  return __builtin_amdgcn_perm(cd, ab, 0x05040100u);
}

// 4x4 transpose over (lane group h = lane >> 4, register i): afterwards lane group h holds v[i] = old v[h] of lane
// group i.  Two stages of 2x2 block swaps (rows {0,1}<->{2,3}, then odd<->even rows); all 64 lanes must be active.
__device__ __forceinline__ void transpose_rows4(uint32_t (&v)[4]) {
  auto a = __builtin_amdgcn_permlane32_swap(v[0], v[2], false, false);
  auto b = __builtin_amdgcn_permlane32_swap(v[1], v[3], false, false);
  auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
  auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
  v[0] = c[0];
  v[1] = c[1];
  v[2] = d[0];
  v[3] = d[1];
}

// Workgroup barrier for LDS hand-over only: waits for this wave's LDS operations (lgkmcnt(0)), not its global
// loads.  __syncthreads() also drains vmcnt, so a voltage prefetch issued before the coefficient phase would have
// to land before the barrier and the contraction would start with nothing in flight.
__device__ __forceinline__ void lds_barrier() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0); vmcnt and expcnt at their maxima (no wait)
  __builtin_amdgcn_s_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Kernel-path override of a launch (flags & BF_FUSED_PATH_MASK): 0 automatic, else one of the BF_FUSED_PATH_* values.
inline int fused_kernel_choice(const FusedArgs& P) { return P.path; }

// Q14 coefficient tables (bf_q14table.hip): (B, C, M, A) words, the 32-beam int8 kernel's item layout, or the
// halved limb image of the config-4 int8 kernel (kLayoutW32H: per (b, c, 32-beam slab) the LDS image the contraction
// copies verbatim -- [step][tile][limb][lane] x 16 bytes of (Wc, -Ws) limb pairs, 1024 words per k-step -- then a
// 256-word block whose first 64 words are the slab's per-beam column sums (sum_a Wc, sum_a Ws)).
constexpr int kLayoutNatural = 0, kLayoutW32 = 1, kLayoutW32H = 2;
constexpr int kW32HSumWords = 256;  // the column-sum block of a kLayoutW32H item (64 words used)
__host__ __device__ inline int w32h_item_words(int Sp) { return 1024 * Sp + kW32HSumWords; }
// k-steps of 32 antennas of the 32-beam int8 kernel, padded to a multiple of 4 (its four-buffer rotation)
__host__ __device__ inline int w32_table_steps(int A) { return 4 * ((((A + 31) >> 5) + 3) / 4); }
// The table-driven 32-beam kernel stages at most 4 units of 8 words per thread: Sp <= 8 (A <= 256).
__host__ __device__ inline bool w32_table_fits(int A) { return w32_table_steps(A) <= 8; }
// Bytes of the int8 wide path's coefficient table of one launch (kLayoutW32): 1024 Sp words per (b, c, 32-beam slab).
inline size_t w32_table_bytes(int B, int C, int A, int M) {
  return static_cast<size_t>(B) * C * ((M + 31) / 32) * 1024 * w32_table_steps(A) * 4;
}
// The diagnostic halved-image layout (kLayoutW32H): w32h_item_words(Sp) words per (b, c, 32-beam slab).
inline size_t w32h_table_bytes(int B, int C, int A, int M) {
  return static_cast<size_t>(B) * C * ((M + 31) / 32) * w32h_item_words(w32_table_steps(A)) * 4;
}
int launch_q14_table(const FusedArgs& P, uint32_t* out, int layout, hipStream_t st);

// Integer wide kernels: int8 beams for many antennas x beams.  bf_wide_i8.hip: a workgroup per 32-beam slab
// (BF_FUSED_PATH_WIDE, and the automatic path beyond the item kernel's shapes).
bool i8_w32_fits(const FusedArgs& P);
template <bool Signed>
int launch_i8_w32(FusedArgs P, hipStream_t st);

// Wide kernel (bf_wide.hip): returns BF_ERR_ARG without launching when the shape does not fit it.
bool wide_fits(const FusedArgs& P);
template <bool Signed, bool Exact>
int launch_wide(FusedArgs P, hipStream_t st);

}  // namespace bf
