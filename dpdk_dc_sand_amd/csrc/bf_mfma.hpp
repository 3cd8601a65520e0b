// Shared MFMA building blocks of the beamform kernels (bf_beamform.hip, bf_fused.hip).  See bf_beamform.hip for
// the operand mapping: Y^T[2M x T] = W^T[2M x 2A] . X^T[2A x T] on v_mfma_f32_16x16x32_f16, coefficients split
// into hi/lo f16 fragments staged in LDS in lane order, 8-bit voltages converted to f16 exactly by v_perm.
#pragma once

#include "bf_common.hpp"

namespace bf {


typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kSelLo = 0x04010400u;  // v_perm: [b0, 0x64, b1, 0x64] -> f16 pair (1024+b0, 1024+b1)
constexpr uint32_t kSelHi = 0x04030402u;  // v_perm: [b2, 0x64, b3, 0x64]

// Two 8-bit values (re, im) -> exact f16 pair.  For signed samples the caller has flipped the sign bits
// (x ^ 0x80 = x + 128 as unsigned), so the bias is 1024 + 128.
template <bool Signed>
__device__ __forceinline__ uint32_t pair_to_f16x2(uint32_t d, uint32_t sel) {
  const uint32_t w = __builtin_amdgcn_perm(0x64646464u, d, sel);
  constexpr _Float16 bias = Signed ? static_cast<_Float16>(1152.0f) : static_cast<_Float16>(1024.0f);
  half2v h = __builtin_bit_cast(half2v, w);
  h = h - half2v{bias, bias};
  return __builtin_bit_cast(uint32_t, h);
}

template <bool Signed>
__device__ __forceinline__ uint32_t flip(uint32_t d) {
  return Signed ? (d ^ 0x80808080u) : d;
}

// 8 bytes (k .. k+7 of one time row) -> B-operand fragment.
template <bool Signed>
__device__ __forceinline__ half8 bytes8_to_frag(uint32_t d0, uint32_t d1) {
  d0 = flip<Signed>(d0);
  d1 = flip<Signed>(d1);
  const uint32_t w[4] = {pair_to_f16x2<Signed>(d0, kSelLo), pair_to_f16x2<Signed>(d0, kSelHi),
                         pair_to_f16x2<Signed>(d1, kSelLo), pair_to_f16x2<Signed>(d1, kSelHi)};
  return __builtin_bit_cast(half8, w);
}

__device__ __forceinline__ f32x4 mfma(half8 a, half8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// LDS image of the coefficient fragments: [s][tau][hi/lo][lane] x half8.  Element (k, local col cl) of the
// slab lives at lane (cl & 15) + 16 * ((k >> 3) & 3), element k & 7, slot (s = k >> 5, tau = cl >> 4).
__device__ __forceinline__ int coef_elem(int k, int cl, int nts) {
  const int s = k >> 5, h = (k >> 3) & 3, j = k & 7, tau = cl >> 4, row = cl & 15;
  return ((((s * nts + tau) * 2) * 64) + row + 16 * h) * 8 + j;
}

__device__ __forceinline__ void put_split(_Float16* lh, int e, float w) {
  const _Float16 hi = static_cast<_Float16>(w);
  const _Float16 lo = static_cast<_Float16>(w - static_cast<float>(hi));  // exact difference, then rounded
  lh[e] = hi;
  lh[e + 64 * 8] = lo;  // the lo fragment follows the hi fragment (next 1 KiB)
}

// Rows k = 2a and 2a + 1 of one column are adjacent halves of a lane's fragment (coef_elem(2a + 1, cl) =
// coef_elem(2a, cl) + 1): one 4-byte LDS write per limb for the pair instead of two 2-byte writes.
__device__ __forceinline__ void put_split2(_Float16* lh, int e, float w0, float w1) {
  const _Float16 h0 = static_cast<_Float16>(w0), h1 = static_cast<_Float16>(w1);
  const _Float16 l0 = static_cast<_Float16>(w0 - static_cast<float>(h0));
  const _Float16 l1 = static_cast<_Float16>(w1 - static_cast<float>(h1));
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  *reinterpret_cast<h2v*>(lh + e) = h2v{h0, h1};
  *reinterpret_cast<h2v*>(lh + e + 64 * 8) = h2v{l0, l1};
}

template <int NTS>
__device__ __forceinline__ void store_f32(float* orow, int col0, int M2, const f32x4& v) {
  if ((M2 & 3) == 0 && col0 + 4 <= M2) {
    *reinterpret_cast<f32x4*>(orow + col0) = v;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (col0 + i < M2) orow[col0 + i] = v[i];
  }
}

__device__ __forceinline__ int8_t q8(float v, float scale) {
  float r = __builtin_rintf(v * scale);
  r = fminf(fmaxf(r, -127.0f), 127.0f);
  return static_cast<int8_t>(static_cast<int>(r));
}

__device__ __forceinline__ void store_i8(int8_t* orow, int col0, int M2, const f32x4& v, float scale) {
  const int8_t q0 = q8(v[0], scale), q1 = q8(v[1], scale), q2 = q8(v[2], scale), q3 = q8(v[3], scale);
  if ((M2 & 3) == 0 && col0 + 4 <= M2) {
    const uint32_t w = static_cast<uint8_t>(q0) | (static_cast<uint32_t>(static_cast<uint8_t>(q1)) << 8) |
                       (static_cast<uint32_t>(static_cast<uint8_t>(q2)) << 16) |
                       (static_cast<uint32_t>(static_cast<uint8_t>(q3)) << 24);
    *reinterpret_cast<uint32_t*>(orow + col0) = w;
  } else {
    const int8_t qs[4] = {q0, q1, q2, q3};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (col0 + i < M2) orow[col0 + i] = qs[i];
  }
}

constexpr size_t kMaxLds = 160 * 1024;

inline size_t coef_lds_bytes(int S, int nts) { return static_cast<size_t>(S) * nts * 2 * 64 * 16; }

}  // namespace bf
