// Beamform complex multiply on CDNA4 MFMA (gfx950).
//
// The reference computes, per (batch b, pol p, channel c, time t),   (complex_mult_kernel.py:89-100)
//     y[t, col] = sum_{k < 2A} x[t, k] * W[k, col],   x[2a] = re, x[2a+1] = im,   W = [[R, I], [-I, R]] blocks
// with one numba thread per (t, k) that each redo the whole row (2A-fold redundant, L2/latency-bound).
//
// Here each (b, p, c) is a real GEMM  Y^T[2M x T] = W^T[2M x 2A] . X^T[2A x T]  on
// v_mfma_f32_16x16x32_f16:
//   * A operand = coefficients: lane l holds W^T[row = l&15][k = 32s + 8(l>>4) + j], j = 0..7 (k-step s);
//   * B operand = voltages:     lane l holds X[t = l&15][k = 32s + 8(l>>4) + j] -- 8 consecutive bytes of one
//     time row, i.e. 4 antennas' (re, im);
//   * D: lane l holds Y[t = l&15][col = 16*tau + 4(l>>4) + i], i = 0..3 -> one 16-byte store per lane.
// 8-bit voltages are exact in f16 (byte -> f16 by v_perm into 0x64xx (= 1024 + byte) and one v_pk_add).
// Coefficients are split w = hi + lo (two f16 with 11-bit significands each, ~2^-23 relative), and each
// product runs as two MFMAs into one f32 accumulator: f32-class accuracy at the f16 MFMA rate (a f32-input
// MFMA would make the 16-beam config compute-bound at ~46 % of the HBM roofline; SURVEY §7 hard part 1).
// The coefficient fragments are staged once per workgroup into LDS in exactly the lane order the MFMA reads
// (one ds_read_b128 per fragment, conflict-free), zero-padded to whole k-steps / 16-column tiles, so every
// antenna count (5, 19, 61, 79, ...) and beam count runs the same code.
//
// Two kernels share that core:
//   beamform_table_kernel  -- MatrixMultiply drop-in: x in the reordered layout (B,P,C,NB,16,A,2), W from
//                             the caller's f32 table (B,P,C,2A,2M).  One workgroup per (b, p, c[, slab]).
//   beamform_fused_kernel  -- reorder + coefficient regeneration + multiply in one pass: x read straight
//                             from the raw (B,A,C,T,2,2) layout (each antenna's (t, p, re/im) run is
//                             contiguous, so a 16-byte load = 4 samples x 2 pols of one antenna and the
//                             reorder costs no HBM traffic), W generated in float64 in-kernel per (b, c) from
//                             the delay model.  One workgroup per (b, c[, slab]), both pols.
#include "bf_common.hpp"
#include "bf_phase.hpp"

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

// ---------------------------------------------------------------------------------------------------------
// MatrixMultiply drop-in.  grid = B*P*C*nslabs; a slab is NTS 16-column tiles of the 2M outputs.
// Vec8: A % 4 == 0, so a lane's 8 bytes are one aligned 8-byte load; otherwise 2-byte antenna granules.
template <bool Signed, int NTS, bool Vec8>
__global__ __launch_bounds__(kThreads) void beamform_table_kernel(const uint8_t* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  float* __restrict__ y, int NB, int A, int M, int S,
                                                                  int NT, int nslabs) {
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slab = blockIdx.x % nslabs;
  const size_t bpc = blockIdx.x / nslabs;
  const int tau0 = slab * NTS;
  const int nts = min(NTS, NT - tau0);
  const int K2 = 2 * A, M2 = 2 * M;

  // Stage W[b,p,c][:, slab columns] -> hi/lo fragments (coalesced along the 2M row).
  {
    const float* wp = w + bpc * static_cast<size_t>(K2) * M2;
    _Float16* lh = reinterpret_cast<_Float16*>(lds);
    const int cols = nts * 16;
    const int nel = S * 32 * cols;
    for (int e = tid; e < nel; e += kThreads) {
      const int k = e / cols, cl = e - k * cols;
      const int col = tau0 * 16 + cl;
      const float v = (k < K2 && col < M2) ? wp[static_cast<size_t>(k) * M2 + col] : 0.0f;
      put_split(lh, coef_elem(k, cl, nts), v);
    }
  }
  __syncthreads();

  const int T = NB * kSamplesPerBlock;
  const uint8_t* xp = x + bpc * static_cast<size_t>(T) * K2;
  float* yp = y + bpc * static_cast<size_t>(T) * M2;
  const int h = lane >> 4, tl = lane & 15;

  for (int rg = wave; rg < NB; rg += kWaves) {
    const int t = rg * kSamplesPerBlock + tl;
    const uint8_t* row = xp + static_cast<size_t>(t) * K2;
    f32x4 acc[NTS];
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau) acc[tau] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < S; ++s) {
      const int k0 = 32 * s + 8 * h;
      uint32_t d0 = 0, d1 = 0;
      if constexpr (Vec8) {
        if (k0 < K2) {
          const uint2 v = *reinterpret_cast<const uint2*>(row + k0);
          d0 = v.x;
          d1 = v.y;
        }
      } else {
        uint32_t g[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int kq = k0 + 2 * q;
          g[q] = kq < K2 ? static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(row + kq)) : 0u;
        }
        d0 = g[0] | (g[1] << 16);
        d1 = g[2] | (g[3] << 16);
      }
      // Padded antennas load as 0 here; for signed data the flip would turn that into -128, so keep the
      // value but rely on the zero coefficient (the product is exactly 0 either way).
      const half8 v = bytes8_to_frag<Signed>(d0, d1);
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if (tau < nts) {
          const int slot = ((s * nts + tau) * 2) * 64;
          const half8 chi = lds[slot + lane];
          const half8 clo = lds[slot + 64 + lane];
          acc[tau] = mfma(chi, v, acc[tau]);
          acc[tau] = mfma(clo, v, acc[tau]);
        }
      }
    }
    float* orow = yp + static_cast<size_t>(t) * M2;
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau)
      if (tau < nts) store_f32<NTS>(orow, 16 * (tau0 + tau) + 4 * h, M2, acc[tau]);
  }
}

// ---------------------------------------------------------------------------------------------------------
// Fused reorder + coefficient regeneration + multiply.  grid = B*C*nslabs.
// Lane (tl = l&15, h = l>>4) owns time quad tq = 16*chunk + tl (samples 4tq .. 4tq+3) and, in k-step s,
// antennas 16s + 4h + q (q = 0..3): four 16-byte loads, each = 4 samples x (p0 re, p0 im, p1 re, p1 im)
// of one antenna; 16 lanes cover 256 contiguous bytes of an antenna run.  Each loaded dword feeds the
// (sample, pol) fragments directly through v_perm, so the reorder never materialises.
template <bool Signed, bool OutI8, int NTS>
__global__ __launch_bounds__(kThreads) void beamform_fused_kernel(
    const uint8_t* __restrict__ raw, const float4* __restrict__ dv, int delay_channels, void* __restrict__ yv,
    int C, int T, int A, int M, int S, int NT, int nslabs, long long base_ch, double ctot, double ts, double t0,
    double batch_dt, float out_scale) {
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slab = blockIdx.x % nslabs;
  const long long bc = blockIdx.x / nslabs;
  const int b = static_cast<int>(bc / C);
  const int c = static_cast<int>(bc % C);
  const int tau0 = slab * NTS;
  const int nts = min(NTS, NT - tau0);
  const int M2 = 2 * M;

  // Per-(b, c) coefficient regeneration (float64 phase, f32 phasor, hi/lo f16 fragments).
  {
    _Float16* lh = reinterpret_cast<_Float16*>(lds);
    const double dt = t0 + static_cast<double>(b) * batch_dt;
    const int cd = delay_channels == 1 ? 0 : c;
    const int nbeam = nts * 8;  // 16 columns per tile = 8 beams
    const int npairs = S * 16 * nbeam;
    const double ch = static_cast<double>(base_ch + c);
    for (int e = tid; e < npairs; e += kThreads) {
      const int a = e / nbeam, ml = e - a * nbeam;
      const int m = tau0 * 8 + ml;
      float re = 0.0f, im = 0.0f;
      if (a < A && m < M) steering_coeff(dv[(static_cast<size_t>(cd) * M + m) * A + a], ch, ctot, ts, dt, &re, &im);
      const int cl = 2 * ml;
      put_split(lh, coef_elem(2 * a, cl, nts), re);          // W[2a][2m]     =  cos
      put_split(lh, coef_elem(2 * a, cl + 1, nts), im);      // W[2a][2m+1]   =  sin
      put_split(lh, coef_elem(2 * a + 1, cl, nts), -im);     // W[2a+1][2m]   = -sin
      put_split(lh, coef_elem(2 * a + 1, cl + 1, nts), re);  // W[2a+1][2m+1] =  cos
    }
  }
  __syncthreads();

  const int T4 = T >> 2;
  const int nchunks = (T4 + 15) >> 4;
  const size_t ant_stride = static_cast<size_t>(C) * T * 4;
  const uint8_t* base = raw + (static_cast<size_t>(b) * A * C + c) * static_cast<size_t>(T) * 4;
  const int h = lane >> 4, tl = lane & 15;

  for (int chunk = wave; chunk < nchunks; chunk += kWaves) {
    const int tq = chunk * 16 + tl;
    const bool tv = tq < T4;
    f32x4 acc[4][2][NTS];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) acc[i][p][tau] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < S; ++s) {
      uint32_t d[4][4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int a = 16 * s + 4 * h + q;
        const uint4 v = (tv && a < A)
                            ? *reinterpret_cast<const uint4*>(base + a * ant_stride + static_cast<size_t>(tq) * 16)
                            : make_uint4(0, 0, 0, 0);
        d[q][0] = flip<Signed>(v.x);
        d[q][1] = flip<Signed>(v.y);
        d[q][2] = flip<Signed>(v.z);
        d[q][3] = flip<Signed>(v.w);
      }
      half8 chi[NTS], clo[NTS];
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if (tau < nts) {
          const int slot = ((s * nts + tau) * 2) * 64;
          chi[tau] = lds[slot + lane];
          clo[tau] = lds[slot + 64 + lane];
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint32_t sel = p ? kSelHi : kSelLo;
          const uint32_t wv[4] = {pair_to_f16x2<Signed>(d[0][i], sel), pair_to_f16x2<Signed>(d[1][i], sel),
                                  pair_to_f16x2<Signed>(d[2][i], sel), pair_to_f16x2<Signed>(d[3][i], sel)};
          const half8 v = __builtin_bit_cast(half8, wv);
#pragma unroll
          for (int tau = 0; tau < NTS; ++tau) {
            if (tau < nts) {
              acc[i][p][tau] = mfma(chi[tau], v, acc[i][p][tau]);
              acc[i][p][tau] = mfma(clo[tau], v, acc[i][p][tau]);
            }
          }
        }
      }
    }
    if (!tv) continue;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t orow = ((static_cast<size_t>(b) * 2 + p) * C + c) * static_cast<size_t>(T) + 4 * tq + i;
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) {
          if (tau < nts) {
            const int col0 = 16 * (tau0 + tau) + 4 * h;
            if constexpr (OutI8) {
              store_i8(reinterpret_cast<int8_t*>(yv) + orow * M2, col0, M2, acc[i][p][tau], out_scale);
            } else {
              store_f32<NTS>(reinterpret_cast<float*>(yv) + orow * M2, col0, M2, acc[i][p][tau]);
            }
          }
        }
      }
    }
  }
}

constexpr size_t kMaxLds = 160 * 1024;

inline size_t coef_lds_bytes(int S, int nts) { return static_cast<size_t>(S) * nts * 2 * 64 * 16; }

template <bool Signed, int NTS, bool Vec8>
int launch_table(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                 hipStream_t st) {
  const int nslabs = (NT + NTS - 1) / NTS;
  const size_t lds = coef_lds_bytes(S, NTS);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform: n_ants=%d too large for one coefficient slab", A);
  const long long grid = bpc * nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform: grid too large");
  hipLaunchKernelGGL((beamform_table_kernel<Signed, NTS, Vec8>), dim3(static_cast<unsigned>(grid)), dim3(kThreads),
                     lds, st, x, w, y, NB, A, M, S, NT, nslabs);
  BF_LAUNCHED("beamform_table_kernel");
}

template <bool Signed, int NTS>
int dispatch_vec(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                 hipStream_t st) {
  if (A % 4 == 0) return launch_table<Signed, NTS, true>(x, w, y, bpc, NB, A, M, S, NT, st);
  return launch_table<Signed, NTS, false>(x, w, y, bpc, NB, A, M, S, NT, st);
}

template <bool Signed>
int dispatch_table(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                   hipStream_t st) {
  // Widest slab whose fragments fit LDS (fewer slabs = fewer re-reads of x).
  if (NT >= 8 && coef_lds_bytes(S, 8) <= kMaxLds) return dispatch_vec<Signed, 8>(x, w, y, bpc, NB, A, M, S, NT, st);
  if (NT >= 4 && coef_lds_bytes(S, 4) <= kMaxLds) return dispatch_vec<Signed, 4>(x, w, y, bpc, NB, A, M, S, NT, st);
  if (NT >= 2 && coef_lds_bytes(S, 2) <= kMaxLds) return dispatch_vec<Signed, 2>(x, w, y, bpc, NB, A, M, S, NT, st);
  return dispatch_vec<Signed, 1>(x, w, y, bpc, NB, A, M, S, NT, st);
}

template <bool Signed, bool OutI8, int NTS>
int launch_fused(const uint8_t* raw, const float* dv, int dch, void* y, int B, int C, int T, int A, int M, int S,
                 int NT, long long base_ch, double ctot, double ts, double t0, double bdt, float scale, hipStream_t st) {
  const int nslabs = (NT + NTS - 1) / NTS;
  const size_t lds = coef_lds_bytes(S, NTS);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform_fused: n_ants=%d too large", A);
  const long long grid = static_cast<long long>(B) * C * nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
  hipLaunchKernelGGL((beamform_fused_kernel<Signed, OutI8, NTS>), dim3(static_cast<unsigned>(grid)), dim3(kThreads),
                     lds, st, raw, reinterpret_cast<const float4*>(dv), dch, y, C, T, A, M, S, NT, nslabs, base_ch,
                     ctot, ts, t0, bdt, scale);
  BF_LAUNCHED("beamform_fused_kernel");
}

template <bool Signed, bool OutI8>
int dispatch_fused(const uint8_t* raw, const float* dv, int dch, void* y, int B, int C, int T, int A, int M, int S,
                   int NT, long long base_ch, double ctot, double ts, double t0, double bdt, float scale,
                   hipStream_t st) {
  if (NT >= 2 && coef_lds_bytes(S, 2) <= kMaxLds)
    return launch_fused<Signed, OutI8, 2>(raw, dv, dch, y, B, C, T, A, M, S, NT, base_ch, ctot, ts, t0, bdt, scale, st);
  return launch_fused<Signed, OutI8, 1>(raw, dv, dch, y, B, C, T, A, M, S, NT, base_ch, ctot, ts, t0, bdt, scale, st);
}

}  // namespace bf

extern "C" int bf_beamform(const uint8_t* x, const float* w, float* y, int B, int P, int C, int NB, int A, int M,
                           int sample_signed, void* stream) {
  BF_REQUIRE(x && w && y, "bf_beamform: null pointer");
  BF_REQUIRE(B > 0 && P > 0 && C > 0 && NB > 0 && A > 0 && M > 0,
             "bf_beamform: bad shape B=%d P=%d C=%d NB=%d A=%d M=%d", B, P, C, NB, A, M);
  BF_REQUIRE((reinterpret_cast<uintptr_t>(x) & 7) == 0 && (reinterpret_cast<uintptr_t>(w) & 3) == 0 &&
                 (reinterpret_cast<uintptr_t>(y) & 15) == 0,
             "bf_beamform: misaligned buffer");
  const int S = (2 * A + 31) / 32;
  const int NT = (2 * M + 15) / 16;
  const long long bpc = static_cast<long long>(B) * P * C;
  hipStream_t st = bf::as_stream(stream);
  if (sample_signed) return bf::dispatch_table<true>(x, w, y, bpc, NB, A, M, S, NT, st);
  return bf::dispatch_table<false>(x, w, y, bpc, NB, A, M, S, NT, st);
}

extern "C" int bf_beamform_fused(const uint8_t* raw, const float* delay_vals, int delay_channels, void* y, int B,
                                 int C, int T, int A, int M, int Ctot, int xeng_id, double sample_period, double t0,
                                 double batch_dt, int sample_signed, int out_int8, float out_scale, void* stream) {
  BF_REQUIRE(raw && delay_vals && y, "bf_beamform_fused: null pointer");
  BF_REQUIRE(B > 0 && C > 0 && T > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_beamform_fused: bad shape B=%d C=%d T=%d A=%d M=%d Ctot=%d", B, C, T, A, M, Ctot);
  BF_REQUIRE(T % bf::kSamplesPerBlock == 0, "bf_beamform_fused: n_samples_per_channel=%d must be a multiple of 16", T);
  BF_REQUIRE(delay_channels == 1 || delay_channels == C, "bf_beamform_fused: delay_channels must be 1 or C");
  BF_REQUIRE(sample_period > 0.0, "bf_beamform_fused: sample_period must be > 0");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(raw) & 15) == 0 && (reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(y) & 15) == 0,
             "bf_beamform_fused: misaligned buffer");
  const int S = (2 * A + 31) / 32;
  const int NT = (2 * M + 15) / 16;
  const long long base_ch = static_cast<long long>(C) * xeng_id;
  const double ctot = static_cast<double>(Ctot);
  hipStream_t st = bf::as_stream(stream);
  const int dch = delay_channels;
  if (sample_signed) {
    if (out_int8)
      return bf::dispatch_fused<true, true>(raw, delay_vals, dch, y, B, C, T, A, M, S, NT, base_ch, ctot,
                                            sample_period, t0, batch_dt, out_scale, st);
    return bf::dispatch_fused<true, false>(raw, delay_vals, dch, y, B, C, T, A, M, S, NT, base_ch, ctot,
                                           sample_period, t0, batch_dt, out_scale, st);
  }
  if (out_int8)
    return bf::dispatch_fused<false, true>(raw, delay_vals, dch, y, B, C, T, A, M, S, NT, base_ch, ctot,
                                           sample_period, t0, batch_dt, out_scale, st);
  return bf::dispatch_fused<false, false>(raw, delay_vals, dch, y, B, C, T, A, M, S, NT, base_ch, ctot, sample_period,
                                          t0, batch_dt, out_scale, st);
}

extern "C" double bf_fused_algorithmic_bytes(int B, int C, int T, int A, int M, int delay_channels, int out_int8) {
  // voltages read once (2 B per complex sample, both pols), outputs written once, delay model once.
  const double samples = static_cast<double>(B) * C * T * 2;  // (b, c, t, p)
  const double vin = samples * A * 2.0;
  const double vout = samples * M * 2.0 * (out_int8 ? 1.0 : 4.0);
  const double dly = static_cast<double>(delay_channels) * M * A * 16.0;
  return vin + vout + dly;
}
