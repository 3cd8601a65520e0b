// Fused pre-beamform reorder + per-batch coefficient regeneration + beamform (one pass over the voltages).
//
// Replaces the reference's three-pass OpSequence (beamform_op_sequence.py:117-157: the reorder reads and writes
// the whole cube, prebeamform_reorder_kernel.mako:37-93; the coefficient generator writes a (B, P, C, 2A, 2M)
// f32 table replicated over batches and pols; the multiply reads both back) and the C++ study's fused kernel
// calculate_beamweights_and_beamform_single_channel (BeamformerKernels.cu:192-367: one sincos per MAC, a shuffle
// tree per sample, a non-complex product).
//
// Voltages are read straight from the raw (B, A, C, T, 2, 2) layout: each antenna's (t, p, re/im) run is
// contiguous, so one 16-byte load is 4 samples x 2 pols of one antenna, and the loaded dwords feed the MFMA
// B-operand fragments directly through v_perm (bf_mfma.hpp) -- the reorder costs no HBM traffic.  Coefficients
// for each (b, c) are generated in-kernel from the delay model into LDS (hi/lo f16 fragments):
//   exact mode: float64 phase in the reference's operation order + float64 sincos, bit-exact to CoeffGenerator
//               (with zero rates the fused output equals OpSequence's bit for bit);
//   fast mode (default): float64 argument without divisions, reduced mod 2 pi, float32 sincos with a
//               first-order correction -- ~1 ulp f32 phasors at a fraction of the VALU cost.
//
// Lane (tl = l&15, h = l>>4) owns time quad tq = 16*chunk + tl (samples 4tq .. 4tq+3) and, in k-step s,
// antennas 16s + 4h + q (q = 0..3); 16 lanes cover 256 contiguous bytes of an antenna run.
#include <algorithm>
#include <cstdlib>

#include "bf_fused.hpp"

namespace bf {

constexpr int kGroup = 4;  // k-steps per register-resident load group (64 antennas)

// Ablation bits for the diagnostic build (tools/diag_fused.py); the product instantiates Mode = 0 only.
constexpr int kSkipCoef = 1, kSkipMfma = 2, kSkipStore = 4, kSkipLoad = 8;
// Cache-policy bits for measurement: the product streams voltages with non-temporal loads (read once: -1.8 %
// time, profiles/r1_v2_ablation_nt.txt); kCachedLoad selects plain loads, kNtStore non-temporal beam stores
// (slower: +17 %).
constexpr int kCachedLoad = 128, kNtStore = 256, kMapChannelFastF32 = 512, kMapBatchFastF32 = 1024,
              kMapXcdBatchF32 = 2048;
// Integer item kernel layout variants (A/B-measured in the diagnostic build, profiles/r1_v7_i8_variants.txt):
// kSerialCoef evaluates the fast Q14 phasors one at a time (fewer live float64 temporaries: no gain), kPolOrder
// restores the pol-outermost contraction of full slabs (the product runs sample-row-outermost with immediate
// requantisation: -1.3 % at 3 waves per SIMD).
constexpr int kSerialCoef = 1024, kPolOrder = 2048;
// Cache-policy variants of the integer item kernel (which streams with non-temporal loads and stores).
constexpr int kI8PlainStore = 8192, kI8PlainLoad = 16384;
// Wave-priority variants (s_setprio 3): while issuing the item's loads / during the store phase.
constexpr int kPrioLoads = 1 << 16, kPrioStores = 1 << 17;
// Workgroup order variant: consecutive workgroups take consecutive batches of a channel instead of channels.
constexpr int kMapBatchFast = 1 << 18, kMapXcdBatch = 1 << 19, kMapXcdRange = 1 << 20, kMapChannelFast = 1 << 21,
              kMapXcdFlat = 1 << 22, kMapXcdBlock = 1 << 23;
// Float-beam store variant: each wave's 8 KiB (64 rows x 128 B, one slab = the whole row) staged through a padded
// wave-private LDS image and written as 1 KiB contiguous pieces per store instruction.
constexpr int kLdsStoreF32 = 1 << 25;
constexpr int kF32StageRow = 36;                        // floats per staged row (32 + 4: 4-way write conflicts)
constexpr size_t kF32StageBytes = 4 * 64 * kF32StageRow * 4;  // 4 waves x 64 rows

// Workgroup -> (batch, channel) of an item kernel.  Workgroups are dealt round-robin to the 8 XCDs (blockIdx % 8),
// so with channel-fastest numbering every XCD reads every 8th KiB run of each antenna stream.  XCD-range order
// gives XCD x the contiguous channel range [x C/8, (x+1) C/8), channel fastest within it and batches outermost:
// each XCD's resident workgroups stream one contiguous window per antenna (cfg3 int8: 461 -> 434 us,
// profiles/r1_v8_i8_order.txt).  Needs C % 8 == 0 (otherwise channel-fastest).  The slab index stays outermost.
__device__ __forceinline__ void item_coords(int item, int C, int B, bool xcd_range, int* b, int* c) {
  if (xcd_range) {
    const int xcd = item & 7, local = (item >> 3) % (B * (C >> 3));
    *b = local / (C >> 3);
    *c = xcd * (C >> 3) + local % (C >> 3);
  } else {
    *c = item % C;
    *b = (item / C) % B;
  }
}

// One group of 4 k-steps: 16 x 16-byte loads per lane, all UNCONDITIONAL: out-of-range antennas (a >= A) read
// antenna A-1 and meet zero coefficient rows, out-of-range time quads read the last quad and are never stored,
// steps s >= S are never contracted.  (A predicated load makes hipcc branch around it and wait vmcnt(0) right
// after it, serialising the group.)  Wave-uniform 64-bit base per (step, q) plus one per-lane 32-bit offset
// keeps the addresses in SGPRs.  Raw bytes are kept; the signed-sample flip happens at the consumer.
template <bool Nt = false>
__device__ __forceinline__ void load_group(const uint8_t* __restrict__ base, size_t ant_stride, int tq, int T4, int g,
                                           int A, int h, uint32_t (&d)[kGroup][4][4]) {
  const int tqc = tq < T4 ? tq : T4 - 1;
#pragma unroll
  for (int ss = 0; ss < kGroup; ++ss) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int a = 16 * (g + ss) + 4 * h + q;
      a = a < A ? a : A - 1;
      const u32x4_t* src = reinterpret_cast<const u32x4_t*>(base + static_cast<size_t>(a) * ant_stride +
                                                            static_cast<uint32_t>(tqc) * 16u);
      const u32x4_t v = Nt ? __builtin_nontemporal_load(src) : *src;
      d[ss][q][0] = v[0];
      d[ss][q][1] = v[1];
      d[ss][q][2] = v[2];
      d[ss][q][3] = v[3];
    }
  }
}

template <bool Signed>
__device__ __forceinline__ void flip_group(uint32_t (&d)[kGroup][4][4]) {
  if constexpr (Signed) {
#pragma unroll
    for (int ss = 0; ss < kGroup; ++ss)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[ss][q][j] ^= 0x80808080u;
  }
}

// Coefficients of item (b, c) for the slab's tiles -> hi/lo fragments in LDS (zero-padded), in two parts so the
// delay-model loads can be issued BEFORE the item's voltage loads (vmcnt counts in order: a load issued after the
// voltages could only be waited for by draining them too).  Pair e = tid + j*kThreads, j < kMaxPairs.
template <int NTS>
struct CoefPrefetch {
  static constexpr int kMaxPairs = (kGroup * 16 * 8 * NTS) / kThreads;  // S <= 4
  float4 dv[kMaxPairs];
  float g[kMaxPairs];
};

template <int NTS>
__device__ __forceinline__ void load_delays(CoefPrefetch<NTS>& cp, const FusedArgs& P, int c, int tau0, int nts,
                                            int tid) {
  const int cd = P.delay_channels == 1 ? 0 : c;
  const int nbeam = nts * 8;
#pragma unroll
  for (int j = 0; j < CoefPrefetch<NTS>::kMaxPairs; ++j) {
    const int e = tid + j * kThreads;
    int a = e / nbeam, m = tau0 * 8 + (e - (e / nbeam) * nbeam);
    a = a < P.A ? a : P.A - 1;
    m = m < P.M ? m : P.M - 1;
    cp.dv[j] = P.dv[(static_cast<size_t>(cd) * P.M + m) * P.A + a];
    cp.g[j] = 1.0f;
    if (P.gain) cp.g[j] = P.gain[m * P.A + a];  // uniform branch; absent gains cost nothing
  }
}

template <bool Exact, int Mode, int NTS>
__device__ __forceinline__ void make_coefs(_Float16* lh, const CoefPrefetch<NTS>& cp, const FusedArgs& P, int b, int c,
                                           int tau0, int nts, int tid) {
  const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
  const int nbeam = nts * 8;
  const int npairs = P.S * 16 * nbeam;
  const double ch = static_cast<double>(P.base_ch + c);
  const double chc = ch - P.ctot / 2.0;
#pragma unroll
  for (int j = 0; j < CoefPrefetch<NTS>::kMaxPairs; ++j) {
    const int e = tid + j * kThreads;
    if (e >= npairs) break;
    const int a = e / nbeam, ml = e - a * nbeam;
    const int m = tau0 * 8 + ml;
    float re = 0.0f, im = 0.0f;
    if constexpr (Mode & kSkipCoef) {
      re = 0.5f + 1e-3f * a;
      im = 0.25f - 1e-3f * m;
    } else if (a < P.A && m < P.M) {
      if constexpr (Exact) {
        steering_coeff(cp.dv[j], ch, make_phase(P.ctot, P.ts), dt, &re, &im);
      } else {
        // hardware v_sin / v_cos on float64-reduced revolutions (<= 3.2 x 2^-24 from the float64 phasor), as the
        // wide kernel since round 4: fewer VALU than the float32 polynomials of steering_coeff_fast
        steering_coeff_hw(cp.dv[j], chc, P.k, dt, &re, &im);
      }
      if (P.gain) apply_gain(cp.g[j], &re, &im);
    }
    const int cl = 2 * ml;
    put_split2(lh, coef_elem(2 * a, cl, nts), re, -im);     // W[2a][2m] = cos, W[2a+1][2m] = -sin
    put_split2(lh, coef_elem(2 * a, cl + 1, nts), im, re);  // W[2a][2m+1] = sin, W[2a+1][2m+1] = cos
  }
}

// Generic-kernel form (any S): straight loop, loads inline.
template <bool Exact>
__device__ __forceinline__ void gen_coefs(_Float16* lh, const FusedArgs& P, int b, int c, int tau0, int nts,
                                          int tid) {
  const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
  const int cd = P.delay_channels == 1 ? 0 : c;
  const int nbeam = nts * 8;
  const int npairs = P.S * 16 * nbeam;
  const double ch = static_cast<double>(P.base_ch + c);
  const double chc = ch - P.ctot / 2.0;
  for (int e = tid; e < npairs; e += kThreads) {
    const int a = e / nbeam, ml = e - a * nbeam;
    const int m = tau0 * 8 + ml;
    float re = 0.0f, im = 0.0f;
    if (a < P.A && m < P.M) {
      const float4 d = P.dv[(static_cast<size_t>(cd) * P.M + m) * P.A + a];
      if constexpr (Exact) {
        steering_coeff(d, ch, make_phase(P.ctot, P.ts), dt, &re, &im);
      } else {
        steering_coeff_hw(d, chc, P.k, dt, &re, &im);
      }
      if (P.gain) apply_gain(P.gain[m * P.A + a], &re, &im);
    }
    const int cl = 2 * ml;
    put_split2(lh, coef_elem(2 * a, cl, nts), re, -im);
    put_split2(lh, coef_elem(2 * a, cl + 1, nts), im, re);
  }
}

// Contract one pol of one group: acc[i][tau] += W^T(s, tau) . X(s, sample 4tq+i, pol p).
// FlipHere: flip the signed samples' sign bits of step s in place just before its first use (pol 0), so step 0's
// MFMAs only wait for step 0's loads while the later steps are still in flight.
template <bool Signed, int NTS, bool Full, bool FlipHere = false>
__device__ __forceinline__ void contract_pol(const half8* __restrict__ buf, int g, int S, int nts, int lane, int p,
                                             uint32_t (&d)[kGroup][4][4], f32x4 (&acc)[4][NTS]) {
  const uint32_t sel = p ? kSelHi : kSelLo;
#pragma unroll
  for (int ss = 0; ss < kGroup; ++ss) {
    const int s = g + ss;
    if (s >= S) break;
    if constexpr (Signed && FlipHere) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[ss][q][j] ^= 0x80808080u;
    }
    half8 chi[NTS], clo[NTS];
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau) {
      if (Full || tau < nts) {
        const int slot = ((s * nts + tau) * 2) * 64;
        chi[tau] = buf[slot + lane];
        clo[tau] = buf[slot + 64 + lane];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv[4] = {pair_to_f16x2<Signed>(d[ss][0][i], sel), pair_to_f16x2<Signed>(d[ss][1][i], sel),
                              pair_to_f16x2<Signed>(d[ss][2][i], sel), pair_to_f16x2<Signed>(d[ss][3][i], sel)};
      const half8 v = __builtin_bit_cast(half8, wv);
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if (Full || tau < nts) {
          acc[i][tau] = mfma(chi[tau], v, acc[i][tau]);
          acc[i][tau] = mfma(clo[tau], v, acc[i][tau]);
        }
      }
    }
  }
}

// Store one pol's beams of the 4 samples of quad tq.  Full: every tile complete and 16-byte aligned (2M a
// multiple of 16*NTS), so each is one unconditional 16-byte (f32) / 4-byte (int8) store.
template <bool OutI8, int NTS, bool Full, bool Nt = false>
__device__ __forceinline__ void store_pol(const FusedArgs& P, int b, int c, int p, int tau0, int nts, int tq, int h,
                                          const f32x4 (&acc)[4][NTS]) {
  const int M2 = 2 * P.M;
  if constexpr (!OutI8 && !Full && NTS == 1) {
    if (M2 == 2 || M2 == 4) {
      // one or two beams (config 2): lane (tl, h = 0) holds every column of rows 4 tq .. 4 tq + 3, 4 M2 contiguous
      // floats: 16-byte stores instead of one 4-byte store per value
      if (h == 0) {
        const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq;
        f32x4* o = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(P.y) + orow * M2);
        if (M2 == 2) {
          o[0] = f32x4{acc[0][0][0], acc[0][0][1], acc[1][0][0], acc[1][0][1]};
          o[1] = f32x4{acc[2][0][0], acc[2][0][1], acc[3][0][0], acc[3][0][1]};
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = acc[i][0];
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq + i;
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau) {
      if (Full || tau < nts) {
        const int col0 = 16 * (tau0 + tau) + 4 * h;
        if constexpr (OutI8) {
          int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow * M2;
          if constexpr (Full) {
            const uint32_t w = static_cast<uint8_t>(q8(acc[i][tau][0], P.out_scale)) |
                               (static_cast<uint32_t>(static_cast<uint8_t>(q8(acc[i][tau][1], P.out_scale))) << 8) |
                               (static_cast<uint32_t>(static_cast<uint8_t>(q8(acc[i][tau][2], P.out_scale))) << 16) |
                               (static_cast<uint32_t>(static_cast<uint8_t>(q8(acc[i][tau][3], P.out_scale))) << 24);
            *reinterpret_cast<uint32_t*>(o + col0) = w;
          } else {
            store_i8(o, col0, M2, acc[i][tau], P.out_scale);
          }
        } else {
          float* o = reinterpret_cast<float*>(P.y) + orow * M2;
          if constexpr (Full) {
            if constexpr (Nt) {
              __builtin_nontemporal_store(acc[i][tau], reinterpret_cast<f32x4*>(o + col0));
            } else {
              *reinterpret_cast<f32x4*>(o + col0) = acc[i][tau];
            }
          } else {
            store_f32<NTS>(o, col0, M2, acc[i][tau]);
          }
        }
      }
    }
  }
}

// int8 beams requantised from the float accumulators of a full slab, stored as whole rows (defined below).
template <int NTS, bool Pow2>
__device__ void store_f32acc_i8_rows(const FusedArgs& P, int b, int c, int p, int tau0, int tq, int h, int lane,
                                     int wave, bool tv, const f32x4 (&acc)[4][NTS]);

// ---------------------------------------------------------------------------------------------------------
// Single-item kernel (A <= 64, T <= 256): grid = items, one (slab, b, c) per workgroup, one register set.
// Issue order delay model -> voltages (16 x 16 B per lane, all in flight) -> coefficient math under them ->
// barrier -> per pol: MFMA contraction + stores.  Memory/compute overlap comes from the 3+ workgroups a CU holds
// at this register footprint (the hardware interleaves their phases).
// Pow2 (int8 beams): out_scale is a power of two, so RN(y * s) is exact and the requantisation's multiply and magic
// add are one exact FMA (as requant_bits<true>).
template <bool Signed, bool OutI8, int NTS, bool Exact, bool Full, int Mode = 0, int Occ = 1, bool Pow2 = false>
__global__ __launch_bounds__(kThreads, Occ) void beamform_fused_item_kernel(FusedArgs P) {
  static_assert(kDiagBuild || (Mode & (kSkipCoef | kSkipMfma | kSkipStore | kSkipLoad)) == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const int T4 = P.T >> 2;
  const int tq = wave * 16 + tl;
  const bool tv = tq < T4;
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const int item = blockIdx.x;
  int b, c;
  if constexpr ((Mode & kMapChannelFastF32) != 0) {  // diagnostics: the earlier channel-fastest order
    c = item % P.C;
    b = (item / P.C) % P.B;
  } else if constexpr ((Mode & kMapBatchFastF32) != 0) {  // diagnostics: batch fastest
    c = (item / P.B) % P.C;
    b = item % P.B;
  } else if constexpr ((Mode & kMapXcdBatchF32) != 0) {  // diagnostics: XCD x -> channels == x mod 8, batch fastest
    const int xcd = item & 7, local = (item >> 3) % (P.B * (P.C >> 3));
    b = local % P.B;
    c = (local / P.B) * 8 + xcd;
  } else {
    item_coords(item, P.C, P.B, P.xcd_order != 0, &b, &c);
  }
  const int slab = item / (P.C * P.B);
  const int tau0 = slab * NTS;
  const int nts = Full ? NTS : min(NTS, P.NT - tau0);

  uint32_t d[kGroup][4][4];
  CoefPrefetch<NTS> cp;
  if constexpr (!(Mode & kSkipCoef)) load_delays<NTS>(cp, P, c, tau0, nts, tid);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (Mode & kSkipLoad) {
#pragma unroll
    for (int ss = 0; ss < kGroup; ++ss)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) d[ss][q][j] = static_cast<uint32_t>(tid * 0x01010101u + ss + q + j);
  } else {
    const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
    load_group<(Mode & kCachedLoad) == 0>(base, ant_stride, tq, T4, 0, P.A, h, d);
  }
  __builtin_amdgcn_sched_barrier(0);
  make_coefs<Exact, Mode, NTS>(reinterpret_cast<_Float16*>(lds), cp, P, b, c, tau0, nts, tid);
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    f32x4 acc[4][NTS];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) acc[i][tau] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (Mode & kSkipMfma) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][0][q] = __builtin_bit_cast(float, d[q][p + 1][i] ^ d[q][p][i]);
    } else {
      if (p == 0) {
        contract_pol<Signed, NTS, Full, true>(lds, 0, P.S, nts, lane, 0, d, acc);
      } else {
        contract_pol<Signed, NTS, Full, false>(lds, 0, P.S, nts, lane, 1, d, acc);
      }
    }
    if constexpr (Mode & kSkipStore) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) sum += acc[i][tau][0] + acc[i][tau][1] + acc[i][tau][2] + acc[i][tau][3];
      if (sum == 1234.5f) reinterpret_cast<float*>(P.y)[tid] = sum;
    } else {
      if constexpr (OutI8 && Full) {
        store_f32acc_i8_rows<NTS, Pow2>(P, b, c, p, tau0, tq, h, lane, wave, tv, acc);
      } else if constexpr (!OutI8 && Full && NTS == 2 && (Mode & kLdsStoreF32) != 0) {
        // M2 == 32 (launcher): the wave's rows 64 w .. 64 w + 63 of (b, p, c) are one contiguous 8 KiB run
        float* stg = reinterpret_cast<float*>(reinterpret_cast<char*>(lds) + static_cast<size_t>(P.S) * NTS * 2 * 64 * 16) +
                     wave * 64 * kF32StageRow;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int tau = 0; tau < 2; ++tau)
            *reinterpret_cast<f32x4*>(stg + (4 * tl + i) * kF32StageRow + 16 * tau + 4 * h) = acc[i][tau];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 64 * wave;
        float* o = reinterpret_cast<float*>(P.y) + orow * 32;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = 8 * k + (lane >> 3), c4 = lane & 7;  // 16-byte piece `lane` of the k-th KiB
          const f32x4 v = *reinterpret_cast<const f32x4*>(stg + row * kF32StageRow + 4 * c4);
          if (64 * wave + row < P.T) {
            if constexpr ((Mode & kNtStore) != 0)
              __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(o + 256 * k + 4 * lane));
            else
              *reinterpret_cast<f32x4*>(o + 256 * k + 4 * lane) = v;
          }
        }
      } else if (tv) {
        store_pol<OutI8, NTS, Full, (Mode & kNtStore) != 0>(P, b, c, p, tau0, nts, tq, h, acc);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Generic kernel: any A (groups of 4 k-steps), any T (chunks of 64 samples per wave).  grid = B*C*nslabs.
template <bool Signed, bool OutI8, int NTS, bool Exact>
__global__ __launch_bounds__(kThreads) void beamform_fused_kernel(FusedArgs P) {
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  // XCD-aware order: workgroup g runs on XCD g % 8, so the nslabs beam slabs of item (b, c) are given to blocks
  // g = 8 (nslabs * j + slab) + x on the same XCD x: they run back to back there and the slabs after the first
  // re-read the item's voltages from that XCD's L2 instead of HBM.
  int slab, bc;
  if (P.xcd_order) {
    const int x = blockIdx.x & 7, local = blockIdx.x >> 3;
    slab = local % P.nslabs;
    bc = (local / P.nslabs) * 8 + x;
    if (bc >= P.B * P.C) return;
  } else {
    slab = blockIdx.x % P.nslabs;
    bc = blockIdx.x / P.nslabs;
  }
  const int b = bc / P.C, c = bc % P.C;
  const int tau0 = slab * NTS;
  const int nts = min(NTS, P.NT - tau0);
  const int T4 = P.T >> 2;
  const int nchunks = (T4 + 15) >> 4;
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;

  uint32_t d[kGroup][4][4];
  int chunk = wave;
  if (P.S <= kGroup) {
    // delay model, then voltages, then the coefficient math under the voltage loads (issue order pinned)
    CoefPrefetch<NTS> cp;
    load_delays<NTS>(cp, P, c, tau0, nts, tid);
    __builtin_amdgcn_sched_barrier(0);
    if (chunk < nchunks) load_group(base, ant_stride, chunk * 16 + tl, T4, 0, P.A, h, d);
    __builtin_amdgcn_sched_barrier(0);
    make_coefs<Exact, 0, NTS>(reinterpret_cast<_Float16*>(lds), cp, P, b, c, tau0, nts, tid);
  } else {
    if (chunk < nchunks) load_group(base, ant_stride, chunk * 16 + tl, T4, 0, P.A, h, d);
    gen_coefs<Exact>(reinterpret_cast<_Float16*>(lds), P, b, c, tau0, nts, tid);
  }
  __syncthreads();

  for (; chunk < nchunks; chunk += kWaves) {
    const int tq = chunk * 16 + tl;
    const bool tv = tq < T4;
    f32x4 acc[2][4][NTS];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) acc[p][i][tau] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int g = 0; g < P.S; g += kGroup) {
      if (g > 0) load_group(base, ant_stride, tq, T4, g, P.A, h, d);
      flip_group<Signed>(d);
      contract_pol<Signed, NTS, false>(lds, g, P.S, nts, lane, 0, d, acc[0]);
      contract_pol<Signed, NTS, false>(lds, g, P.S, nts, lane, 1, d, acc[1]);
    }
    const int next = chunk + kWaves;
    if (next < nchunks) load_group(base, ant_stride, next * 16 + tl, T4, 0, P.A, h, d);
    if (tv) {
      store_pol<OutI8, NTS, false>(P, b, c, 0, tau0, nts, tq, h, acc[0]);
      store_pol<OutI8, NTS, false>(P, b, c, 1, tau0, nts, tq, h, acc[1]);
    }
  }
}

// ---------------------------------------------------------------------------------------------------------
// Integer int8-output kernel: bit-exact requantised beams.
//
// Contract (oracle.fused_beamform_int8): W = rne(w * 2^14) from the exact float32 phasor w (Q14, |W| <= 16384),
// y = sum_k x_k W_k exactly (integers), q = clamp(rne(f32(y) * f32(scale * 2^-14)), -127, 127).  The float rounding
// is single, deterministic and restated in NumPy, so the output matches the oracle bit for bit.
// On v_mfma_i32_16x16x64_i8 (lane l: A[row l&15][kslot(l>>4, byte j)], B[kslot(l>>4, j)][col l&15], probed in
// tools/probes/mfma_i8_layout.hip): W = 256 W_hi + W_lo in balanced int8 limbs, per 16x16 tile
//     t = (sum hi * x) << 8;  t += sum lo * x        (i32, exact for A <= 256)
// i.e. half the MFMAs of the f16 hi/lo path and no byte->f16 conversion: each fragment dword is one v_perm of
// two antennas' raw dwords.  k-slot (s, h, j) <-> antenna a = 32 s + 8 h + j/2, re/im = j & 1.  Unsigned samples
// run as x - 128 (one xor) plus the exact correction 128 * sum_k W_k per column.



__device__ __forceinline__ void put_q14(int8_t* lb, int* colsum, int k, int cl, int nts, int W) {
  const int lo = ((W + 128) & 255) - 128;
  const int hi = (W - lo) >> 8;
  lb[coef8_byte(k, cl, nts, 0)] = static_cast<int8_t>(hi);
  lb[coef8_byte(k, cl, nts, 1)] = static_cast<int8_t>(lo);
  if (W) atomicAdd(colsum + cl, W);
}

// grid = B*C*nslabs; any A (groups of 64 antennas = two i8 k-steps), any T (64-sample chunks per wave).
template <bool Signed, int NTS>
__global__ __launch_bounds__(kThreads) void beamform_fused_i8_kernel(FusedArgs P) {
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const int slab = blockIdx.x % P.nslabs;
  const int bc = blockIdx.x / P.nslabs;
  const int b = bc / P.C, c = bc % P.C;
  const int tau0 = slab * NTS;
  const int nts = min(NTS, P.NT - tau0);
  const int S8 = (2 * P.A + 63) / 64;  // i8 k-steps
  const int T4 = P.T >> 2;
  const int nchunks = (T4 + 15) >> 4;
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
  int8_t* lb = reinterpret_cast<int8_t*>(lds);
  int* colsum = reinterpret_cast<int*>(lb + static_cast<size_t>(S8) * nts * 2 * 64 * 16);
  const int M2 = 2 * P.M;

  // 1. coefficients (Q14 of the exact phasors, bf_phase.hpp q14_coeffs) -> limbs + column sums
  for (int e = tid; e < nts * 16; e += kThreads) colsum[e] = 0;
  __syncthreads();
  {
    const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
    const int cd = P.delay_channels == 1 ? 0 : c;
    const int nbeam = nts * 8;
    const int npairs = S8 * 32 * nbeam;
    const double ch = static_cast<double>(P.base_ch + c);
    for (int e = tid; e < npairs; e += kThreads) {
      const int a = e / nbeam, ml = e - a * nbeam;
      const int m = tau0 * 8 + ml;
      const bool valid[1] = {a < P.A && m < P.M};
      const float4 dv[1] = {P.dv[(static_cast<size_t>(cd) * P.M + min(m, P.M - 1)) * P.A + min(a, P.A - 1)]};
      const float g[1] = {P.gain ? P.gain[min(m, P.M - 1) * P.A + min(a, P.A - 1)] : 1.0f};
      int wc[1], ws[1];
      q14_coeffs<1>(dv, g, valid, ch, P.ctot, P.ts, P.k, dt, P.gain, wc, ws);
      const int cl = 2 * ml;
      put_q14(lb, colsum, 2 * a, cl, nts, wc[0]);
      put_q14(lb, colsum, 2 * a, cl + 1, nts, ws[0]);
      put_q14(lb, colsum, 2 * a + 1, cl, nts, -ws[0]);
      put_q14(lb, colsum, 2 * a + 1, cl + 1, nts, wc[0]);
    }
  }
  __syncthreads();
  const int4* fr = reinterpret_cast<const int4*>(lds);
  const float s32 = P.out_scale * 0x1p-14f;  // exact: power-of-two scaling (the float rounding of scale is the oracle's)

  for (int chunk = wave; chunk < nchunks; chunk += kWaves) {
    const int tq = chunk * 16 + tl;
    const bool tv = tq < T4;
    const int tqc = tv ? tq : T4 - 1;
    i32x4_t acc[2][4][NTS];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) acc[p][i][tau] = i32x4_t{0, 0, 0, 0};
    for (int g = 0; g < S8; g += 2) {  // 64 antennas per group: 2 k-steps x 8 antennas per lane
      uint32_t d[2][8][4];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          int a = 32 * (g + ss) + 8 * h + q;
          a = a < P.A ? a : P.A - 1;  // padded antennas meet zero coefficients
          const u32x4_t v = __builtin_nontemporal_load(
              reinterpret_cast<const u32x4_t*>(base + static_cast<size_t>(a) * ant_stride + tqc * 16u));
#pragma unroll
          for (int j = 0; j < 4; ++j) d[ss][q][j] = Signed ? v[j] : (v[j] ^ 0x80808080u);
        }
      }
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if (tau >= nts) break;
        i32x4_t chi[2], clo[2];
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          const int s = min(g + ss, S8 - 1);
          const int4 x0 = fr[(((s * nts + tau) * 2 + 0) * 64) + lane];
          const int4 x1 = fr[(((s * nts + tau) * 2 + 1) * 64) + lane];
          chi[ss] = i32x4_t{x0.x, x0.y, x0.z, x0.w};
          clo[ss] = (g + ss < S8) ? i32x4_t{x1.x, x1.y, x1.z, x1.w} : i32x4_t{0, 0, 0, 0};
          if (g + ss >= S8) chi[ss] = i32x4_t{0, 0, 0, 0};
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint32_t sel = p ? kSelP1 : kSelP0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            i32x4_t f[2];
#pragma unroll
            for (int ss = 0; ss < 2; ++ss)
              f[ss] = i32x4_t{static_cast<int>(__builtin_amdgcn_perm(d[ss][1][i], d[ss][0][i], sel)),
                              static_cast<int>(__builtin_amdgcn_perm(d[ss][3][i], d[ss][2][i], sel)),
                              static_cast<int>(__builtin_amdgcn_perm(d[ss][5][i], d[ss][4][i], sel)),
                              static_cast<int>(__builtin_amdgcn_perm(d[ss][7][i], d[ss][6][i], sel))};
            i32x4_t t = mfma_i8(chi[0], f[0], i32x4_t{0, 0, 0, 0});
            t = mfma_i8(chi[1], f[1], t);
            t = t << 8;
            t = mfma_i8(clo[0], f[0], t);
            t = mfma_i8(clo[1], f[1], t);
            acc[p][i][tau] += t;
          }
        }
      }
    }
    if (!tv) continue;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq + i;
        int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow * M2;
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) {
          if (tau >= nts) break;
          const int col0 = 16 * (tau0 + tau) + 4 * h;
          uint32_t qb[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            int y = acc[p][i][tau][r];
            if constexpr (!Signed) y += 128 * colsum[16 * tau + 4 * h + r];  // x = (x - 128) + 128
            qb[r] = requant_bits(y, s32);
          }
          const uint32_t packed = pack_low_bytes(qb[0], qb[1], qb[2], qb[3]);
          if ((M2 & 3) == 0 && col0 + 4 <= M2) {
            *reinterpret_cast<uint32_t*>(o + col0) = packed;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (col0 + r < M2) o[col0 + r] = static_cast<int8_t>((packed >> (8 * r)) & 255);
          }
        }
      }
    }
  }
}

// Requantise 4 int32 beam components (columns cl0..cl0+3 of the slab) to packed int8: the integer contract
// q = clamp(rne(f32(y) * f32(scale * 2^-14)), +-127); unsigned input adds back 128 * column sum (4 wave partials).
template <bool Signed, bool Pow2 = false>
__device__ __forceinline__ uint32_t requant4(const i32x4_t& acc, const int* colsum, int cl0, float s32) {
  uint32_t q[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    int y = acc[r];
    if constexpr (!Signed) {  // x = (x - 128) + 128
      const int cl = cl0 + r;
      y += 128 * (colsum[cl] + colsum[32 + cl] + colsum[64 + cl] + colsum[96 + cl]);
    }
    q[r] = requant_bits<Pow2>(y, s32);
  }
  return pack_low_bytes(q[0], q[1], q[2], q[3]);
}


template <int Mode>
__device__ __forceinline__ void st_i8(u32x4_t v, u32x4_t* p) {
  if constexpr (Mode & kI8PlainStore)
    *p = v;
  else
    __builtin_nontemporal_store(v, p);
}

// The item's Q14 coefficient table: exact-contract phasors of this thread's (antenna, beam) pairs (fast + fixup) ->
// hi/lo int8 limb fragments in LDS (coef8_byte layout) + the per-wave column sums of the unsigned correction.
// Mode (diagnostics): kSkipCoef synthetic values, 16 float32 phasors only (inexact), 128 exact only, kSerialCoef.
template <bool Signed, int NTS, int Mode>
__device__ __forceinline__ void i8_coef_phase(int8_t* lb, int* colsum, const CoefPrefetch<NTS>& cp, const FusedArgs& P,
                                              int b, int c, int tau0, int nts, int S8, int tid, int lane, int wave) {
  const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
  const int nbeam = nts * 8;
  const int npairs = S8 * 32 * nbeam;
  const double ch = static_cast<double>(P.base_ch + c);
  // this thread's contributions to columns 2ml, 2ml+1: ml = tid % nbeam for every pair it owns (256 % nbeam == 0)
  int cs0 = 0, cs1 = 0;
  constexpr int NP = CoefPrefetch<NTS>::kMaxPairs;
  bool valid[NP];
  int wc[NP], ws[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int e = tid + j * kThreads;
    const int a = e / nbeam, m = tau0 * 8 + (e - a * nbeam);
    valid[j] = e < npairs && a < P.A && m < P.M;
  }
  if constexpr (Mode & kSkipCoef) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      wc[j] = 8192 + 16 * j + tid;
      ws[j] = 4096 - 16 * j;
    }
  } else if constexpr (Mode & 16) {  // diagnostics: float32 phasors only (not the contract)
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      float re, im;
      steering_coeff_fast(cp.dv[j], ch - P.ctot / 2.0, P.k, dt, &re, &im);
      wc[j] = static_cast<int>(__builtin_rintf(re * 16384.0f));
      ws[j] = static_cast<int>(__builtin_rintf(im * 16384.0f));
    }
  } else {
    q14_coeffs<NP, !(Mode & 128), (Mode & kSerialCoef) != 0>(cp.dv, cp.g, valid, ch, P.ctot, P.ts, P.k, dt,
                                                               P.gain, wc, ws);
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int e = tid + j * kThreads;
    if (e >= npairs) break;
    const int a = e / nbeam, ml = e - a * nbeam;
    const int Wc = wc[j], Ws = ws[j];
    const int cl = 2 * ml;
    // (k, k + 1) = (2a, 2a + 1) are adjacent bytes of one column: one 16-bit write per (column, limb)
    const int col_w[2][2] = {{Wc, -Ws}, {Ws, Wc}};  // [column cl + ec][k = 2a + f]
#pragma unroll
    for (int ec = 0; ec < 2; ++ec) {
      int h2[2], l2[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        l2[f] = ((col_w[ec][f] + 128) & 255) - 128;
        h2[f] = (col_w[ec][f] - l2[f]) >> 8;
      }
      *reinterpret_cast<uint16_t*>(lb + coef8_byte(2 * a, cl + ec, nts, 0)) =
          static_cast<uint16_t>((h2[0] & 255) | ((h2[1] & 255) << 8));
      *reinterpret_cast<uint16_t*>(lb + coef8_byte(2 * a, cl + ec, nts, 1)) =
          static_cast<uint16_t>((l2[0] & 255) | ((l2[1] & 255) << 8));
    }
    cs0 += Wc - Ws;  // column 2m:   W[2a][2m] + W[2a+1][2m]
    cs1 += Ws + Wc;  // column 2m+1: W[2a][2m+1] + W[2a+1][2m+1]
  }
  if constexpr (!Signed) {
    // nbeam (8 or 16) divides 64: lanes with equal lane % nbeam share ml; reduce them, one partial per wave
    for (int off = nbeam; off < 64; off <<= 1) {
      cs0 += __shfl_xor(cs0, off);
      cs1 += __shfl_xor(cs1, off);
    }
    if (lane < nbeam) {
      colsum[wave * 32 + 2 * lane] = cs0;
      colsum[wave * 32 + 2 * lane + 1] = cs1;
    }
  }
}

// Full-slab contraction: sample row i outermost, both pols inside, each 4-MFMA chain (hi limbs, << 8, lo limbs)
// requantised at once into packed int8 columns pkall[p][tau][i] (lane (tl, h): row 4 tq + i, columns 16 tau + 4 h ..).
template <bool Signed, int NTS, bool Pow2 = false>
__device__ __forceinline__ void i8_contract_rows(const int4* fr, const uint32_t (&d)[2][8][4], const int* colsum,
                                                 float s32, int S8, int lane, int h, uint32_t (&pkall)[2][NTS][4]) {
  i32x4_t chi[2][NTS], clo[2][NTS];
#pragma unroll
  for (int ss = 0; ss < 2; ++ss)
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau) {
      if (ss < S8) {
        const int4 x0 = fr[(((ss * NTS + tau) * 2 + 0) * 64) + lane];
        const int4 x1 = fr[(((ss * NTS + tau) * 2 + 1) * 64) + lane];
        chi[ss][tau] = i32x4_t{x0.x, x0.y, x0.z, x0.w};
        clo[ss][tau] = i32x4_t{x1.x, x1.y, x1.z, x1.w};
      } else {
        chi[ss][tau] = clo[ss][tau] = i32x4_t{0, 0, 0, 0};
      }
    }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const uint32_t sel = p ? kSelP1 : kSelP0;
      i32x4_t f[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        uint32_t w[4];
#pragma unroll
        for (int m2 = 0; m2 < 4; ++m2) {
          uint32_t lo = d[ss][2 * m2][i], hi = d[ss][2 * m2 + 1][i];
          if constexpr (!Signed) {
            lo ^= 0x80808080u;
            hi ^= 0x80808080u;
          }
          w[m2] = __builtin_amdgcn_perm(hi, lo, sel);
        }
        f[ss] = i32x4_t{static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]),
                        static_cast<int>(w[3])};
      }
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        i32x4_t t = mfma_i8(chi[0][tau], f[0], i32x4_t{0, 0, 0, 0});
        t = mfma_i8(chi[1][tau], f[1], t);
        t = t << 8;
        t = mfma_i8(clo[0][tau], f[0], t);
        t = mfma_i8(clo[1][tau], f[1], t);
        pkall[p][tau][i] = requant4<Signed, Pow2>(t, colsum, 16 * tau + 4 * h, s32);
      }
    }
  }
}

// A wave's 64 output rows of a full-width slab (M2 == 16 NTS) are one contiguous 1-2 KiB block: after the row
// transpose lane (tl, h) holds row 4 tl + h; ds_bpermute the row-per-lane chunks so that store instruction si
// writes bytes [1024 si, 1024 si + 1024) of the block.  rows = valid rows of the block (T - 64 wave).
template <int NTS, int Mode>
__device__ __forceinline__ void i8_store_block(const uint32_t (&pk)[NTS][4], int8_t* block, int lane, int rows) {
#pragma unroll
  for (int si = 0; si < NTS; ++si) {
    const int f = 64 * si + lane;  // flat 16-B chunk of the block
    const int r = f / NTS, ch = f % NTS;
    const int src = 4 * ((r >> 2) + 16 * (r & 3));  // lane (tl, h) = (r >> 2, r & 3) holds row r
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(pk[0][j])));
      if constexpr (NTS == 2) {
        const uint32_t w1 = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(pk[1][j])));
        w[j] = ch ? w1 : w[j];
      }
    }
    if (r < rows) st_i8<Mode>(u32x4_t{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4_t*>(block + 16 * lane + 1024 * si));
  }
}

// Float accumulators -> int8 beams (requantise(y, scale) = clamp(rint(RN(y * scale)), +-127), as q8) for a full
// slab: the magic-number requantisation of the integer path (requant_bits on RN(y * scale)), 4 bytes per v_perm
// pack, the 4x4 row transpose, then whole-row stores -- 1 KiB ds_bpermute blocks when the slab is the whole row --
// instead of one 4-byte store per (sample, tile) (the int8 item kernel's store path, 4x fewer, wider stores).
// Every lane of the wave must be here (permlane / bpermute); `tv` guards only the stores.
template <int NTS, bool Pow2>
__device__ void store_f32acc_i8_rows(const FusedArgs& P, int b, int c, int p, int tau0, int tq, int h, int lane,
                                     int wave, bool tv, const f32x4 (&acc)[4][NTS]) {
  constexpr float kMagic = 12582912.0f;  // 1.5 * 2^23
  const float s = P.out_scale;
  const int M2 = 2 * P.M;
  uint32_t pk[NTS][4];
#pragma unroll
  for (int tau = 0; tau < NTS; ++tau) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t q[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v;
        if constexpr (Pow2) {
          v = __builtin_fmaf(acc[i][tau][r], s, kMagic);  // y * s exact: the one FMA is the two roundings
        } else {
#pragma clang fp contract(off)  // RN(y * s), then the magic add: two roundings (see requant_bits)
          v = acc[i][tau][r] * s + kMagic;
        }
        q[r] = __float_as_uint(__builtin_amdgcn_fmed3f(v, kMagic - 127.0f, kMagic + 127.0f));
      }
      pk[tau][i] = pack_low_bytes(q[0], q[1], q[2], q[3]);
    }
    transpose_rows4(pk[tau]);
  }
  const size_t prow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T);
  if (M2 == 16 * NTS) {
    i8_store_block<NTS, 0>(pk, reinterpret_cast<int8_t*>(P.y) + (prow + 64 * wave) * M2, lane, P.T - 64 * wave);
    return;
  }
  if (tv) {
    int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 4 * tq + h) * M2 + 16 * tau0;
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau)
      st_i8<0>(u32x4_t{pk[tau][0], pk[tau][1], pk[tau][2], pk[tau][3]}, reinterpret_cast<u32x4_t*>(o + 16 * tau));
  }
}

// Item form of the integer kernel (A <= 64, T <= 256): one (slab, b, c) per workgroup in XCD-range order
// (item_coords), issue order delay model -> voltages (16 x 16 B per lane, non-temporal) -> exact-contract
// coefficients + Q14 limbs under them -> barrier -> full slabs: sample row outermost, both pols, 4 i8 MFMAs per
// (row, pol, tile) requantised at once, row transpose + ds_bpermute into 1 KiB store blocks; partial slabs and
// one/two beams: the per-pol path below.  3 waves per SIMD (launch bound; 4 spills).
// Mode (diagnostics only): kSkipCoef / kSkipMfma / kSkipStore / kSkipLoad as the float item kernel; 16 = fast
// (f32 sincos) coefficients only (inexact); 128 = exact coefficients only (no fast attempt); the layout, cache
// policy, priority and workgroup-order variants defined above.
// A64: exactly 64 antennas and every in-item offset below 2^32 (the launcher checks), so no antenna is clamped.
// Pow2: out_scale * 2^-14 is a power of two (requant_bits<true>: one exact FMA).
template <bool Signed, int NTS, bool Full, int Mode = 0, int Occ = 3, bool A64 = false, bool Pow2 = false>
__global__ __launch_bounds__(kThreads, Occ) void beamform_fused_i8_item_kernel(FusedArgs P) {
  static_assert(kDiagBuild || (Mode & (kSkipCoef | kSkipMfma | kSkipStore | kSkipLoad)) == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const int T4 = P.T >> 2;
  const int tq = wave * 16 + tl;
  const bool tv = tq < T4;
  const int tqc = tv ? tq : T4 - 1;
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const int item = blockIdx.x;
  // item -> (b, c): XCD-range order (item_coords); diagnostics: kMapChannelFast (channel fastest, the earlier
  // order), kMapBatchFast (batch fastest), kMapXcdBatch (XCD x: channels == x mod 8, batch fastest), kMapXcdRange
  // (XCD-range, batch fastest)
  int c, b;
  if constexpr ((Mode & kMapXcdRange) != 0) {
    const int xcd = item & 7, local = (item >> 3) % (P.B * (P.C >> 3));
    b = local % P.B;
    c = xcd * (P.C >> 3) + local / P.B;
  } else if constexpr ((Mode & kMapXcdBlock) != 0) {  // XCD x: 64-channel blocks x, x + 8, ... (C % 512 == 0)
    const int xcd = item & 7, local = (item >> 3) % (P.B * (P.C >> 3));
    const int cl = local % (P.C >> 3);
    b = local / (P.C >> 3);
    c = ((cl >> 6) * 8 + xcd) * 64 + (cl & 63);
  } else if constexpr ((Mode & kMapXcdFlat) != 0) {  // XCD x: items [x B C/8, (x+1) B C/8) of the (b, c) order
    const int xcd = item & 7, local = (item >> 3) % (P.B * (P.C >> 3));
    const int flat = xcd * (P.B * (P.C >> 3)) + local;
    b = flat / P.C;
    c = flat % P.C;
  } else if constexpr ((Mode & kMapXcdBatch) != 0) {
    const int xcd = item & 7, local = (item >> 3) % (P.B * (P.C >> 3));
    b = local % P.B;
    c = (local / P.B) * 8 + xcd;
  } else if constexpr ((Mode & kMapBatchFast) != 0) {
    c = (item / P.B) % P.C;
    b = item % P.B;
  } else if constexpr ((Mode & kMapChannelFast) != 0) {
    c = item % P.C;
    b = (item / P.C) % P.B;
  } else {
    item_coords(item, P.C, P.B, P.xcd_order != 0, &b, &c);
  }
  const int slab = item / (P.C * P.B);
  const int tau0 = slab * NTS;
  const int nts = Full ? NTS : min(NTS, P.NT - tau0);
  const int S8 = (2 * P.A + 63) / 64;  // 1 or 2
  const int M2 = 2 * P.M;
  int8_t* lb = reinterpret_cast<int8_t*>(lds);
  int* colsum = reinterpret_cast<int*>(lb + static_cast<size_t>(2) * NTS * 2 * 64 * 16);

  // 1. delay model (oldest), 2. voltages, 3. coefficients under them
  if constexpr ((Mode & kPrioLoads) != 0) __builtin_amdgcn_s_setprio(3);
  CoefPrefetch<NTS> cp;
  if constexpr (!(Mode & kSkipCoef)) load_delays<NTS>(cp, P, c, tau0, nts, tid);
  __builtin_amdgcn_sched_barrier(0);
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
  const uint32_t loff64 = static_cast<uint32_t>(8 * h) * static_cast<uint32_t>(ant_stride) + tqc * 16u;  // A64 only
  uint32_t d[2][8][4];
#pragma unroll
  for (int ss = 0; ss < 2; ++ss) {
    if constexpr (Mode & kSkipLoad) {
#pragma unroll
      for (int q = 0; q < 8; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) d[ss][q][jj] = static_cast<uint32_t>(tid * 0x01010101u + ss + q + jj);
      continue;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const u32x4_t* src;
      if constexpr (A64) {  // wave-uniform base + one 32-bit lane offset: no per-load VALU address arithmetic
        src = reinterpret_cast<const u32x4_t*>(base + static_cast<size_t>(32 * ss + q) * ant_stride + loff64);
      } else {
        int a = 32 * ss + 8 * h + q;
        a = a < P.A ? a : P.A - 1;
        src = reinterpret_cast<const u32x4_t*>(base + static_cast<size_t>(a) * ant_stride + tqc * 16u);
      }
      const u32x4_t v = (Mode & kI8PlainLoad) ? *src : __builtin_nontemporal_load(src);
      d[ss][q][0] = v[0];
      d[ss][q][1] = v[1];
      d[ss][q][2] = v[2];
      d[ss][q][3] = v[3];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr ((Mode & kPrioLoads) != 0) __builtin_amdgcn_s_setprio(0);
  i8_coef_phase<Signed, NTS, Mode>(lb, colsum, cp, P, b, c, tau0, nts, S8, tid, lane, wave);
  __syncthreads();
  const int4* fr = reinterpret_cast<const int4*>(lds);
  const float s32 = P.out_scale * 0x1p-14f;

  // Full slabs: sample row i outermost, both pols inside, each 4-MFMA chain requantised at once, so only the
  // packed bytes (16 VGPRs) stay live and the voltage registers of row i die after it.
  constexpr bool kTile = Full && !(Mode & (kSkipMfma | kSkipStore | kSkipLoad | kPolOrder));
  uint32_t pkall[2][NTS][4];
  if constexpr (kTile) i8_contract_rows<Signed, NTS, Pow2>(fr, d, colsum, s32, S8, lane, h, pkall);
  if constexpr ((Mode & kPrioStores) != 0) __builtin_amdgcn_s_setprio(3);

#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint32_t sel = p ? kSelP1 : kSelP0;
    i32x4_t acc[4][NTS];
#pragma unroll
    for (int tau = 0; tau < NTS; ++tau) {
      if constexpr (kTile) break;
      if (!Full && tau >= nts) break;
      i32x4_t chi[2], clo[2];
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) {
        if (ss < S8) {
          const int4 x0 = fr[(((ss * nts + tau) * 2 + 0) * 64) + lane];
          const int4 x1 = fr[(((ss * nts + tau) * 2 + 1) * 64) + lane];
          chi[ss] = i32x4_t{x0.x, x0.y, x0.z, x0.w};
          clo[ss] = i32x4_t{x1.x, x1.y, x1.z, x1.w};
        } else {
          chi[ss] = clo[ss] = i32x4_t{0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (Mode & kSkipMfma) {
          uint32_t x = static_cast<uint32_t>(chi[0][i] ^ clo[1][i]) + p;
#pragma unroll
          for (int ss = 0; ss < 2; ++ss)
#pragma unroll
            for (int q = 0; q < 8; ++q) x = (x ^ d[ss][q][i]) + q;  // every load stays live
          acc[i][tau] = i32x4_t{static_cast<int>(x), static_cast<int>(x >> 3), static_cast<int>(x >> 5),
                                static_cast<int>(x >> 7)};
          continue;
        }
        i32x4_t f[2];
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
          uint32_t w[4];
#pragma unroll
          for (int m2 = 0; m2 < 4; ++m2) {
            uint32_t lo = d[ss][2 * m2][i], hi = d[ss][2 * m2 + 1][i];
            if constexpr (!Signed) {
              lo ^= 0x80808080u;
              hi ^= 0x80808080u;
            }
            w[m2] = __builtin_amdgcn_perm(hi, lo, sel);
          }
          f[ss] = i32x4_t{static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]),
                          static_cast<int>(w[3])};
        }
        i32x4_t t = mfma_i8(chi[0], f[0], i32x4_t{0, 0, 0, 0});
        t = mfma_i8(chi[1], f[1], t);
        t = t << 8;
        t = mfma_i8(clo[0], f[0], t);
        acc[i][tau] = mfma_i8(clo[1], f[1], t);
      }
    }
    if constexpr (Full && !(Mode & kSkipStore)) {
      // requantise, then a 4x4 transpose across the lane groups h (v_permlane32/16_swap) so lane (tl, h) holds
      // all 16 * NTS bytes of output row 4 tq + h: a wave's 64 rows x 32 B go out as 2 KB of 16-B stores.
      uint32_t pk[NTS][4];
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (kTile)
            pk[tau][i] = pkall[p][tau][i];
          else
            pk[tau][i] = requant4<Signed, Pow2>(acc[i][tau], colsum, 16 * tau + 4 * h, s32);
        }
        transpose_rows4(pk[tau]);
      }
      if constexpr (Mode & 32) {  // diagnostics: contiguous 1 KB per store instruction (timing only, wrong data)
        const size_t orow0 = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 64 * wave;
        int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow0 * M2 + 16 * lane;
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau)
          __builtin_nontemporal_store(u32x4_t{pk[tau][0], pk[tau][1], pk[tau][2], pk[tau][3]},
                                      reinterpret_cast<u32x4_t*>(o + 1024 * tau));
        continue;
      }
      if (M2 == 16 * NTS) {
        // the slab is the whole row, so the wave's 64 rows are one contiguous 1-2 KB block: ds_bpermute the
        // row-per-lane chunks so that store instruction s writes bytes [1024 s, 1024 s + 1024) of it.
        const size_t orow0 = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 64 * wave;
        i8_store_block<NTS, Mode>(pk, reinterpret_cast<int8_t*>(P.y) + orow0 * M2, lane, P.T - 64 * wave);
        continue;
      }
      if (tv) {
        const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq + h;
        int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow * M2 + 16 * tau0;
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau)
          st_i8<Mode>(u32x4_t{pk[tau][0], pk[tau][1], pk[tau][2], pk[tau][3]}, reinterpret_cast<u32x4_t*>(o + 16 * tau));
      }
      continue;
    }
    if (!tv) continue;
    if constexpr (Mode & kSkipStore) {
      int sum = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) sum += acc[i][tau][0] ^ acc[i][tau][1] ^ acc[i][tau][2] ^ acc[i][tau][3];
      if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[tid] = sum;
      continue;
    }
    if constexpr (NTS == 1) {
      if (M2 == 2 || M2 == 4) {
        // one or two beams (config 2): lane (tl, h = 0) holds every column of rows 4 tq .. 4 tq + 3, which are
        // 4 M2 contiguous bytes: one 8- or 16-byte store per lane instead of 4 M2 byte stores
        uint32_t pk[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) pk[i] = requant4<Signed, Pow2>(acc[i][0], colsum, 4 * h, s32);
        if (h == 0) {
          const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq;
          int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow * M2;
          if (M2 == 2)
            __builtin_nontemporal_store(u32x2_t{__builtin_amdgcn_perm(pk[1], pk[0], 0x05040100u),
                                                __builtin_amdgcn_perm(pk[3], pk[2], 0x05040100u)},
                                        reinterpret_cast<u32x2_t*>(o));
          else
            st_i8<Mode>(u32x4_t{pk[0], pk[1], pk[2], pk[3]}, reinterpret_cast<u32x4_t*>(o));
        }
        continue;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t orow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq + i;
      int8_t* o = reinterpret_cast<int8_t*>(P.y) + orow * M2;
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if (!Full && tau >= nts) break;
        const int col0 = 16 * (tau0 + tau) + 4 * h;
        const uint32_t packed = requant4<Signed, Pow2>(acc[i][tau], colsum, 16 * tau + 4 * h, s32);
        if ((M2 & 3) == 0 && col0 + 4 <= M2) {
          *reinterpret_cast<uint32_t*>(o + col0) = packed;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (col0 + r < M2) o[col0 + r] = static_cast<int8_t>((packed >> (8 * r)) & 255);
        }
      }
    }
  }
}

// Workgroup order of the item kernels (item_coords): XCD-range when C % 8 == 0 and the beams are at least 8 (config
// 3: 450-461 -> 432-433 us); channel-fastest for one or two beams, whose read-dominated traffic measured no better
// that way (config 2: 334-357 vs 332-340 us, profiles/r1_v8_order_bench_ab.txt).  BF_FUSED_ORDER_XCD / _CHANNEL force.
bool item_xcd_order(const FusedArgs& P) {
  if (P.order == BF_FUSED_ORDER_CHANNEL) return false;
  if (P.order == BF_FUSED_ORDER_XCD) return (P.C & 7) == 0;
  return (P.C & 7) == 0 && P.M >= 8;
}

template <bool Signed, int NTS, bool Full, int Mode = 0, int Occ = 3>
int launch_i8_item(FusedArgs P, hipStream_t st, size_t min_lds = 0) {
  P.nslabs = (P.NT + NTS - 1) / NTS;
  P.xcd_order = item_xcd_order(P);
  const size_t lds = std::max<size_t>(static_cast<size_t>(2) * NTS * 2 * 64 * 16 + 4 * 32 * 4, min_lds);
  const long long n_items = static_cast<long long>(P.nslabs) * P.B * P.C;
  BF_REQUIRE(n_items < (1LL << 31), "bf_beamform_fused: too many items");
  const char* ae = diag_env("BF_I8_A64");  // measurement: 0 forces the clamped per-lane addressing
  const bool a64 = P.A == 64 && 24ull * P.C * P.T * 4 + P.T * 4ull < (1ull << 32) && !(ae && ae[0] == '0');
  const bool pow2 = scale_is_pow2(P.out_scale * 0x1p-14f);  // the requantisation's exact single FMA
  const dim3 grid(static_cast<unsigned>(n_items)), block(kThreads);
  if (a64 && pow2)
    hipLaunchKernelGGL((beamform_fused_i8_item_kernel<Signed, NTS, Full, Mode, Occ, true, true>), grid, block, lds, st, P);
  else if (a64)
    hipLaunchKernelGGL((beamform_fused_i8_item_kernel<Signed, NTS, Full, Mode, Occ, true, false>), grid, block, lds, st, P);
  else if (pow2)
    hipLaunchKernelGGL((beamform_fused_i8_item_kernel<Signed, NTS, Full, Mode, Occ, false, true>), grid, block, lds, st, P);
  else
    hipLaunchKernelGGL((beamform_fused_i8_item_kernel<Signed, NTS, Full, Mode, Occ, false, false>), grid, block, lds, st, P);
  BF_LAUNCHED("beamform_fused_i8_item_kernel");
}

template <bool Signed>
int launch_i8(FusedArgs P, hipStream_t st) {
  const int S8 = (2 * P.A + 63) / 64;
  const int choice = fused_kernel_choice(P);
  const bool small = S8 <= 2 && P.T <= 256;
  // the 32-beam slab kernels up to A = 512 (their Q14 limb image in LDS); beyond, the generic kernel (groups of 64
  // antennas).  (The round-1 16-beam slab kernel, which also covered 512 < A <= 724, is in the diagnostic build only.)
  if ((choice == BF_FUSED_PATH_WIDE || (choice == 0 && !small)) && i8_w32_fits(P)) return launch_i8_w32<Signed>(P, st);
  if (small && choice != BF_FUSED_PATH_GENERIC) {
    const int M2 = 2 * P.M;
    if (P.NT >= 2) {
      if (M2 % 32 == 0) return launch_i8_item<Signed, 2, true>(P, st);
      return launch_i8_item<Signed, 2, false>(P, st);
    }
    if (M2 == 16) return launch_i8_item<Signed, 1, true>(P, st);
    return launch_i8_item<Signed, 1, false>(P, st);
  }
  auto lds_bytes = [&](int nts) { return static_cast<size_t>(S8) * nts * 2 * 64 * 16 + nts * 16 * 4; };
  if (P.NT >= 2 && lds_bytes(2) <= kMaxLds) {
    P.nslabs = (P.NT + 1) / 2;
    const long long grid = static_cast<long long>(P.B) * P.C * P.nslabs;
    BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
    hipLaunchKernelGGL((beamform_fused_i8_kernel<Signed, 2>), dim3(static_cast<unsigned>(grid)), dim3(kThreads),
                       lds_bytes(2), st, P);
  } else {
    BF_REQUIRE(lds_bytes(1) <= kMaxLds, "bf_beamform_fused: n_ants=%d too large", P.A);
    P.nslabs = P.NT;
    const long long grid = static_cast<long long>(P.B) * P.C * P.nslabs;
    BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
    hipLaunchKernelGGL((beamform_fused_i8_kernel<Signed, 1>), dim3(static_cast<unsigned>(grid)), dim3(kThreads),
                       lds_bytes(1), st, P);
  }
  BF_LAUNCHED("beamform_fused_i8_kernel");
}

template <bool Signed, bool OutI8, int NTS, bool Exact, bool Full, int Mode, int Occ, bool Pow2>
int launch_item_k(FusedArgs P, hipStream_t st) {
  P.nslabs = (P.NT + NTS - 1) / NTS;
  P.xcd_order = item_xcd_order(P);
  if constexpr ((Mode & kLdsStoreF32) != 0)
    BF_REQUIRE(!OutI8 && Full && NTS == 2 && P.M == 16 && P.T <= 256, "item kernel: staged f32 stores need M == 16");
  const size_t lds = coef_lds_bytes(P.S, NTS) + ((Mode & kLdsStoreF32) ? kF32StageBytes : 0);
  const long long n_items = static_cast<long long>(P.nslabs) * P.B * P.C;
  BF_REQUIRE(n_items < (1LL << 31), "bf_beamform_fused: too many (batch, channel) items");
  hipLaunchKernelGGL((beamform_fused_item_kernel<Signed, OutI8, NTS, Exact, Full, Mode, Occ, Pow2>),
                     dim3(static_cast<unsigned>(n_items)), dim3(kThreads), lds, st, P);
  BF_LAUNCHED("beamform_fused_item_kernel");
}

template <bool Signed, bool OutI8, int NTS, bool Exact, bool Full, int Mode = 0, int Occ = 1>
int launch_item(FusedArgs P, hipStream_t st) {
  if constexpr (OutI8) {
    // a power-of-two scale: the float path's requantisation as one exact FMA (its round-4 two-rounding form had
    // cost cfg3 int8-via-f32 ~3 %, BENCH_r03 460.8 -> BENCH_r04 476.3 us; A/B in DESIGN §5)
    if (scale_is_pow2(P.out_scale)) return launch_item_k<Signed, OutI8, NTS, Exact, Full, Mode, Occ, true>(P, st);
  }
  return launch_item_k<Signed, OutI8, NTS, Exact, Full, Mode, Occ, false>(P, st);
}

template <bool Signed, bool OutI8, int NTS, bool Exact>
int launch_generic(FusedArgs P, hipStream_t st) {
  P.nslabs = (P.NT + NTS - 1) / NTS;
  const size_t lds = coef_lds_bytes(P.S, NTS);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform_fused: n_ants=%d too large", P.A);
  P.xcd_order = P.nslabs > 1 && P.order != BF_FUSED_ORDER_CHANNEL;
  const long long items = static_cast<long long>(P.B) * P.C;
  const long long grid = P.xcd_order ? (items + 7) / 8 * 8 * P.nslabs : items * P.nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
  hipLaunchKernelGGL((beamform_fused_kernel<Signed, OutI8, NTS, Exact>), dim3(static_cast<unsigned>(grid)),
                     dim3(kThreads), lds, st, P);
  BF_LAUNCHED("beamform_fused_kernel");
}

template <bool Signed, bool OutI8, bool Exact>
int dispatch(FusedArgs P, hipStream_t st) {
  const int choice = fused_kernel_choice(P);
  const bool small = P.S <= kGroup && P.T <= 256;
  if constexpr (!OutI8) {
    // many antennas x beams (config 4): the wide kernel keeps every beam of the item in one workgroup
    const bool wide = choice == BF_FUSED_PATH_WIDE || (choice == 0 && P.M >= 24 && (!small || P.M > 32));
    if (wide && wide_fits(P)) return launch_wide<Signed, Exact>(P, st);
  }
  if (small && choice != BF_FUSED_PATH_GENERIC) {
    // int8 beams from the float path: bounded to 4 waves per SIMD (124 VGPRs, no spills; cfg3 489 -> 465 us,
    // profiles/r3_i_cfg3_f32contract_ablation.txt); float32 beams keep the unbounded form (816 vs 811 us)
    constexpr int kOcc = OutI8 ? 4 : 1;
    const int M2 = 2 * P.M;
    if (P.NT >= 2) {
      // float beams of 16 beams (config 3): 1 KiB contiguous non-temporal stores staged through LDS, 807 -> 784 us
      // same process (profiles/r3_v_f32_staged_stores.txt, r3_x_f32_staged_ab.txt)
      if constexpr (!OutI8)
        if (P.M == 16 && P.T <= 256) return launch_item<Signed, false, 2, Exact, true, kLdsStoreF32 | kNtStore>(P, st);
      if (M2 % 32 == 0) return launch_item<Signed, OutI8, 2, Exact, true, 0, kOcc>(P, st);
      return launch_item<Signed, OutI8, 2, Exact, false, 0, kOcc>(P, st);
    }
    if (M2 == 16) return launch_item<Signed, OutI8, 1, Exact, true, 0, kOcc>(P, st);
    return launch_item<Signed, OutI8, 1, Exact, false, 0, kOcc>(P, st);
  }
  const char* wn = diag_env("BF_FUSED_GENERIC_NTS");  // measurement: force the slab width
  const int want = wn ? atoi(wn) : 2;
  if (want >= 4 && P.NT >= 4 && coef_lds_bytes(P.S, 4) <= kMaxLds) return launch_generic<Signed, OutI8, 4, Exact>(P, st);
  if (want >= 2 && P.NT >= 2 && coef_lds_bytes(P.S, 2) <= kMaxLds) return launch_generic<Signed, OutI8, 2, Exact>(P, st);
  return launch_generic<Signed, OutI8, 1, Exact>(P, st);
}

}  // namespace bf

extern "C" int bf_beamform_fused(const uint8_t* raw, const float* delay_vals, int delay_channels, void* y, int B,
                                 int C, int T, int A, int M, int Ctot, int xeng_id, double sample_period, double t0,
                                 double batch_dt, int flags, float out_scale, void* stream) {
  return bf_beamform_fused_weighted(raw, delay_vals, delay_channels, nullptr, y, B, C, T, A, M, Ctot, xeng_id,
                                    sample_period, t0, batch_dt, flags, out_scale, stream);
}

extern "C" int bf_beamform_fused_weighted(const uint8_t* raw, const float* delay_vals, int delay_channels,
                                          const float* gains, void* y, int B, int C, int T, int A, int M, int Ctot,
                                          int xeng_id, double sample_period, double t0, double batch_dt, int flags,
                                          float out_scale, void* stream) {
  return bf_beamform_fused_ws(raw, delay_vals, delay_channels, gains, y, B, C, T, A, M, Ctot, xeng_id, sample_period,
                              t0, batch_dt, flags, out_scale, nullptr, 0, stream);
}

// The workspace the automatic path of bf_beamform_fused_ws can use: the int8 wide path's Q14 coefficient table
// (bf_q14table.hip) when the shape takes the 32-beam int8 kernel, else 0.
extern "C" int bf_fused_workspace_bytes(int B, int C, int T, int A, int M, int flags, size_t* bytes) {
  BF_REQUIRE(bytes != nullptr, "bf_fused_workspace_bytes: null pointer");
  *bytes = 0;
  BF_REQUIRE(B > 0 && C > 0 && T > 0 && A > 0 && M > 0, "bf_fused_workspace_bytes: bad shape");
  const char* ferr = bf::fused_flags_error(flags);
  BF_REQUIRE(ferr == nullptr, "bf_fused_workspace_bytes: %s (flags 0x%x)", ferr, flags);
  const int path = flags & BF_FUSED_PATH_MASK;
  if ((flags & BF_FUSED_OUT_INT8) && !(flags & BF_FUSED_INT8_VIA_F32) && (path == 0 || path == BF_FUSED_PATH_WIDE)) {
    bf::FusedArgs P{};
    P.B = B, P.C = C, P.T = T, P.A = A, P.M = M;
    const bool small = (2 * A + 63) / 64 <= 2 && T <= 256;
    if ((path == BF_FUSED_PATH_WIDE || !small) && bf::i8_w32_fits(P) && bf::w32_table_fits(A))
      *bytes = bf::w32_table_bytes(B, C, A, M);
  }
  return BF_OK;
}

extern "C" int bf_beamform_fused_ws(const uint8_t* raw, const float* delay_vals, int delay_channels,
                                    const float* gains, void* y, int B, int C, int T, int A, int M, int Ctot,
                                    int xeng_id, double sample_period, double t0, double batch_dt, int flags,
                                    float out_scale, void* workspace, size_t workspace_bytes, void* stream) {
  BF_REQUIRE(raw && delay_vals && y, "bf_beamform_fused: null pointer");
  BF_REQUIRE(B > 0 && C > 0 && T > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_beamform_fused: bad shape B=%d C=%d T=%d A=%d M=%d Ctot=%d", B, C, T, A, M, Ctot);
  BF_REQUIRE(T % bf::kSamplesPerBlock == 0, "bf_beamform_fused: n_samples_per_channel=%d must be a multiple of 16", T);
  BF_REQUIRE(delay_channels == 1 || delay_channels == C, "bf_beamform_fused: delay_channels must be 1 or C");
  BF_REQUIRE(sample_period > 0.0, "bf_beamform_fused: sample_period must be > 0");
  const char* ferr = bf::fused_flags_error(flags);
  BF_REQUIRE(ferr == nullptr, "bf_beamform_fused: %s (flags 0x%x)", ferr, flags);
  BF_REQUIRE((reinterpret_cast<uintptr_t>(raw) & 15) == 0 && (reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0 &&
                 (reinterpret_cast<uintptr_t>(y) & 15) == 0,
             "bf_beamform_fused: misaligned buffer");
  bf::FusedArgs P{};
  P.raw = raw;
  P.dv = reinterpret_cast<const float4*>(delay_vals);
  P.gain = gains;
  P.y = y;
  BF_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "bf_beamform_fused: misaligned workspace");
  P.table = static_cast<const uint32_t*>(workspace);
  P.table_bytes = workspace ? workspace_bytes : 0;
  P.delay_channels = delay_channels;
  P.B = B;
  P.C = C;
  P.T = T;
  P.A = A;
  P.M = M;
  P.S = (2 * A + 31) / 32;
  P.NT = (2 * M + 15) / 16;
  P.base_ch = static_cast<long long>(C) * xeng_id;
  P.ctot = static_cast<double>(Ctot);
  P.ts = sample_period;
  P.k = -3.141592653589793 / (static_cast<double>(Ctot) * sample_period);
  P.t0 = t0;
  P.batch_dt = batch_dt;
  P.out_scale = out_scale;
  P.path = flags & BF_FUSED_PATH_MASK;
  P.order = flags & BF_FUSED_ORDER_MASK;
  hipStream_t st = bf::as_stream(stream);
  const bool sgn = flags & BF_FUSED_SIGNED, i8 = flags & BF_FUSED_OUT_INT8, ex = flags & BF_FUSED_EXACT_COEFF;
  // int8 beams: the Q14 integer contract (default), or requantised float beams (BF_FUSED_INT8_VIA_F32)
  if (i8 && !(flags & BF_FUSED_INT8_VIA_F32)) {
    // The contract's int32 sum: |y| <= A * max|x| * (|Wc| + |Ws|) with |Wc| + |Ws| <= sqrt(2) * 2^14 + 1 = 23171 at
    // unit gain.  Beyond that the int32 accumulators would wrap (the oracle sums in int64): refuse.  With gains the
    // caller, which owns the weights, checks the bound (FusedBeamformerTemplate.check_weights).
    BF_REQUIRE(gains || static_cast<double>(A) * (sgn ? 128 : 255) * 23171.0 < 2147483648.0,
               "bf_beamform_fused: n_ants=%d overflows the int8 path's int32 beam sums (%s samples); use float beams "
               "or BF_FUSED_INT8_VIA_F32", A, sgn ? "int8" : "uint8");
    return sgn ? bf::launch_i8<true>(P, st) : bf::launch_i8<false>(P, st);
  }
  if (sgn) {
    if (i8) return ex ? bf::dispatch<true, true, true>(P, st) : bf::dispatch<true, true, false>(P, st);
    return ex ? bf::dispatch<true, false, true>(P, st) : bf::dispatch<true, false, false>(P, st);
  }
  if (i8) return ex ? bf::dispatch<false, true, true>(P, st) : bf::dispatch<false, true, false>(P, st);
  return ex ? bf::dispatch<false, false, true>(P, st) : bf::dispatch<false, false, false>(P, st);
}

extern "C" double bf_fused_algorithmic_bytes(int B, int C, int T, int A, int M, int delay_channels, int out_int8) {
  // voltages read once (2 B per complex sample, both pols), beams written once, delay model once.
  const double samples = static_cast<double>(B) * C * T * 2;  // (b, c, t, p)
  const double vin = samples * A * 2.0;
  const double vout = samples * M * 2.0 * (out_int8 ? 1.0 : 4.0);
  const double dly = static_cast<double>(delay_channels) * M * A * 16.0;
  return vin + vout + dly;
}

#ifdef BF_DIAG
#include "diag/fused_diag.inc"
#endif
