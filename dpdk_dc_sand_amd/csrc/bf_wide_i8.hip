// Integer wide fused beamformer: many antennas x beams (config 4: 256 antennas, 64 beams), int8 beams, bit-exact.
// The 32-beam slab kernels are the product (BF_FUSED_PATH_WIDE); the measured-slower forms (the round-1 16-beam slabs,
// round 4's halved-image kernel) and the measurement entry points live in diag/*.inc, compiled only with -DBF_DIAG.
//
// Same integer contract as beamform_fused_i8_item_kernel (oracle.fused_beamform_int8: Q14 coefficients of the
// exact float32 phasors, exact int32 products, one float rounding to int8), organised like the float wide kernel
// (bf_wide.hip) for a per-item GEMM too large for the item kernel.  The full [[R, I], [-I, R]] Q14 table (the float
// kernel's [R, -I] + [x_im, -x_re] trick would need -x_re, which overflows int8 at -128).  Per k-step (64 k = 32
// antennas) a lane loads 8 antennas' runs (uniform base + 32-bit lane offset; the last step is pulled back to
// [A - 32, A) with zero rows for antennas already covered) and builds each pol's fragment with one v_perm per dword;
// hi and lo limbs accumulate in separate int32 registers, combined once at the end as (hi << 8) + lo.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "bf_fused.hpp"

namespace bf {

namespace {

constexpr int kW8Threads = 256;

__device__ __forceinline__ int w8_step_base(int s, int A) { return min(32 * s, A - 32); }
// k-steps of 32 antennas, padded to an even count (ping-pong, see the float wide kernel)
__host__ __device__ inline int w8_padded_steps(int A) { return 2 * ((((A + 31) >> 5) + 1) / 2); }

#ifdef BF_DIAG
#include "diag/wide_i8_w8.inc"  // the 16-beam slab kernel (diagnostic build only)
#endif

// ---- 32-beam slabs (the default integer wide kernel) -------------------------------------------------------------
// The 16-beam kernel above re-reads each item's voltages once per slab (4x at 64 beams) with a prefetch distance of
// one step: tools/diag_fused.py showed it latency-bound on those re-reads (no-coef, no-MFMA 442 us against a 164 us
// read of the same bytes in the same item-major order).  Here a workgroup slab is 32 beams (the Q14 table is 64 KiB:
// two workgroups per CU) and a wave 32 samples x 32 beams: half the voltage bytes per MFMA (each lane loads
// 8-byte runs = 2 samples of 8 antennas), four step buffers of 16 registers (three steps in flight while one is
// contracted), and the prefetch runs on across the wave's chunks so the next chunk's steps load under the stores.
constexpr int kW32Beams = 32;

// k-steps of 32 antennas padded to a multiple of 4 (the four-buffer rotation); padded steps have zero table rows
__host__ __device__ inline int w32_steps(int A) { return w32_table_steps(A); }
// LDS: the Q14 limb image (Sp steps x 4 tiles x 2 limbs x 64 lanes x 16 B) + the unsigned correction's partial
// column sums (4 waves x 64 columns)
__host__ __device__ inline size_t w32_lds_bytes(int A) {
  return static_cast<size_t>(w32_steps(A)) * 4 * 2 * 64 * 16 + 4 * 64 * 4;
}

typedef uint16_t u16x2_t __attribute__((ext_vector_type(2)));

// One table unit -- beam ml of the slab x 8 slot antennas (group g: step g >> 2, lane group g & 3) as 8 words
// (Wc | Ws << 16) -- into the LDS limb image: 4 entries of 16 bytes, one per (column 2 ml / 2 ml + 1, limb).  Column
// 2 ml holds (Wc, -Ws) per antenna, column 2 ml + 1 (Ws, Wc); balanced limbs W = 256 hi + lo: lo is W's byte 0, hi
// byte 1 of W + 128 (16-bit lanes: no carry between the halves).  Per antenna 3 packed 16-bit ops, per antenna
// pair one v_perm per entry dword.
__device__ __forceinline__ void w32_expand_unit(int8_t* lb, int ml, int g, const u32x4_t& q0, const u32x4_t& q1) {
  const uint32_t d[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
  uint32_t n[8], np[8], pp[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const u16x2_t v = __builtin_bit_cast(u16x2_t, d[i]);
    const u16x2_t neg = v * u16x2_t{1, 0xffff};  // (Wc, -Ws)
    n[i] = __builtin_bit_cast(uint32_t, neg);
    np[i] = __builtin_bit_cast(uint32_t, neg + u16x2_t{128, 128});
    pp[i] = __builtin_bit_cast(uint32_t, v + u16x2_t{128, 128});
  }
  u32x4_t e_hi0, e_lo0, e_hi1, e_lo1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    e_lo0[q] = __builtin_amdgcn_perm(n[2 * q + 1], n[2 * q], 0x06040200u);    // [Wc.b0, -Ws.b0] x 2 antennas
    e_hi0[q] = __builtin_amdgcn_perm(np[2 * q + 1], np[2 * q], 0x07050301u);  // hi limbs of (Wc, -Ws)
    e_lo1[q] = __builtin_amdgcn_perm(d[2 * q + 1], d[2 * q], 0x04060002u);    // [Ws.b0, Wc.b0]
    e_hi1[q] = __builtin_amdgcn_perm(pp[2 * q + 1], pp[2 * q], 0x05070103u);  // hi limbs of (Ws, Wc)
  }
  const int st = g >> 2, h = g & 3, tau = ml >> 3, row = (2 * ml) & 15;
  int8_t* o = lb + ((((st * 4 + tau) * 2) * 64) + row + 16 * h) * 16;  // column 2 ml, limb 0 (= hi)
  *reinterpret_cast<u32x4_t*>(o) = e_hi0;
  *reinterpret_cast<u32x4_t*>(o + 64 * 16) = e_lo0;
  *reinterpret_cast<u32x4_t*>(o + 16) = e_hi1;
  *reinterpret_cast<u32x4_t*>(o + 16 + 64 * 16) = e_lo1;
}

// One step's voltages: 8 antennas' 8-byte runs.  (Raw buffer loads with the row offsets as soffsets would save the
// ~28 VALU of 64-bit address arithmetic per step, but their SGPRs pushed this 247-VGPR kernel into spills.)
// (kept as 8-byte vectors: split into scalar arrays, the pairs were re-packed into the loop's registers with copies
// that made the prologue wait for its own prefetch)
template <int Mode>
__device__ __forceinline__ void w32_load(const uint8_t* __restrict__ base, size_t ant_stride, uint32_t loff, int s,
                                         int A, u32x2_t (&d)[8]) {
  const int a0 = w8_step_base(s, A);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if constexpr (Mode & 8) {
      d[q] = u32x2_t{loff * 0x01010101u + s + q, loff * 0x01010101u + s - q};
      continue;
    }
    d[q] = *reinterpret_cast<const u32x2_t*>(base + static_cast<size_t>(a0 + q) * ant_stride + loff);
  }
}

// The same loads through a buffer resource on the workgroup's (b, c0) block: every load is buffer_load_dwordx2 with
// the lane part of the offset in one VGPR (antenna group 8h of the step, the sample pair) and the wave-uniform part
// -- row (a0 + q) of the step, the channel -- in an SGPR soffset: no per-load 64-bit address arithmetic on the VALU
// (the pointer form spends a v_mad_u64_u32 and moves per load).  Offsets below 2^31 (the host checks A C T 4).
template <int Mode>
__device__ __forceinline__ void w32_load_buf(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t sbase, uint32_t stride,
                                             u32x2_t (&d)[8]) {
  if constexpr ((Mode & 256) != 0) {
    // diagnostics (timing only, wrong beams): the same bytes in half the instructions -- lane pair (tl, tl ^ 1) loads
    // 16 bytes of row 2q + (tl & 1) at the pair's sample offset, without the swap that would hand each lane its own
    // rows back: is the TA's address rate (8-byte lane loads) what bounds the kernel?
    const uint32_t odd = (voff >> 3) & 1;  // tl & 1 (voff = hoff + 8 tl)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4_t v = __builtin_bit_cast(
          u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, voff - 8 * odd + odd * stride, sbase + 2 * q * stride, 0));
      d[2 * q] = u32x2_t{v[0], v[1]};
      d[2 * q + 1] = u32x2_t{v[2], v[3]};
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if constexpr (Mode & 8) {
      d[q] = u32x2_t{voff * 0x01010101u + sbase + q, voff * 0x01010101u + sbase - q};
      continue;
    }
    // (Mode 128, diagnostics: non-temporal voltage loads)
    d[q] = __builtin_bit_cast(u32x2_t, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, sbase + q * stride, (Mode & 128) ? 2 : 0));
  }
}

// The step's B fragments [pol][sample] (one v_perm per dword); the voltage registers are free afterwards.
template <bool Signed>
__device__ __forceinline__ void w32_frags(const u32x2_t (&d)[8], i32x4_t (&f)[2][2]) {
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t w[4];
#pragma unroll
      for (int m2 = 0; m2 < 4; ++m2) {
        const u32x2_t da = d[2 * m2], db = d[2 * m2 + 1];
        uint32_t a = i ? da.y : da.x, b = i ? db.y : db.x;
        if constexpr (!Signed) {  // x - 128 as int8 (128 * column sum added back at the end)
          a ^= 0x80808080u;
          b ^= 0x80808080u;
        }
        w[m2] = __builtin_amdgcn_perm(b, a, p ? kSelP1 : kSelP0);
      }
      f[p][i] = i32x4_t{static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]), static_cast<int>(w[3])};
    }
}

// The step's second B fragments [x_im, ~x_re] per pol and sample: the halved limb image's y_im operand (~x = -x - 1
// stays in int8 where -x overflows at -128; the bias is sum_a Ws per beam, removed at requantisation).  Per raw dword
// one xor (the re bytes of both pols; unsigned samples: x - 128 in the im bytes, ~(x - 128) in the re bytes) and per
// fragment dword one v_perm.
template <bool Signed = true>
__device__ __forceinline__ void w32_frags_im(const u32x2_t (&d)[8], i32x4_t (&f)[2][2]) {
  constexpr uint32_t kFlip = Signed ? 0x00ff00ffu : 0x807f807fu;
  uint32_t nd[8][2];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    nd[q][0] = d[q].x ^ kFlip;
    nd[q][1] = d[q].y ^ kFlip;
  }
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint32_t w[4];
#pragma unroll
      for (int m2 = 0; m2 < 4; ++m2)
        w[m2] = __builtin_amdgcn_perm(nd[2 * m2 + 1][i], nd[2 * m2][i], p ? 0x06070203u : 0x04050001u);
      f[p][i] = i32x4_t{static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]), static_cast<int>(w[3])};
    }
}

// 32 MFMAs of one step: per tile t (16 real columns) the two limbs' A fragments from LDS, 2 pols x 2 samples.
template <int Mode>
__device__ __forceinline__ void w32_mfma(const int4* __restrict__ fr, int s, int lane, const i32x4_t (&f0)[2][2],
                                         i32x4_t (&hi)[2][2][4], i32x4_t (&lo)[2][2][4],
                                         const i32x4_t (&f1)[2][2] = {}) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const i32x4_t (&f)[2][2] = (Mode & 16) && t >= 2 ? f1 : f0;  // measurement: tiles 2, 3 on the second fragments
    const int4 x0 = fr[(((s * 4 + t) * 2 + 0) * 64) + lane];
    const int4 x1 = fr[(((s * 4 + t) * 2 + 1) * 64) + lane];
    const i32x4_t chi = i32x4_t{x0.x, x0.y, x0.z, x0.w}, clo = i32x4_t{x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (Mode & 2) {
          hi[p][i][t] += f[p][i] + chi;
          lo[p][i][t] += f[p][i] + clo;
        } else {
          hi[p][i][t] = mfma_i8(chi, f[p][i], hi[p][i][t]);
          lo[p][i][t] = mfma_i8(clo, f[p][i], lo[p][i][t]);
        }
      }
  }
}

// The same 32 MFMAs with the next tile's two A fragments read from LDS while the current tile's MFMAs issue (two
// register sets): the single-set form made the compiler issue each tile's reads one MFMA before their use, so every
// step waited out the LDS latency four times (ISA: s_waitcnt lgkmcnt(1) between the MFMAs of consecutive tiles).
template <int Mode>
__device__ __forceinline__ void w32_mfma_pf(const int4* __restrict__ fr, int s, int lane, const i32x4_t (&f)[2][2],
                                            i32x4_t (&hi)[2][2][4], i32x4_t (&lo)[2][2][4]) {
  int4 a[2][2];  // [register set][limb]
  a[0][0] = fr[((s * 4 + 0) * 2 + 0) * 64 + lane];
  a[0][1] = fr[((s * 4 + 0) * 2 + 1) * 64 + lane];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t + 1 < 4) {
      a[(t + 1) & 1][0] = fr[((s * 4 + t + 1) * 2 + 0) * 64 + lane];
      a[(t + 1) & 1][1] = fr[((s * 4 + t + 1) * 2 + 1) * 64 + lane];
    }
    __builtin_amdgcn_sched_barrier(0);  // (else the scheduler sinks the reads back to one MFMA before their use)
    const int4 x0 = a[t & 1][0], x1 = a[t & 1][1];
    const i32x4_t chi = i32x4_t{x0.x, x0.y, x0.z, x0.w}, clo = i32x4_t{x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        hi[p][i][t] = mfma_i8(chi, f[p][i], hi[p][i][t]);
        lo[p][i][t] = mfma_i8(clo, f[p][i], lo[p][i][t]);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Mode (diagnostics only): 1 synthetic coefficients, 2 no MFMA, 4 no stores, 8 no voltage loads, 64 model loads
// without the phasor math, 256 the phasor math on register-made delays (no model loads).
template <bool Signed, int Mode = 0, bool Gain = false>
__global__ __launch_bounds__(kW8Threads, 2) void beamform_fused_i8_w32_kernel(FusedArgs P) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) int4 lds4[];
  // Mode 128 (diagnostics): per-wave s_memtime cycles of the phases -> P.gain as uint64 [wave][4]: coefficient
  // phase (to the barrier), contraction loops, requantise + stores, total
  unsigned long long st_t0 = 0, st_c = 0, st_l = 0, st_s = 0, st_m = 0;
  if constexpr ((Mode & 128) != 0) st_t0 = __builtin_amdgcn_s_memtime();
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  int slab, bc;
  if (P.xcd_order) {  // the slabs of one item back to back on one XCD: the second re-reads the voltages from L2
    const int x = blockIdx.x & 7, local = blockIdx.x >> 3;
    slab = local % P.nslabs;
    bc = (local / P.nslabs) * 8 + x;
    if (bc >= P.B * P.C) return;
  } else {
    slab = blockIdx.x % P.nslabs;
    bc = blockIdx.x / P.nslabs;
  }
  const int b = bc / P.C, c = bc % P.C;
  const int m0 = slab * kW32Beams;
  const int Sp = w32_steps(P.A);
  const int T2 = P.T >> 1;
  const int nchunks = (T2 + 15) >> 4;               // 32-sample chunks
  const int npasses = (nchunks + 3) >> 2;           // per wave, the same count for every wave
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const uint32_t hoff = static_cast<uint32_t>(8 * h) * static_cast<uint32_t>(ant_stride);  // < 24 * stride
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
  int8_t* lb = reinterpret_cast<int8_t*>(lds4);
  int* partial = reinterpret_cast<int*>(lb + static_cast<size_t>(Sp) * 4 * 2 * 64 * 16);  // [4 waves][32 columns]

  // the voltage prefetch: step ls of chunk lchunk next; runs on from one chunk into the wave's next one
  __builtin_assume(Sp >= 4 && (Sp & 3) == 0 && npasses >= 1);  // w32_steps, T >= 2: the 4 priming loads are real
  const int total = npasses * Sp;
  int issued = 0, ls = 0, lchunk = wave;
  // (past the wave's last step it repeats that step: the same, just-fetched bytes, and straight-line code)
  auto issue = [&](u32x2_t (&d)[8]) {
    const uint32_t loff = hoff + static_cast<uint32_t>(min(lchunk * 16 + tl, T2 - 1)) * 8u;
    w32_load<Mode>(base, ant_stride, loff, ls, P.A, d);
    // advance with selects, not branches: a branch here made the compiler re-home the step buffers through copies
    // (and wait for their loads) at the merge
    ++issued;
    const bool adv = issued < total;
    const bool wrap = ls + 1 == Sp;
    ls = adv ? (wrap ? 0 : ls + 1) : ls;
    lchunk = (adv && wrap) ? lchunk + 4 : lchunk;
  };
  // Q14 limbs of the slab's [[R, I], [-I, R]] blocks (as the 16-beam kernel), under the voltage loads.  Pair e -> 4
  // consecutive slot antennas x beam row ml = (tid >> 2) % 32, slot antenna sa0 + 8 J.  The first batch's delay
  // model is requested BEFORE the voltage prefetch (vmcnt counts in order: loaded after it, the first batch waited
  // for all 32 voltage loads before its phasors could start).
  const int ml = (tid >> 2) & (kW32Beams - 1);
  const int sa0 = 4 * (tid >> 7) + (tid & 3);
  const bool m_ok = m0 + ml < P.M;
  const float4* dv_row =
      P.dv + (static_cast<size_t>(P.delay_channels == 1 ? 0 : c) * P.M + min(m0 + ml, P.M - 1)) * P.A;
  // gains: the launch picks the Gain instantiation, so no branch sits between the loads and their use (a branch
  // around the gain loads made the compiler wait for every earlier load at the merge)
  const float* g_row = Gain ? P.gain + static_cast<size_t>(min(m0 + ml, P.M - 1)) * P.A : nullptr;
  constexpr int kBatch = 8;
  auto batch_model = [&](int j0, float4 (&dv)[kBatch], float (&gv)[kBatch]) {
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const int sa = sa0 + 8 * (j0 + j), st = sa >> 5;
      const int a = min(w8_step_base(st, P.A) + (sa & 31), P.A - 1);
      if constexpr ((Mode & 256) != 0) {  // diagnostics: no model loads, register-made delays (same math after)
        const float u = static_cast<float>(a * 37 + ml * 11 + j0);
        dv[j] = float4{u * 1e-10f, 0.0f, u * 1e-3f - 3.0f, 0.0f};
        gv[j] = 1.0f;
        continue;
      }
      dv[j] = dv_row[a];
      if constexpr (Gain)
        gv[j] = g_row[a];
      else
        gv[j] = 1.0f;
    }
  };
  float4 dv_first[kBatch];
  float gv_first[kBatch];
  if constexpr (!(Mode & 1)) batch_model(0, dv_first, gv_first);
  __builtin_amdgcn_sched_barrier(0);

  u32x2_t d0[8], d1[8], d2[8], d3[8];
  issue(d0);
  issue(d1);
  issue(d2);
  issue(d3);
  __builtin_amdgcn_sched_barrier(0);

  {
    const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
    const double ch = static_cast<double>(P.base_ch + c);
    const int nj = 4 * Sp;  // 32 Sp slot antennas x 32 beams / 256 threads
    int cs0 = 0, cs1 = 0;
    const int off0 = coef8_byte(2 * sa0, 2 * ml, 4, 0);
    // the model batches are software-pipelined: batch j0 + kBatch is requested before batch j0's phasors, so each
    // batch's (L2) load latency hides under the previous batch's float64 work -- measured per wave (s_memtime,
    // diagnostics Mode 128), four load-then-compute batches were 40 % of a wave's lifetime
    float4 dv[kBatch];
    float gv[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      dv[j] = dv_first[j];
      gv[j] = gv_first[j];
    }
    for (int j0 = 0; j0 < nj; j0 += kBatch) {
      float4 dvn[kBatch];
      float gvn[kBatch];
      if constexpr (!(Mode & 1)) batch_model(j0 + kBatch, dvn, gvn);  // clamped: past the end it rereads the row
      bool valid[kBatch];
      int wc[kBatch], ws[kBatch];
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        const int sa = sa0 + 8 * (j0 + j), st = sa >> 5;
        const int a = w8_step_base(st, P.A) + (sa & 31);
        valid[j] = j0 + j < nj && m_ok && a >= 32 * st;  // rows an earlier step already covered stay zero
      }
      if constexpr (Mode & 1) {
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          wc[j] = valid[j] ? 8192 + 16 * j + tid : 0;
          ws[j] = valid[j] ? 4096 - 16 * j : 0;
        }
      } else if constexpr ((Mode & 64) != 0) {  // diagnostics: model loads kept, a few VALU instead of the phasors
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          wc[j] = valid[j] ? (static_cast<int>(dv[j].x * 1e12f + dv[j].y) & 8191) : 0;
          ws[j] = valid[j] ? (static_cast<int>(dv[j].z * 1e3f + dv[j].w) & 8191) : 0;
        }
      } else {
        q14_coeffs<kBatch, true, false, true>(dv, gv, valid, ch, P.ctot, P.ts, P.k, dt, P.gain, wc, ws);
      }
#pragma unroll
      for (int j = 0; j < kBatch; ++j) {
        if (j0 + j >= nj) break;
        const int J = j0 + j;
        const int Wc = wc[j], Ws = ws[j], nWs = -Ws;
        // k = 2 sa0 + 16 J: step J >> 2, lane group J & 3 (2 sa0 < 16)
        int8_t* o = lb + off0 + 8192 * (J >> 2) + 256 * (J & 3);
        *reinterpret_cast<uint16_t*>(o) = static_cast<uint16_t>(__builtin_amdgcn_perm(nWs + 128, Wc + 128, 0x0c0c0501u));
        *reinterpret_cast<uint16_t*>(o + 64 * 16) = static_cast<uint16_t>(__builtin_amdgcn_perm(nWs, Wc, 0x0c0c0400u));
        *reinterpret_cast<uint16_t*>(o + 16) = static_cast<uint16_t>(__builtin_amdgcn_perm(Wc + 128, Ws + 128, 0x0c0c0501u));
        *reinterpret_cast<uint16_t*>(o + 16 + 64 * 16) = static_cast<uint16_t>(__builtin_amdgcn_perm(Wc, Ws, 0x0c0c0400u));
        cs0 += Wc - Ws;
        cs1 += Ws + Wc;
      }
      if constexpr (!(Mode & 1)) {
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          dv[j] = dvn[j];
          gv[j] = gvn[j];
        }
      }
    }
    if constexpr (!Signed) {
      cs0 += __shfl_xor(cs0, 1);
      cs1 += __shfl_xor(cs1, 1);
      cs0 += __shfl_xor(cs0, 2);
      cs1 += __shfl_xor(cs1, 2);
      if ((lane & 3) == 0) {  // wave w holds columns 32 (w & 1) + [0, 32)
        partial[wave * 32 + 2 * (lane >> 2)] = cs0;
        partial[wave * 32 + 2 * (lane >> 2) + 1] = cs1;
      }
    }
  }
  lds_barrier();  // the table is complete; the voltage prefetch stays in flight
  if constexpr ((Mode & 128) != 0) {
    st_m = __builtin_amdgcn_s_memtime();
    st_c = st_m - st_t0;
  }

  const float s32 = P.out_scale * 0x1p-14f;
  const int M2 = 2 * P.M;
  const bool full = m0 + kW32Beams <= P.M && (M2 & 15) == 0;  // 16-byte row pieces (uniform)
  int chunk = wave;
  for (int pass = 0; pass < npasses; ++pass) {
    const int tq = chunk * 16 + tl;  // sample pair
    i32x4_t hi[2][2][4], lo[2][2][4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) hi[p][i][t] = lo[p][i][t] = i32x4_t{0, 0, 0, 0};
    // four steps in flight; a step's buffer is reloaded as soon as its fragments are built
    if constexpr ((Mode & 128) != 0) st_m = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < Sp; s += 4) {
      i32x4_t f[2][2];
      w32_frags<Signed>(d0, f);
      issue(d0);
      w32_mfma<Mode>(lds4, s, lane, f, hi, lo);
      w32_frags<Signed>(d1, f);
      issue(d1);
      w32_mfma<Mode>(lds4, s + 1, lane, f, hi, lo);
      w32_frags<Signed>(d2, f);
      issue(d2);
      w32_mfma<Mode>(lds4, s + 2, lane, f, hi, lo);
      w32_frags<Signed>(d3, f);
      issue(d3);
      w32_mfma<Mode>(lds4, s + 3, lane, f, hi, lo);
    }
    if constexpr ((Mode & 128) != 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      st_l += t - st_m;
      st_m = t;
    }
    if constexpr (Mode & 4) {
      int sum = 0;
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 4; ++t) sum += hi[p][i][t][0] ^ lo[p][i][t][3];
      if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[tid] = sum;
    } else {
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        uint32_t pk[2][4];  // [sample i][tile t] -> 4 packed int8 columns 16 t + 4 h + r
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            uint32_t qb[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              int y = (hi[p][i][t][r] << 8) + lo[p][i][t][r];
              if constexpr (!Signed) {  // unsigned samples: 128 * the column sum (wave partials)
                const int cl = 16 * t + 4 * h + r;
                y += 128 * (partial[(cl >> 5) * 32 + (cl & 31)] + partial[((cl >> 5) + 2) * 32 + (cl & 31)]);
              }
              qb[r] = requant_bits(y, s32);
            }
            pk[i][t] = pack_low_bytes(qb[0], qb[1], qb[2], qb[3]);
          }
        const size_t prow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T);
        if (full) {
          // 4x4 transpose over (h, t): lane (tl, h) gets columns 16 h .. 16 h + 15 of sample 2 tq + i
#pragma unroll
          for (int i = 0; i < 2; ++i) transpose_rows4(pk[i]);
          if (tq < T2) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 2 * tq + i) * M2 + 2 * m0 + 16 * h;
              if constexpr ((Mode & 16) != 0)  // diagnostics: non-temporal stores
                __builtin_nontemporal_store(u32x4_t{pk[i][0], pk[i][1], pk[i][2], pk[i][3]},
                                            reinterpret_cast<u32x4_t*>(o));
              else
                *reinterpret_cast<u32x4_t*>(o) = u32x4_t{pk[i][0], pk[i][1], pk[i][2], pk[i][3]};
            }
          }
        } else if (tq < T2) {  // partial slab / unaligned rows: byte stores with the beam guard
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 2 * tq + i) * M2 + 2 * m0;
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int col = 16 * t + 4 * h + r;
                if (2 * m0 + col < M2) o[col] = static_cast<int8_t>((pk[i][t] >> (8 * r)) & 255);
              }
          }
        }
      }
    }
    if constexpr ((Mode & 128) != 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      st_s += t - st_m;
    }
    chunk += 4;
  }
  if constexpr ((Mode & 128) != 0) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(const_cast<float*>(P.gain)) +
                            (static_cast<size_t>(blockIdx.x) * 4 + wave) * 4;
    if (lane == 0) {
      o[0] = st_c;
      o[1] = st_l;
      o[2] = st_s;
      o[3] = __builtin_amdgcn_s_memtime() - st_t0;
    }
  }
}


// ---- the table-driven 32-beam kernel (the default with a workspace) -----------------------------------------------
// The Q14 coefficients come from the launch's table (q14_table_kernel, kLayoutW32: per (b, c, slab) 1024 Sp words,
// thread tid's units j = tid + 256 j as two 16-byte loads each) instead of phasors evaluated here, and a workgroup
// walks kCh consecutive channels of its slab (kW32TChannels; 8 at config 4's shape): the next channel's table is
// requested after the current channel's last MFMAs (its latency under the stores), and the voltage prefetch runs on
// from one channel into the next, so only a workgroup's first channel starts cold (measured on the one-channel form: a cold start -- table +
// first voltage steps -- per (channel, slab) cost ~50 us of 430 at config 4 in a round-3 ablation whose record was
// not kept).
// Mode (diagnostics): 1 no table loads / expansion, 4 no stores, 8 no voltage loads.
constexpr int kW32TChannels = 4;

// Early: request the next channel's table during the last pass's pol-1 stores (else after the last pass).
// kSp, kNP: compile-time k-steps and passes (config 4: 8 and 2; 0 = from the shape).  With both known, the channel's
// 16 steps are straight-line code: the four step buffers keep their registers, and the compiler no longer re-homes
// them through copies behind s_waitcnt vmcnt(22 .. 0) at every loop header -- a full drain of the voltage prefetch
// every four steps in the runtime-bounded form.
// BufLd: voltage loads through a buffer resource (w32_load_buf).  Pow2: the output scale is a power of two, so the
// requantisation's multiply and magic add fuse into one exact FMA (requant_bits<true>).
template <bool Signed, int Mode = 0, bool Early = true, int kSp = 0, int kNP = 0, int kNB = 4, int kCh = kW32TChannels,
          bool BufLd = false, bool Pow2 = false>
__global__ __launch_bounds__(kW8Threads, 2) void beamform_fused_i8_w32t_kernel(FusedArgs P) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) int4 lds4[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const int Cn = P.c_count ? P.c_count : P.C;  // channels of this launch (a chunk: pointers offset by the host)
  const int gpb = (Cn + kCh - 1) / kCh;  // channel groups per batch
  int slab, grp;
  if (P.xcd_order) {  // the slabs of one channel group back to back on one XCD: the second re-reads from L2
    const int x = blockIdx.x & 7, local = blockIdx.x >> 3;
    slab = local % P.nslabs;
    grp = (local / P.nslabs) * 8 + x;
    if (grp >= P.B * gpb) return;
  } else {
    slab = blockIdx.x % P.nslabs;
    grp = blockIdx.x / P.nslabs;
  }
  const int b = grp / gpb, c0 = (grp - b * gpb) * kCh;
  const int nk = min(kCh, Cn - c0);
  const int m0 = slab * kW32Beams;
  const int Sp = kSp ? kSp : w32_steps(P.A);
  const int T2 = P.T >> 1;
  const int nchunks = (T2 + 15) >> 4;                      // 32-sample chunks
  const int npasses = kNP ? kNP : (nchunks + 3) >> 2;  // per wave, the same count for every wave
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const uint32_t hoff = static_cast<uint32_t>(8 * h) * static_cast<uint32_t>(ant_stride);  // < 24 * stride
  const uint32_t ch_bytes = static_cast<uint32_t>(P.T) * 4;  // next channel of an antenna row
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * P.C + c0) * static_cast<size_t>(P.T) * 4;
  int8_t* lb = reinterpret_cast<int8_t*>(lds4);
  int* partial = reinterpret_cast<int*>(lb + static_cast<size_t>(Sp) * 4 * 2 * 64 * 16);  // [4 waves][64 columns]
  const u32x4_t* tbase = reinterpret_cast<const u32x4_t*>(P.table) +
                         ((static_cast<size_t>(b) * P.C + c0) * P.nslabs + slab) * 256 * Sp;
  const size_t tstride = static_cast<size_t>(P.nslabs) * 256 * Sp;  // u32x4 per channel

  // the voltage prefetch: step ls of pass lp of channel lk next, across the workgroup's channels
  __builtin_assume(Sp >= 4 && (Sp & 3) == 0 && npasses >= 1 && nk >= 1);
  const int total = nk * npasses * Sp;
  int issued = 0, ls = 0, lp = 0, lk = 0;
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, 0x7fffffff,
                                                                        0x00020000);
  auto issue = [&](u32x2_t (&d)[8]) {
    if constexpr (BufLd) {
      const uint32_t voff = hoff + static_cast<uint32_t>(min((wave + 4 * lp) * 16 + tl, T2 - 1)) * 8u;
      const uint32_t sbase = static_cast<uint32_t>(w8_step_base(ls, P.A)) * static_cast<uint32_t>(ant_stride) +
                             static_cast<uint32_t>(lk) * ch_bytes;
      w32_load_buf<Mode>(vrs, voff, sbase, static_cast<uint32_t>(ant_stride), d);
    } else {
      const uint32_t loff = hoff + static_cast<uint32_t>(lk) * ch_bytes +
                            static_cast<uint32_t>(min((wave + 4 * lp) * 16 + tl, T2 - 1)) * 8u;
      w32_load<Mode>(base, ant_stride, loff, ls, P.A, d);
    }
    ++issued;  // selects, not branches (see the one-channel kernel); past the last step it repeats that step
    const bool adv = issued < total;
    const bool wrap = ls + 1 == Sp, pwrap = lp + 1 == npasses;
    ls = adv ? (wrap ? 0 : ls + 1) : ls;
    lp = (adv && wrap) ? (pwrap ? 0 : lp + 1) : lp;
    lk = (adv && wrap && pwrap) ? lk + 1 : lk;
  };
  u32x4_t tq[4][2];  // this thread's table units of the channel being staged
  auto load_table = [&](int kc) {
    if constexpr ((Mode & 1) == 0) {
      // a buffer resource on the channel's (uniform) table block + 32-bit lane offsets: no 64-bit per-lane pointers
      // (hoisted out of the channel loop they were spilled)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<u32x4_t*>(tbase + static_cast<size_t>(kc) * tstride), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int j = 0; j < 4; ++j)  // Sp / 2 units (4 or 2); unconditional loads (clamped unit)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
          tq[j][hf] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rs, static_cast<uint32_t>(((min(j, Sp / 2 - 1) * 2 + hf) * 256 + tid) * 16), 0,
                                                      (Mode & 64) ? 2 : 0));  // (Mode 64, diagnostics: non-temporal)
    }
  };
  load_table(0);
  __builtin_amdgcn_sched_barrier(0);
  constexpr int NB = kSp ? kNB : 2;  // step buffers (NB - 1 steps in flight while one is contracted)
  u32x2_t db[NB][8];
#pragma unroll
  for (int j = 0; j < NB; ++j) issue(db[j]);
  __builtin_amdgcn_sched_barrier(0);

  const float s32 = P.out_scale * 0x1p-14f;
  const int M2 = 2 * P.M;
  const bool full = m0 + kW32Beams <= P.M && (M2 & 15) == 0;  // 16-byte row pieces (uniform)
  for (int kc = 0; kc < nk; ++kc) {
    const int c = c0 + kc;
    if constexpr ((Mode & 1) == 0) {  // the channel's table -> LDS limb image (+ unsigned column sums)
      const int ml = tid & 31;
      int cs0 = 0, cs1 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (2 * j >= Sp) break;  // uniform
        w32_expand_unit(lb, ml, (tid >> 5) + 8 * j, tq[j][0], tq[j][1]);
        if constexpr (!Signed) {
#pragma unroll
          for (int hf = 0; hf < 2; ++hf)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int wc = static_cast<int16_t>(tq[j][hf][q] & 0xffffu), ws = static_cast<int>(tq[j][hf][q]) >> 16;
              cs0 += wc - ws;
              cs1 += ws + wc;
            }
        }
      }
      if constexpr (!Signed) {  // + the other half-wave's antennas; one partial per wave and column
        cs0 += __shfl_xor(cs0, 32);
        cs1 += __shfl_xor(cs1, 32);
        if (lane < 32) {
          partial[wave * 64 + 2 * ml] = cs0;
          partial[wave * 64 + 2 * ml + 1] = cs1;
        }
      }
    }
    lds_barrier();  // the image is complete; the voltage prefetch stays in flight
    if constexpr (!Signed) {  // the four waves' partials -> one total per column
      if (tid < 64) partial[tid] += partial[64 + tid] + partial[128 + tid] + partial[192 + tid];
      lds_barrier();
    }
    // the passes; the last one is peeled so that the next channel's table registers are never live across an MFMA
    // loop (a conditional request inside the loop kept them live through every pass: 188 B/lane of spills)
    auto run_pass = [&](int pass, auto last) {
      constexpr bool kLast = decltype(last)::value;
      const int tq2 = (wave + 4 * pass) * 16 + tl;  // sample pair
      i32x4_t hi[2][2][4], lo[2][2][4];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 4; ++t) hi[p][i][t] = lo[p][i][t] = i32x4_t{0, 0, 0, 0};
      if constexpr (kSp != 0) {
        // straight-line: step g of the channel contracts buffer g % NB (compile-time), scheduling barriers keep each
        // step's refill after its fragments
#pragma unroll
        for (int s = 0; s < kSp; ++s) {
          constexpr int dummy = 0;
          (void)dummy;
          i32x4_t f[2][2], fi[2][2];
          const int j = (pass * kSp + s) % NB;
          w32_frags<Signed>(db[j], f);
          if constexpr ((Mode & 16) != 0) w32_frags_im(db[j], fi);
          __builtin_amdgcn_sched_barrier(0);
          issue(db[j]);
          if constexpr ((Mode & 32) != 0)
            w32_mfma_pf<0>(lds4, s, lane, f, hi, lo);
          else
            w32_mfma<Mode & 16>(lds4, s, lane, f, hi, lo, fi);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        // runtime step count (Sp a multiple of 4): the two-buffer ring, a pair of steps per iteration, so every
        // channel's steps start at buffer 0
        for (int s = 0; s < Sp; s += 2) {
          i32x4_t f[2][2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            w32_frags<Signed>(db[j], f);
            issue(db[j]);
            w32_mfma<0>(lds4, s + j, lane, f, hi, lo);
          }
        }
      }
      // unconditional in the last pass (the workgroup's last channel re-reads its own table, from L2): with a
      // conditional request the previous table's registers stayed live through every pass (phi at the back-edge)
      constexpr bool next_table = kLast && Early;
      if constexpr (Mode & 4) {
        if constexpr (next_table) load_table(min(kc + 1, nk - 1));
        int sum = 0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) sum += hi[p][i][t][0] ^ lo[p][i][t][3];
        if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[tid] = sum;
      } else {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          // the next channel's table, requested once pol 0's accumulators are dead (registers) -- its latency runs
          // under pol 1's stores and the barrier
          if constexpr (next_table)
            if (p == 1) {  // pinned: scheduled earlier, the loads overlapped pol 0's accumulators (spills)
              __builtin_amdgcn_sched_barrier(0);
              load_table(min(kc + 1, nk - 1));
              __builtin_amdgcn_sched_barrier(0);
            }
          uint32_t pk[2][4];  // [sample i][tile t] -> 4 packed int8 columns 16 t + 4 h + r
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              uint32_t qb[4];
              int4 cs = int4{0, 0, 0, 0};  // unsigned: the 4 columns' sums, one 16-byte LDS read
              if constexpr (!Signed) cs = reinterpret_cast<const int4*>(partial)[4 * t + h];
              const int csr[4] = {cs.x, cs.y, cs.z, cs.w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                int y = (hi[p][i][t][r] << 8) + lo[p][i][t][r];
                if constexpr (!Signed) y += 128 * csr[r];
                qb[r] = requant_bits<Pow2>(y, s32);
              }
              pk[i][t] = pack_low_bytes(qb[0], qb[1], qb[2], qb[3]);
            }
          const size_t prow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T);
          if (full) {
#pragma unroll
            for (int i = 0; i < 2; ++i) transpose_rows4(pk[i]);
            if (tq2 < T2) {
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 2 * tq2 + i) * M2 + 2 * m0 + 16 * h;
                *reinterpret_cast<u32x4_t*>(o) = u32x4_t{pk[i][0], pk[i][1], pk[i][2], pk[i][3]};
              }
            }
          } else if (tq2 < T2) {  // partial slab / unaligned rows: byte stores with the beam guard
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 2 * tq2 + i) * M2 + 2 * m0;
#pragma unroll
              for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int col = 16 * t + 4 * h + r;
                  if (2 * m0 + col < M2) o[col] = static_cast<int8_t>((pk[i][t] >> (8 * r)) & 255);
                }
            }
          }
        }
      }
    };
    if constexpr (Early) {
      if constexpr (kNP != 0) {
#pragma unroll
        for (int pass = 0; pass + 1 < kNP; ++pass) run_pass(pass, std::false_type{});
      } else {
        for (int pass = 0; pass + 1 < npasses; ++pass) run_pass(pass, std::false_type{});
      }
      run_pass(npasses - 1, std::true_type{});
    } else {
      if constexpr (kNP != 0) {
#pragma unroll
        for (int pass = 0; pass < kNP; ++pass) run_pass(pass, std::false_type{});
      } else {
        for (int pass = 0; pass < npasses; ++pass) run_pass(pass, std::false_type{});
      }
      load_table(min(kc + 1, nk - 1));
    }
    if constexpr (kSp != 0 && (kSp * kNP) % NB != 0) {  // re-align the ring: the next channel starts at buffer 0
      constexpr int r = (kSp * kNP) % NB;
      u32x2_t tmp[NB][8];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) tmp[j][q] = db[(j + r) % NB][q];
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) db[j][q] = tmp[j][q];
    }
    if (kc + 1 < nk) lds_barrier();  // every wave is done with this image (MFMAs) and column sums (stores)
  }
}

// ---- config 4's shape: a wave-private LDS-DMA voltage ring over the halved limb image (round 5) --------------------
// The table kernel above loads each wave-step's 4 KiB of voltages as 8 buffer_load_dwordx2 per lane (512 B per
// instruction): per CU and channel 1024 such instructions (both slabs) -- as many TA address cycles as the channel's
// MFMA cycles (SQ_VMEM_TA_ADDR_FIFO_FULL 1.06e8 per launch, r4_t).  Here a wave DMAs its step into LDS with four
// 1 KiB `buffer_load_dwordx4 ... lds` (half the TA cycles, no VGPR destination) and reads it back with eight
// ds_read_b64 in exactly the register layout of the table kernel.  The LDS for that comes from the halved image
// (y_re = [x_re, x_im].(Wc, -Ws), y_im = [x_im, ~x_re].(Wc, -Ws) + sum_a Ws -- same MFMAs, half the A fragments):
// 32 KiB of image + 2 x 16 KiB of slots + 512 B of column sums per workgroup, two workgroups per CU.
//   ring: step n's voltages in slot n & 1 of the wave (DMA'd two steps ahead); each step reads its slot, builds its
//         fragments, then DMAs step n + 2 into the same slot (the compiler counts the DMA in vmcnt and waits for it
//         before the slot's next read only: the slots are distinct __shared__ objects);
//   image: expanded from the kLayoutW32 table (the q14_table_kernel generator) into (Wc, -Ws) limb pairs after each
//         channel barrier, the slab's sum_a Ws per beam reduced through LDS (y_im's bias);
//   slot layout: antenna row 8h + q of the step at position 4q + h (128 B each), so the two lane halves of a
//         ds_read_b64 read adjacent 128 B rows (no bank conflict); the DMA writes lane-linearly, so the permutation
//         goes on its source address (lane i of instruction k: antenna 8((i >> 3) & 3) + 2k + (i >> 5), bytes
//         16 (i & 7) of the wave's 128-byte sample run).
// Shape: int8 voltages, 8 k-steps (224 < A <= 256), T = 256 (2 passes of 8 straight-line steps), M % 32 == 0,
// in-workgroup voltage offsets and the beams below 2^31 bytes; 8 channels per workgroup.
constexpr int kW32RChannels = 8;
__shared__ __attribute__((aligned(16))) int4 w32r_img[8 * 2 * 2 * 64];  // [step][tile][limb][lane] x 16 B
__shared__ __attribute__((aligned(16))) int4 w32r_slot0[4 * 256];       // [wave][4 KiB]: even steps
__shared__ __attribute__((aligned(16))) int4 w32r_slot1[4 * 256];       // odd steps
__shared__ __attribute__((aligned(16))) int w32r_ws[4 * 32];            // [wave][beam] partial sum_a Ws

typedef __attribute__((address_space(3))) void* lds_void_ptr;

// One table unit (beam ml, slot-antenna group g: step g >> 2, lane group g & 3) -> the halved image's two entries:
// per antenna the (Wc, -Ws) pair as balanced limbs (lo = byte 0 as int8, hi = byte 1 of W + 128), w32_expand_unit's
// column-2 ml entries at the halved layout's place.
__device__ __forceinline__ void w32r_expand_unit(int4* img, int ml, int g, const u32x4_t& q0, const u32x4_t& q1) {
  const uint32_t d[8] = {q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], q1[2], q1[3]};
  uint32_t n[8], np[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const u16x2_t neg = __builtin_bit_cast(u16x2_t, d[i]) * u16x2_t{1, 0xffff};  // (Wc, -Ws)
    n[i] = __builtin_bit_cast(uint32_t, neg);
    np[i] = __builtin_bit_cast(uint32_t, neg + u16x2_t{128, 128});
  }
  u32x4_t ehi, elo;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    elo[q] = __builtin_amdgcn_perm(n[2 * q + 1], n[2 * q], 0x06040200u);
    ehi[q] = __builtin_amdgcn_perm(np[2 * q + 1], np[2 * q], 0x07050301u);
  }
  int4* o = img + ((g >> 2) * 2 + (ml >> 4)) * 2 * 64 + (ml & 15) + 16 * (g & 3);
  o[0] = __builtin_bit_cast(int4, ehi);
  o[64] = __builtin_bit_cast(int4, elo);
}

// y_im's B fragment from y_re's: [x_re, x_im, ...] -> [x_im, ~x_re, ...] per antenna (~x = -x - 1 stays in int8).
__device__ __forceinline__ i32x4_t w32r_frag_im(const i32x4_t& f) {
  i32x4_t r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t n = static_cast<uint32_t>(f[q]) ^ 0x00ff00ffu;
    r[q] = static_cast<int>(__builtin_amdgcn_perm(n, n, 0x02030001u));
  }
  return r;
}

// Mode (diagnostics only): 4 no stores, 8 no voltage DMA (the slots' stale bytes), 16 no table loads / expansion,
// 32 the step's four DMA pieces issued as one burst before its MFMAs (the product spreads them, one per 8 MFMAs),
// 64 a pass's four beam stores back to back after its requantisation; 128 the DMA pieces issued through a
// zero-record descriptor (the instructions and waits stay, no bytes move: their issue cost alone), 256 the same for
// the beam stores; 512 the four pieces of a step at one M0 (the LDS offset in the instruction's immediate, the
// global offset compensated in soffset); 1024 every channel's voltages from the workgroup's first channel (L2
// hits after the first), 2048 every beam store into one of 256 8 KiB blocks (L2-resident writes), 4096 the second
// slab's voltage DMA through a zero-record descriptor (one slab's bytes through the CU path: wrong beams for it).
template <bool Pow2, int Mode = 0>
__global__ __launch_bounds__(kW8Threads, 2) void beamform_fused_i8_w32r_kernel(FusedArgs P) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  constexpr int Sp = 8, NP = 2, kCh = kW32RChannels;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, tl = lane & 15;
  const int C = P.C;
  const int gpb = (C + kCh - 1) / kCh;  // channel groups per batch
  int slab, grp;
  if (P.xcd_order) {  // the slabs of one channel group back to back on one XCD: the second re-reads from L2
    const int x = blockIdx.x & 7, local = blockIdx.x >> 3;
    slab = local % P.nslabs;
    grp = (local / P.nslabs) * 8 + x;
    if (grp >= P.B * gpb) return;
  } else {
    slab = blockIdx.x % P.nslabs;
    grp = blockIdx.x / P.nslabs;
  }
  const int b = grp / gpb, c0 = (grp - b * gpb) * kCh;
  const int nk = min(kCh, C - c0);
  const int m0 = slab * kW32Beams;
  const uint32_t ant_stride = static_cast<uint32_t>(C) * static_cast<uint32_t>(P.T) * 4u;  // host: A C T 4 < 2^31
  const uint32_t ch_bytes = static_cast<uint32_t>(P.T) * 4u;
  const uint8_t* base = P.raw + (static_cast<size_t>(b) * P.A * C + c0) * static_cast<size_t>(P.T) * 4;
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(base), 0, ((Mode & 128) || ((Mode & 4096) && slab == 1)) ? 0 : 0x7fffffff, 0x00020000);
  const uint32_t dma_voff = static_cast<uint32_t>(8 * ((lane >> 3) & 3) + (lane >> 5)) * ant_stride +
                            16u * static_cast<uint32_t>(lane & 7);
  int4* const slot0 = w32r_slot0 + 256 * wave;
  int4* const slot1 = w32r_slot1 + 256 * wave;

  // the voltage ring: step ls of pass lp of channel lk is DMA'd next (past the last step it repeats that step)
  const int total = nk * NP * Sp;
  int issued = 0, ls = 0, lp = 0, lk = 0;
  // the step's uniform source offset, one 1 KiB piece of its DMA, and the ring's advance (selects, not branches)
  auto dma_sb = [&]() {
    // (readfirstlane: a loop-carried part of it landed in a VGPR, and the DMA's soffset then became a waterfall loop)
    return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(w8_step_base(ls, P.A)) * ant_stride +
                                          static_cast<uint32_t>((Mode & 1024) ? 0 : lk) * ch_bytes +
                                          static_cast<uint32_t>(wave + 4 * lp) * 128u);
  };
  auto dma_piece = [&](int4* slot, int k, uint32_t sb) {
    if constexpr ((Mode & 8) == 0) {
      if constexpr ((Mode & 512) != 0) {
        const uint32_t so = sb + 2u * static_cast<uint32_t>(k) * ant_stride - 1024u * k;
        switch (k) {  // (the immediate must be a constant: k is one after unrolling)
#define BF_W32R_DMA(K) \
  case K: __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lds_void_ptr)slot, 16, dma_voff, so, 1024 * K, 0); break;
          BF_W32R_DMA(0) BF_W32R_DMA(1) BF_W32R_DMA(2) BF_W32R_DMA(3)
#undef BF_W32R_DMA
        }
      } else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(vrs, (lds_void_ptr)(slot + 64 * k), 16, dma_voff,
                                                 sb + 2u * static_cast<uint32_t>(k) * ant_stride, 0, 0);
    }
  };
  auto advance = [&]() {
    ++issued;
    const bool adv = issued < total;
    const bool wrap = ls + 1 == Sp, pwrap = lp + 1 == NP;
    ls = adv ? (wrap ? 0 : ls + 1) : ls;
    lp = (adv && wrap) ? (pwrap ? 0 : lp + 1) : lp;
    lk = (adv && wrap && pwrap) ? lk + 1 : lk;
  };
  auto dma = [&](int4* slot) {
    const uint32_t sb = dma_sb();
#pragma unroll
    for (int k = 0; k < 4; ++k) dma_piece(slot, k, sb);
    advance();
  };
  // this lane's 8 antenna rows x its sample pair from the wave's slot: the table kernel's register layout
  auto read_slot = [&](const int4* slot, u32x2_t (&d)[8]) {
    const u32x2_t* s2 = reinterpret_cast<const u32x2_t*>(slot);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] = s2[(4 * q + h) * 16 + tl];
  };

  // the channel's table units (kLayoutW32: two 16-byte loads per unit, a buffer resource on the channel's block)
  const u32x4_t* tbase = reinterpret_cast<const u32x4_t*>(P.table) +
                         ((static_cast<size_t>(b) * C + c0) * P.nslabs + slab) * 256 * Sp;
  const size_t tstride = static_cast<size_t>(P.nslabs) * 256 * Sp;  // u32x4 per channel
  u32x4_t tq[4][2];
  auto load_table = [&](int kc) {
    if constexpr ((Mode & 16) == 0) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<u32x4_t*>(tbase + static_cast<size_t>(kc) * tstride), 0, 0x7fffffff, 0x00020000);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
          tq[j][hf] = __builtin_bit_cast(
              u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<uint32_t>(((j * 2 + hf) * 256 + tid) * 16), 0, 0));
    }
  };
  // the image of the staged channel + this wave's partial sum_a Ws per beam (lanes ml and ml + 32 hold the same beam)
  auto expand = [&]() {
    if constexpr ((Mode & 16) == 0) {
      const int ml = tid & 31;
      int ws = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        w32r_expand_unit(w32r_img, ml, (tid >> 5) + 8 * j, tq[j][0], tq[j][1]);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
#pragma unroll
          for (int q = 0; q < 4; ++q) ws += static_cast<int>(tq[j][hf][q]) >> 16;
      }
      ws += __shfl_xor(ws, 32);
      if (lane < 32) w32r_ws[32 * wave + ml] = ws;
    }
  };

  load_table(0);
  __builtin_amdgcn_sched_barrier(0);
  dma(slot0);
  dma(slot1);
  __builtin_amdgcn_sched_barrier(0);
  expand();
  lds_barrier();

  const float s32 = P.out_scale * 0x1p-14f;
  const int M2 = 2 * P.M;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(P.y, 0, (Mode & 256) ? 0 : 0x7fffffff,
                                                                        0x00020000);
  // the lane's part of a beam-row store offset (sample 2 tl + i of the wave's 32, row piece of lane group h)
  const uint32_t so_lane = static_cast<uint32_t>(2 * tl * M2 + 16 * (h >> 1) + 32 * (h & 1));
  for (int kc = 0; kc < nk; ++kc) {
    const int c = c0 + kc;
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      i32x4_t rh[2][2][2], rl[2][2][2], ih[2][2][2], il[2][2][2];  // [pol][sample i][tile]
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int t = 0; t < 2; ++t) rh[p][i][t] = rl[p][i][t] = ih[p][i][t] = il[p][i][t] = i32x4_t{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < Sp; ++s) {
        int4* const slot = (s & 1) ? slot1 : slot0;  // (16 steps per channel: the parity is the step's)
        u32x2_t d[8];
        read_slot(slot, d);
        i32x4_t f[2][2], fi[2][2];
        w32_frags<true>(d, f);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 2; ++i) fi[p][i] = w32r_frag_im(f[p][i]);
        // the slot's reads have returned (its bytes are in the fragments) before the DMA that refills it is issued:
        // nothing else orders a ds_read before a later LDS-DMA write to the same bytes (WAR)
        asm volatile("" ::"v"(f[0][0]), "v"(f[0][1]), "v"(f[1][0]), "v"(f[1][1]) : "memory");
        __builtin_amdgcn_sched_barrier(0);
        const uint32_t sb = dma_sb();
        if constexpr ((Mode & 32) != 0) {  // (diagnostics: the four pieces as one burst -- 370.0 vs 362.7 us spread)
#pragma unroll
          for (int k = 0; k < 4; ++k) dma_piece(slot, k, sb);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int4 x0 = w32r_img[((s * 2 + t) * 2 + 0) * 64 + lane];
          const int4 x1 = w32r_img[((s * 2 + t) * 2 + 1) * 64 + lane];
          const i32x4_t ahi = i32x4_t{x0.x, x0.y, x0.z, x0.w}, alo = i32x4_t{x1.x, x1.y, x1.z, x1.w};
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            if constexpr ((Mode & 32) == 0) {  // one DMA piece per 8 MFMAs, not a burst of 4 (-2 %, r5_ab1)
              __builtin_amdgcn_sched_barrier(0);
              dma_piece(slot, 2 * t + p, sb);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              rh[p][i][t] = mfma_i8(ahi, f[p][i], rh[p][i][t]);
              rl[p][i][t] = mfma_i8(alo, f[p][i], rl[p][i][t]);
              ih[p][i][t] = mfma_i8(ahi, fi[p][i], ih[p][i][t]);
              il[p][i][t] = mfma_i8(alo, fi[p][i], il[p][i][t]);
            }
          }
        }
        advance();
        __builtin_amdgcn_sched_barrier(0);
      }
      // the next channel's table, requested after the last pass's MFMAs (its latency under the stores and barrier)
      if (pass == NP - 1) {
        __builtin_amdgcn_sched_barrier(0);
        load_table(min(kc + 1, nk - 1));
        __builtin_amdgcn_sched_barrier(0);
      }
      // requantise + store: lane (tl, h) holds beams 16 t + 4 h + r (re and im) of samples 2 tq2 + i; per tile two
      // dwords [re, im, re, im] = bytes [32 t + 8 h, + 8) of the slab's 64-byte row; one permlane16_swap per dword
      // pair gives lane group h the 16 bytes at 16 (h >> 1) + 32 (h & 1).
      int bias[2][4];  // -sum_a Ws of beams 16 t + 4 h + r (y_im's bias)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        int4 acc = int4{0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int4 v = *reinterpret_cast<const int4*>(w32r_ws + 32 * w + 16 * t + 4 * h);
          acc.x += v.x;
          acc.y += v.y;
          acc.z += v.z;
          acc.w += v.w;
        }
        bias[t][0] = -acc.x;
        bias[t][1] = -acc.y;
        bias[t][2] = -acc.z;
        bias[t][3] = -acc.w;
      }
      if constexpr ((Mode & 4) != 0) {
        int sum = 0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int t = 0; t < 2; ++t) sum += rh[p][i][t][0] ^ rl[p][i][t][1] ^ ih[p][i][t][2] ^ il[p][i][t][3] ^ bias[t][p];
        if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[tid] = sum;
      } else {
        u32x4_t sd[2][2];  // [pol][sample i]: the 16 store bytes of this lane
        uint32_t soff[2][2];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const uint32_t prow = static_cast<uint32_t>(((b * 2 + p) * C + c) * P.T);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            uint32_t pk[2][2];  // [tile][dword]
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              uint32_t qr[4], qi[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                qr[r] = requant_bits<Pow2>((rh[p][i][t][r] << 8) + rl[p][i][t][r], s32);
                qi[r] = requant_bits<Pow2>((ih[p][i][t][r] << 8) + il[p][i][t][r] + bias[t][r], s32);
              }
              pk[t][0] = pack_low_bytes(qr[0], qi[0], qr[1], qi[1]);
              pk[t][1] = pack_low_bytes(qr[2], qi[2], qr[3], qi[3]);
            }
            const auto sw0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
            const auto sw1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
            sd[p][i] = u32x4_t{sw0[0], sw1[0], sw0[1], sw1[1]};
            soff[p][i] = (prow + static_cast<uint32_t>(2 * (wave + 4 * pass) * 16 + i)) * static_cast<uint32_t>(M2) +
                         static_cast<uint32_t>(2 * m0);
            if constexpr ((Mode & 2048) != 0) soff[p][i] = static_cast<uint32_t>(blockIdx.x & 255) * 8192u;
            if constexpr ((Mode & 64) == 0) {
              __builtin_amdgcn_raw_buffer_store_b128(sd[p][i], yrs, so_lane, soff[p][i], 0);
              // Two wait states before any VALU may rewrite the store's data VGPRs: hipcc scheduled a write of its
              // 4th data register right behind this store, and that dword of lanes 12-15 of every row went out
              // wrong (~1e-5 of the bytes, run to run; tools/diag_w32r.py, tools/store_hazard_check.py).
              __builtin_amdgcn_sched_barrier(0);
              asm volatile("s_nop 1");
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        if constexpr ((Mode & 64) != 0) {  // (diagnostics: the pass's four stores back to back, one guard)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int i = 0; i < 2; ++i) __builtin_amdgcn_raw_buffer_store_b128(sd[p][i], yrs, so_lane, soff[p][i], 0);
          __builtin_amdgcn_sched_barrier(0);
          asm volatile("s_nop 1");
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    if (kc + 1 < nk) {
      lds_barrier();  // every wave is done with this channel's image and column sums
      expand();
      lds_barrier();
    }
  }
  // The ring's last two DMAs (the last step again, unread) must land before the wave ends: an LDS-DMA still in
  // flight when the workgroup's LDS is handed to the next workgroup on this CU would write into that workgroup's slots.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

#ifdef BF_DIAG
#include "diag/wide_i8_w32h.inc"  // round 4's halved-image kernel (diagnostic build only)
#include "diag/wide_i8_w32r3.inc"  // round 6's three-slot ring (measured slower; diagnostic build only)
#include "diag/wide_i8_w32s.inc"  // round 6's loader-wave form (measured slower; diagnostic build only)
#endif

template <bool Signed, int Mode>
int launch_w32t_contract(FusedArgs P, hipStream_t st);
#ifdef BF_DIAG
template <bool Signed, int Mode>
int launch_w32_overlapped(FusedArgs P, int k, hipStream_t st);
#endif

// The LDS-DMA ring contraction's shape (beamform_fused_i8_w32r_kernel): 8 k-steps, T = 256, whole 32-beam slabs,
// every in-workgroup voltage offset and every beam offset below 2^31, a whole launch (no channel chunk).
bool w32r_fits(const FusedArgs& P) {
  return w32_steps(P.A) == 8 && P.A > 224 && P.T == 256 && P.M % kW32Beams == 0 && P.c_count == 0 &&
         static_cast<unsigned long long>(P.A) * P.C * P.T * 4 < (1ull << 31) &&
         static_cast<unsigned long long>(P.B) * 2 * P.C * P.T * 2 * P.M < (1ull << 31);
}

// The LDS-DMA ring contraction of one launch whose kLayoutW32 table is ready in P.table on `st` (int8 voltages).
template <int Mode = 0>
int launch_w32r_contract(FusedArgs P, hipStream_t st) {
  const long long groups = static_cast<long long>(P.B) * ((P.C + kW32RChannels - 1) / kW32RChannels);
  const long long grid = P.xcd_order ? (groups + 7) / 8 * 8 * P.nslabs : groups * P.nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
  if (scale_is_pow2(P.out_scale * 0x1p-14f))
    hipLaunchKernelGGL((beamform_fused_i8_w32r_kernel<true, Mode>), dim3(static_cast<unsigned>(grid)),
                       dim3(kW8Threads), 0, st, P);
  else
    hipLaunchKernelGGL((beamform_fused_i8_w32r_kernel<false, Mode>), dim3(static_cast<unsigned>(grid)),
                       dim3(kW8Threads), 0, st, P);
  BF_LAUNCHED("beamform_fused_i8_w32r_kernel");
}

template <bool Signed, int Mode = 0>
int launch_w32(FusedArgs P, hipStream_t st) {
  const size_t lds = w32_lds_bytes(P.A);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform_fused: n_ants=%d too large for the integer wide kernel", P.A);
  P.nslabs = (P.M + kW32Beams - 1) / kW32Beams;
  P.xcd_order = P.nslabs > 1 && P.order != BF_FUSED_ORDER_CHANNEL;
  const long long items = static_cast<long long>(P.B) * P.C;
  const long long grid = P.xcd_order ? (items + 7) / 8 * 8 * P.nslabs : items * P.nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform_fused: grid too large");
  if (P.table && w32_table_fits(P.A) && P.table_bytes >= w32_table_bytes(P.B, P.C, P.A, P.M)) {
    // the coefficient table of this launch, written by q14_table_kernel just before on `st`
#ifdef BF_DIAG
    // measurement (BF_W32_CHUNKS): generator and contraction alternated over channel chunks
    const char* ck = diag_env("BF_W32_CHUNKS");
    const int nchunks = ck ? std::max(1, atoi(ck)) : 1;
    if (nchunks > 1 && P.B == 1 && P.c_count == 0 && P.delay_channels == 1) {
      const int per = (P.C + nchunks - 1) / nchunks;
      for (int c0 = 0; c0 < P.C; c0 += per) {
        FusedArgs Q = P;
        Q.c_count = std::min(per, P.C - c0);
        Q.raw = P.raw + static_cast<size_t>(c0) * P.T * 4;
        Q.y = static_cast<int8_t*>(P.y) + static_cast<size_t>(c0) * P.T * 2 * P.M;
        Q.table = P.table + static_cast<size_t>(c0) * ((P.M + 31) / 32) * 1024 * w32_table_steps(P.A);
        Q.base_ch = P.base_ch + c0;
        const int e = launch_w32<Signed, Mode>(Q, st);
        if (e != BF_OK) return e;
      }
      return BF_OK;
    }
    // measurement (BF_W32_OVERLAP = k chunks): the generator's chunks on a second stream, each chunk's contraction
    // on the caller's stream after its chunk of the table.  Measured slower than the serial pair (round 4,
    // profiles/r4_s_overlap_ab.txt: 2 / 4 / 8 chunks 494 / 505 / 843 vs 478 us, bitwise equal), so diagnostic only.
    const char* ov = diag_env("BF_W32_OVERLAP");
    const int nover = ov ? std::min(16, std::max(1, atoi(ov))) : 1;
    if (nover > 1 && P.B == 1 && P.c_count == 0 && P.delay_channels == 1)
      return launch_w32_overlapped<Signed, Mode>(P, nover, st);
    // measurement (BF_W32H=1): the halved-image generator + the w32h contraction at config 4's shape -- bitwise equal
    // to the table kernel, measured no faster (profiles/r4_*)
    if (Mode == 0 && w32h_fits(P) && diag_env("BF_W32H")) {
      const int e = launch_q14_table(P, const_cast<uint32_t*>(P.table), kLayoutW32H, st);
      if (e != BF_OK) return e;
      return launch_w32h_contract<Signed>(P, st);
    }
#endif
    const int e = launch_q14_table(P, const_cast<uint32_t*>(P.table), kLayoutW32, st);
    if (e != BF_OK) return e;
    if constexpr (Signed && Mode == 0)
      if (w32r_fits(P)) return launch_w32r_contract(P, st);  // config 4's shape: the LDS-DMA voltage ring
    return launch_w32t_contract<Signed, Mode>(P, st);
  }
  if (P.gain)
    hipLaunchKernelGGL((beamform_fused_i8_w32_kernel<Signed, Mode, true>), dim3(static_cast<unsigned>(grid)),
                       dim3(kW8Threads), lds, st, P);
  else
    hipLaunchKernelGGL((beamform_fused_i8_w32_kernel<Signed, Mode, false>), dim3(static_cast<unsigned>(grid)),
                       dim3(kW8Threads), lds, st, P);
  BF_LAUNCHED("beamform_fused_i8_w32_kernel");
}

// The table-driven contraction of one launch (or channel chunk: P.c_count, pointers offset by the caller) whose
// kLayoutW32 table is ready in P.table on `st`.
template <bool Signed, int Mode>
int launch_w32t_contract(FusedArgs P, hipStream_t st) {
  const size_t lds = w32_lds_bytes(P.A);
  {
    const int Cn = P.c_count ? P.c_count : P.C;
    const int npasses = ((((P.T >> 1) + 15) >> 4) + 3) >> 2;
    // config 4's shape walks 8 channels per workgroup (385.5 vs 389.4 us for 4, profiles/r3_ad*), the others 4
    const bool straight = w32_steps(P.A) == 8 && npasses == 2;
    const int ch = straight ? 8 : kW32TChannels;
    const long long groups = static_cast<long long>(P.B) * ((Cn + ch - 1) / ch);
    const long long tgrid = P.xcd_order ? (groups + 7) / 8 * 8 * P.nslabs : groups * P.nslabs;
    // buffer-resource voltage loads (no per-load VALU addressing) while every in-workgroup offset is below 2^31
    const bool buf = static_cast<unsigned long long>(P.A) * P.C * P.T * 4 < (1ull << 31);
    // a power-of-two scale: the requantisation's multiply and magic add as one exact FMA
    const bool pow2 = scale_is_pow2(P.out_scale * 0x1p-14f);
    const dim3 grid3(static_cast<unsigned>(tgrid)), block(kW8Threads);
    // config 4's shape: the straight-line ring, two step buffers (one step in flight while one is contracted):
    // 377 vs 384 us for three buffers and 403 for the runtime loop (profiles/r3_ab_*, r3_g_*)
    if (straight && buf && pow2)
      hipLaunchKernelGGL((beamform_fused_i8_w32t_kernel<Signed, Mode, false, 8, 2, 2, 8, true, true>), grid3, block,
                         lds, st, P);
    else if (straight && buf)
      hipLaunchKernelGGL((beamform_fused_i8_w32t_kernel<Signed, Mode, false, 8, 2, 2, 8, true, false>), grid3, block,
                         lds, st, P);
    else if (buf)
      hipLaunchKernelGGL((beamform_fused_i8_w32t_kernel<Signed, Mode, false, 0, 0, 4, kW32TChannels, true, false>),
                         grid3, block, lds, st, P);
    else  // offsets past 2^31 (A C T 4 >= 2 GiB): the pointer form
      hipLaunchKernelGGL((beamform_fused_i8_w32t_kernel<Signed, Mode, false>), grid3, block, lds, st, P);
    BF_LAUNCHED("beamform_fused_i8_w32t_kernel");
  }
}

#ifdef BF_DIAG
#include "diag/wide_i8_overlap.inc"  // generator / contraction overlap (measured slower)
#endif

}  // namespace

bool i8_w32_fits(const FusedArgs& P) {
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  return P.A >= 32 && (P.T & 1) == 0 && 24 * ant_stride + static_cast<size_t>(P.T) * 4 < (1ull << 32) &&
         w32_lds_bytes(P.A) <= kMaxLds;
}

template <bool Signed>
int launch_i8_w32(FusedArgs P, hipStream_t st) {
  return launch_w32<Signed>(P, st);
}

template int launch_i8_w32<false>(FusedArgs, hipStream_t);
template int launch_i8_w32<true>(FusedArgs, hipStream_t);

}  // namespace bf

#ifdef BF_DIAG
#include "diag/wide_i8_entries.inc"
#endif
