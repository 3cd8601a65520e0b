// DIAGNOSTIC BUILD ONLY (-DBF_DIAG, tools/diag_fused.py w32t modes 700+ / 800+): a measured and rejected design
// for config 4's int8 beams, kept as the record of its A/B (profiles/r3_s_*, r3_t_*, r3_uvw_*).  At config 4 it ran
// 425-468 us against the slab kernel's 392-415 us in the same processes, bitwise equal; its compute floor alone (no
// DMA, no stores) was 190-230 us -- the two-limb MFMAs at the clock the chip holds under them, plus a barrier and an
// LDS round trip per k-step that did not hide.
//
// Integer wide fused beamformer, config 4's shape (A % 32 == 0, A <= 256, 64 beams, T = 256, signed samples):
// output-stationary over half items, one 8-wave workgroup per CU walking a contiguous run of (b, c, sample half)
// units, every operand staged in LDS by LDS-DMA.  Same integer contract as the 32-beam slab kernels
// (oracle.fused_beamform_int8: Q14 coefficients of the exact float32 phasors from q14_table_kernel's kLayoutW32
// table, exact int32 sums, one float rounding to int8).
//
// Why: the slab kernel (bf_wide_i8.hip, beamform_fused_i8_w32t_kernel) loads its voltages
// into registers as 8-byte lane runs of 8 antenna rows -- 4 pieces of 128 B per wave-instruction, each item's 256 KiB
// read twice (once per 32-beam slab) -- and is bound by that load latency (TA address FIFO full, no-load ablation
// 237 of 395 us).  Here one `global_load_lds_dwordx4` moves two antennas' 512-byte half runs (128 samples x 2 pols) of
// a channel straight into LDS, each voltage byte is read from HBM once for all 64 beams, and nothing waits in VGPRs.
//
// Unit = (b, c, half h2: samples [128 h2, 128 h2 + 128)): 256 rows (samples x pols) x 128 real columns (64 beams).
// Per k-step (32 antennas): 16 KiB of voltage half runs (2 DMAs per wave) + 8 KiB of Q14 table units (1 DMA per
// wave), four of each in a ring (three steps in flight); the table is expanded once per workgroup into a 16 KiB
// two-limb image (two in a ring); wave (sg, bh) contracts 64 rows (32 samples x 2 pols) x 64 columns (32 beams): 8
// ds_read_b64 of voltages (2 samples x 2 pols x 2 bytes of one antenna per read), one v_perm per fragment dword, 8
// limb fragments from the image, 32 v_mfma_i32_16x16x64_i8 into separate hi / lo int32 accumulators (128 registers,
// combined once per unit as (hi << 8) + lo).  A whole item per workgroup (design A: 128 rows per wave, the hi
// product folded into the accumulator every step) measured no faster than the slab kernel (404 vs 402 us): the fold
// (128 VALU per wave-step) did not hide under the MFMAs (profiles/r3_t_os_fullitem_ablation_pmc.txt).
// The item's table is read once per half (the second time from L2 / the Infinity Cache, 8 steps later).
//
// Pipeline (flattened over the workgroup's units x k-steps, g = 0 .. G-1), one barrier per step, R-deep rings:
//   wait for D(g), T(g+1) (counted vmcnt) -> barrier -> issue T(g+R), D(g+R-1) -> expand T(g+1) -> contract step g
//   [-> requantise + store the unit after its last step].
// The DMAs are issued from inline asm: with the builtin, hipcc inserts s_waitcnt vmcnt(0) before every ds_read that
// may alias an in-flight LDS-DMA, which drains the ring at every step.  The kernel has no other global loads, so the
// compiler's own counted waits (it sees none of these DMAs) stay correct: completions are in order.
// LDS image of the voltages: antenna q's 512-byte half run in slot q, rotated by 128 B for (q >> 3) odd, so the two
// 16-lane groups of a ds_read_b64 lane half (antennas 8 g4 + ...) hit different banks.
#include <algorithm>
#include <cstdlib>

#include "../bf_fused.hpp"

#ifdef BF_DIAG
namespace bf {

namespace {

// NW = 8: one 512-thread workgroup per CU, unit = (b, c, sample half), both 32-beam slabs (wave = (sg, bh)).
// NW = 4: two 256-thread workgroups per CU, unit = (b, c, sample half) x one slab (the workgroup's bh); the two
// slabs of a unit run on workgroups w and w + 8 (same XCD, started together: the second voltage read from L2).
template <int NW>
struct OsCfg {
  static constexpr int kThreads = 64 * NW;
  static constexpr int kR = NW == 8 ? 4 : 3;             // ring depth of the voltage and table stages
  static constexpr int kVBytes = 16 * 1024;              // one k-step's voltages: 32 antenna half runs of 512 B
  static constexpr int kTBytes = NW == 8 ? 8192 : 4096;  // one k-step's table units: slabs x 128 units x 32 B
  static constexpr int kCBytes = NW == 8 ? 16384 : 8192; // limb image: tiles x 2 limbs x 64 lanes x 16 B
  static constexpr int kLds = kR * (kVBytes + kTBytes) + 2 * kCBytes;  // 128 KiB (NW 8) / 76 KiB (NW 4)
  static constexpr int kVG = 16 / NW;                    // voltage DMAs per wave and step (2 antennas each)
};

// One 16-byte-per-lane LDS-DMA: lane l's 16 bytes at gp land at LDS byte lds + 16 l (lds wave-uniform).
__device__ __forceinline__ void glds16(const void* gp, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gp),
               "s"(__builtin_amdgcn_readfirstlane(lds))
               : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt");
  // vmcnt(N), expcnt(7), lgkmcnt(15): only the vector-memory counter
  __builtin_amdgcn_s_waitcnt(0x0f70 | N);
}

// Half a table unit (4 of its 8 slot antennas, one 16-byte load of the kLayoutW32 table) into the limb image: the
// same entries as w32_expand_unit (bf_wide_i8.hip), 8 of each entry's 16 bytes.
__device__ __forceinline__ void os_expand_half(int8_t* img, int ml, int h, int hf, int slab, const u32x4_t& q) {
  typedef uint16_t u16x2_t __attribute__((ext_vector_type(2)));
  const uint32_t d[4] = {q[0], q[1], q[2], q[3]};
  uint32_t n[4], np[4], pp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const u16x2_t v = __builtin_bit_cast(u16x2_t, d[i]);
    const u16x2_t neg = v * u16x2_t{1, 0xffff};  // (Wc, -Ws)
    n[i] = __builtin_bit_cast(uint32_t, neg);
    np[i] = __builtin_bit_cast(uint32_t, neg + u16x2_t{128, 128});
    pp[i] = __builtin_bit_cast(uint32_t, v + u16x2_t{128, 128});
  }
  u32x2_t e_hi0, e_lo0, e_hi1, e_lo1;
#pragma unroll
  for (int qd = 0; qd < 2; ++qd) {
    e_lo0[qd] = __builtin_amdgcn_perm(n[2 * qd + 1], n[2 * qd], 0x06040200u);    // [Wc.b0, -Ws.b0] x 2 antennas
    e_hi0[qd] = __builtin_amdgcn_perm(np[2 * qd + 1], np[2 * qd], 0x07050301u);  // hi limbs of (Wc, -Ws)
    e_lo1[qd] = __builtin_amdgcn_perm(d[2 * qd + 1], d[2 * qd], 0x04060002u);    // [Ws.b0, Wc.b0]
    e_hi1[qd] = __builtin_amdgcn_perm(pp[2 * qd + 1], pp[2 * qd], 0x05070103u);  // hi limbs of (Ws, Wc)
  }
  const int tau = 4 * slab + (ml >> 3), row = (2 * ml) & 15;
  int8_t* o = img + ((tau * 2 * 64) + row + 16 * h) * 16 + 8 * hf;  // column 2 ml, limb 0 (= hi)
  *reinterpret_cast<u32x2_t*>(o) = e_hi0;
  *reinterpret_cast<u32x2_t*>(o + 64 * 16) = e_lo0;
  *reinterpret_cast<u32x2_t*>(o + 16) = e_hi1;
  *reinterpret_cast<u32x2_t*>(o + 16 + 64 * 16) = e_lo1;
}

// Mode (diagnostics only): 1 no table DMA / expansion, 2 no MFMA, 4 no stores, 8 no voltage DMA, 16 no LDS
// fragment reads (register-made operands), 32 no per-step barrier (timing only: races).
template <int Mode, int NW>
__global__ __launch_bounds__(OsCfg<NW>::kThreads, 8 / NW) void beamform_fused_i8_os_kernel(FusedArgs P) {
  using K = OsCfg<NW>;
  constexpr int kOsR = K::kR, kOsVBytes = K::kVBytes, kOsTBytes = K::kTBytes, kOsCBytes = K::kCBytes;
  extern __shared__ __attribute__((aligned(16))) int4 lds4[];
  int8_t* const lb = reinterpret_cast<int8_t*>(lds4);
  const uint32_t lbase = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lb));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n16 = lane & 15, g4 = lane >> 4;
  // the wave's 32 samples of the half and 32 beams; NW = 4: the workgroup's slab and its place among the slab pairs
  const bool xpair = (gridDim.x & 15) == 0;
  const int sg = wave & 3;
  const int bh = NW == 8 ? wave >> 2 : (xpair ? (blockIdx.x >> 3) & 1 : blockIdx.x & 1);
  const int pos = NW == 8 ? blockIdx.x : (xpair ? (blockIdx.x >> 4) * 8 + (blockIdx.x & 7) : blockIdx.x >> 1);
  const int npos = NW == 8 ? gridDim.x : gridDim.x >> 1;
  const int tb0 = NW == 8 ? 0 : 4 * bh;  // the slab's first tile in the table / image numbering

  // this workgroup's units: a contiguous, balanced run of (b, c, half), half fastest, then channel
  const long long nunits = 2LL * P.B * P.C;
  const int u0 = static_cast<int>(nunits * pos / npos);
  const int u1 = static_cast<int>(nunits * (pos + 1) / npos);
  const int Sa = P.A >> 5;  // k-steps of 32 antennas
  const int Sp = w32_table_steps(P.A);
  const int G = (u1 - u0) * Sa;
  const size_t crun = static_cast<size_t>(P.C) * 1024;  // next antenna's run of the same channel (T = 256)

  // LDS: vbuf[R] | tbuf[R] | cimg[2]
  int8_t* const cimg0 = lb + kOsR * (kOsVBytes + kOsTBytes);

  // issue counters: D(gd) = unit ud, step sd; T(gt) = unit ut, step st
  int gd = 0, ud = u0, sd = 0;
  int gt = 0, ut = u0, st = 0;
  auto issue_D = [&]() {
    if constexpr ((Mode & 8) == 0) {
      const int i = ud >> 1, b = i / P.C, c = i - b * P.C;
      // lanes 0-31: antenna 4 wave + 2 j, lanes 32-63: the next one; 16-byte piece (l & 31) of the slot holds the
      // half run's piece (l - rot) & 31, rot = 8 pieces for antennas with bit 3 set
      const int qa = 2 * K::kVG * wave + (lane >> 5);  // + 2 j (all in one group of 8 antennas)
      const int rot = ((qa >> 3) & 1) * 8;
      const uint8_t* src = P.raw + ((static_cast<size_t>(b) * P.A + 32 * sd + qa) * P.C + c) * 1024 + 512 * (ud & 1) +
                           16 * ((lane - rot) & 31);
      const uint32_t dst = lbase + (gd % kOsR) * kOsVBytes + (2 * K::kVG * wave) * 512;
#pragma unroll
      for (int j = 0; j < K::kVG; ++j) glds16(src + 2 * j * crun, dst + j * 1024);
    }
    ++gd;
    if (++sd == Sa) sd = 0, ++ud;
  };
  auto issue_T = [&]() {
    if constexpr ((Mode & 1) == 0) {
      const int slab = NW == 8 ? wave >> 2 : bh, hf = (wave >> 1) & 1, hp = wave & 1;
      const u32x4_t* src = reinterpret_cast<const u32x4_t*>(P.table) +
                           (static_cast<size_t>(ut >> 1) * 2 + slab) * 256 * Sp + ((st >> 1) * 2 + hf) * 256 +
                           128 * (st & 1) + 64 * hp + lane;
      glds16(src, lbase + kOsR * kOsVBytes + (gt % kOsR) * kOsTBytes + wave * 1024);
    }
    ++gt;
    if (++st == Sa) st = 0, ++ut;
  };
  // expand T(j) (its DMA retired and visible) into cimg[j % 2]
  auto expand = [&](int j) {
    if constexpr ((Mode & 1) == 0) {
      const u32x4_t q = *reinterpret_cast<const u32x4_t*>(lb + kOsR * kOsVBytes + (j % kOsR) * kOsTBytes + 16 * tid);
      const int slab = NW == 8 ? tid >> 8 : 0, hf = (tid >> 7) & 1, t7 = tid & 127;  // slab of the image
      os_expand_half(cimg0 + (j & 1) * kOsCBytes, t7 & 31, t7 >> 5, hf, slab, q);
    }
  };

  // prologue: T(0), then [T(j + R), D(j + R - 1)] for j = 1 - R .. -1, then T(0) into the image
  if (G > 0) issue_T();
#pragma unroll
  for (int j = 1; j < kOsR; ++j) {
    if (j < G) issue_T();
    if (j - 1 < G) issue_D();
  }
  constexpr int kPer = 1 + K::kVG;  // DMAs per wave and iteration: T + D
  if (G >= kOsR) wait_vm<kPer * (kOsR - 1)>(); else wait_vm<0>();
  lds_barrier();
  expand(0);

  i32x4_t hi[4][2][2], lo[4][2][2];  // [tile][sample dt][pol]
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int p = 0; p < 2; ++p) hi[t][dt][p] = lo[t][dt][p] = i32x4_t{0, 0, 0, 0};

  const float s32 = P.out_scale * 0x1p-14f;
  constexpr int M2 = 128;
  // this lane's voltage reads: antenna slot 8 g4 + qq, sample pair 16 sg + n16 of the half, rotated
  const int voff = (8 * g4) * 512 + ((128 * sg + 8 * n16 + 128 * (g4 & 1)) & 511);
  int cu = u0, cs = 0;  // the unit and step being contracted
  for (int g = 0; g < G; ++g) {
    // D(g) and T(g+1) retired: what may stay in flight is the R - 2 later iterations' DMAs
    if (g + kOsR - 1 < G) wait_vm<kPer * (kOsR - 2)>(); else wait_vm<0>();
    if constexpr ((Mode & 32) == 0) lds_barrier();
    if (g + kOsR < G) issue_T();
    if (g + kOsR - 1 < G) issue_D();
    if (g + 1 < G) expand(g + 1);

    {  // contract step g
      const int8_t* vb = lb + (g % kOsR) * kOsVBytes + voff;
      u32x2_t d[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        if constexpr (Mode & 16) {  // diagnostics: register-made voltages (no LDS reads)
          d[q] = u32x2_t{static_cast<uint32_t>(g * 0x01010101 + q + lane), static_cast<uint32_t>(g - q) * 0x9e37u};
        } else {
          d[q] = *reinterpret_cast<const u32x2_t*>(vb + q * 512);
        }
      }
      i32x4_t vf[2][2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          uint32_t w[4];
#pragma unroll
          for (int m2 = 0; m2 < 4; ++m2)
            w[m2] = __builtin_amdgcn_perm(d[2 * m2 + 1][dt], d[2 * m2][dt], p ? kSelP1 : kSelP0);
          vf[dt][p] = i32x4_t{static_cast<int>(w[0]), static_cast<int>(w[1]), static_cast<int>(w[2]),
                              static_cast<int>(w[3])};
        }
      const int4* img = reinterpret_cast<const int4*>(cimg0 + (g & 1) * kOsCBytes);
#pragma unroll
      for (int tl = 0; tl < 4; ++tl) {
        const int tau = (NW == 8 ? 4 * bh : 0) + tl;
        int4 x0, x1;
        if constexpr (Mode & 16) {
          x0 = int4{tau + g, lane, g, 7};
          x1 = int4{lane ^ g, tau, 3, g};
        } else {
          x0 = img[(tau * 2 + 0) * 64 + lane];
          x1 = img[(tau * 2 + 1) * 64 + lane];
        }
        const i32x4_t chi = i32x4_t{x0.x, x0.y, x0.z, x0.w}, clo = i32x4_t{x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int p = 0; p < 2; ++p) {
            if constexpr (Mode & 2) {  // one VALU per dword in place of the two MFMAs
              hi[tl][dt][p] ^= vf[dt][p];
              if (dt == 0 && p == 0) lo[tl][dt][p] ^= chi ^ clo;
            } else {
              hi[tl][dt][p] = mfma_i8(chi, vf[dt][p], hi[tl][dt][p]);
              lo[tl][dt][p] = mfma_i8(clo, vf[dt][p], lo[tl][dt][p]);
            }
          }
      }
    }

    if (++cs == Sa) {  // the unit is complete: requantise, store, restart the accumulators
      const int i = cu >> 1, b = i / P.C, c = i - b * P.C;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        int8_t* const prow = reinterpret_cast<int8_t*>(P.y) +
                             ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(256) * M2 +
                             64 * bh + 16 * g4;
        (void)tb0;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          uint32_t pk[4];
#pragma unroll
          for (int tl = 0; tl < 4; ++tl) {
            uint32_t qb[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) qb[r] = requant_bits((hi[tl][dt][p][r] << 8) + lo[tl][dt][p][r], s32);
            pk[tl] = pack_low_bytes(qb[0], qb[1], qb[2], qb[3]);
          }
          transpose_rows4(pk);  // lane group g4 now holds columns [16 g4, 16 g4 + 16) of its row
          const int t = 128 * (cu & 1) + 32 * sg + 2 * n16 + dt;
          if constexpr (Mode & 4) {
            if ((pk[0] ^ pk[1] ^ pk[2] ^ pk[3]) == 0x9e3779b9u) reinterpret_cast<int*>(P.y)[tid] = 1;
          } else {
            __builtin_nontemporal_store(u32x4_t{pk[0], pk[1], pk[2], pk[3]},
                                        reinterpret_cast<u32x4_t*>(prow + static_cast<size_t>(t) * M2));
          }
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
#pragma unroll
          for (int p = 0; p < 2; ++p) hi[t][dt][p] = lo[t][dt][p] = i32x4_t{0, 0, 0, 0};
      cs = 0;
      ++cu;
    }
  }
}

}  // namespace

namespace {
bool i8_os_fits(const FusedArgs& P, bool sample_signed) {
  return sample_signed && P.M == 64 && P.T == 256 && P.A >= 32 && P.A % 32 == 0 && w32_table_fits(P.A) &&
         P.table != nullptr && P.table_bytes >= w32_table_bytes(P.B, P.C, P.A, P.M);
}

// The table (kLayoutW32) must already be written on `st` (launch_q14_table).
template <int Mode, int NW = 4>
int launch_i8_os_mode(FusedArgs P, hipStream_t st) {
  BF_REQUIRE(i8_os_fits(P, true), "bf_beamform_fused: shape does not fit the output-stationary int8 kernel");
  const long long units = 2LL * P.B * P.C;  // (b, c, sample half)
  BF_REQUIRE(units < (1LL << 31), "bf_beamform_fused: too many items");
  const long long n_cu = cu_count();
  // NW 8: one workgroup per CU; NW 4: two per CU, one per slab of a unit (an even grid)
  const long long grid = NW == 8 ? std::min(units, n_cu) : 2 * std::min(units, n_cu);
  hipLaunchKernelGGL((beamform_fused_i8_os_kernel<Mode, NW>), dim3(static_cast<unsigned>(grid)),
                     dim3(OsCfg<NW>::kThreads), OsCfg<NW>::kLds, st, P);
  BF_LAUNCHED("beamform_fused_i8_os_kernel");
}

}  // namespace

}  // namespace bf

// Diagnostics: the output-stationary kernel alone on a table made outside the timing (tools/diag_fused.py w32t
// modes 700 + Mode).
extern "C" int bf_diag_i8_os(int mode, const uint8_t* raw, void* y, const void* table, int B, int C, int T, int A,
                             int M, void* stream) {
  bf::FusedArgs P{};
  P.raw = raw;
  P.y = y;
  P.table = static_cast<const uint32_t*>(table);
  P.table_bytes = bf::w32_table_bytes(B, C, A, M);
  P.B = B, P.C = C, P.T = T, P.A = A, P.M = M;
  P.out_scale = 1.0f / 64;
  hipStream_t st = bf::as_stream(stream);
  switch (mode) {  // Mode bits; + 100: the 8-wave, one-workgroup-per-CU form
#define BF_OS(m) \
    case m: return bf::launch_i8_os_mode<m, 4>(P, st); \
    case 100 + m: return bf::launch_i8_os_mode<m, 8>(P, st)
    BF_OS(0); BF_OS(1); BF_OS(2); BF_OS(4); BF_OS(8); BF_OS(9); BF_OS(12); BF_OS(13); BF_OS(15);
    BF_OS(29); BF_OS(45); BF_OS(61); BF_OS(32);
#undef BF_OS
    default: return BF_ERR_ARG;
  }
}
#endif
