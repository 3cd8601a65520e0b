// Integer wide fused beamformer, loader/consumer form: many antennas x beams (config 4: 256 antennas, 64 beams),
// int8 beams, bit-exact to the integer contract (oracle.fused_beamform_int8).
//
// Why a second wide kernel.  The slab-per-workgroup kernel (bf_wide_i8.hip) reads each (batch, channel) item's
// 256 KiB of voltages once per 16-beam slab (4x, the later reads from L2) and keeps at most two k-steps of loads in
// flight per wave; its load path alone (no coefficients, no MFMA) took 443 us at config 4 against a 217 us stream
// ceiling, and it did not get faster when each item was read only once (profiles/r2_*_w8_ablation.txt): it is
// latency-bound, not traffic-bound.  This kernel reads every voltage byte ONCE per CU and keeps ~96 KiB per CU in
// flight, continuously, across items:
//
//   one persistent 512-thread workgroup per CU (LDS-limited), items (b, c) in XCD-contiguous runs;
//   waves 4..7 are LOADERS: each loads 2 antennas x 16 B per lane per k-step into a 12-deep register ring
//     (ordinary global loads: a loader wave's vmcnt holds nothing else), builds the MFMA B fragments with one v_perm
//     per dword (and the x - 128 flip for uint8 samples), and writes them into a 3-slot LDS ring two k-steps ahead
//     of their use, in the exact lane order the consumers read (ds_read_b128, conflict-free);
//   waves 0..3 are CONSUMERS: wave w owns beam slab w (16 beams) of every item: it generates its slab's Q14 limb
//     table (32 KiB at A = 256) for the item in its own LDS region (fast float64 phasors + exact fix-up, no
//     cross-wave sync), then contracts the item's 4 quarters x 8 k-steps: per k-step 32 v_mfma_i32_16x16x64_i8 on
//     fragments prefetched one step ahead, requantises and stores each quarter's rows as the slab kernel does.
//   The ring is handed forward by LDS counters (full / free per slot), not barriers: loaders and consumers run
//   decoupled, a consumer waits only when its next slot is not yet written.
// A consumer's vector-memory counter holds only its own delay-model loads and beam stores, so the phasor phase's
// loads never wait behind the voltage stream (they would: vmcnt completes in order).
#include <algorithm>

#include "bf_fused.hpp"

namespace bf {

namespace {

constexpr int kLcConsumers = 4;                            // one 16-beam slab each
constexpr int kLcLoaders = 4;
constexpr int kLcThreads = 64 * (kLcConsumers + kLcLoaders);
constexpr int kLcRing = 3;                                 // LDS slots (loaders write two k-steps ahead)
constexpr int kLcDepth = 12;                               // register slots in flight per loader (multiple of 3)
constexpr int kLcSlot = 8 * 1024;                          // (i, pol) fragments of one k-step: 8 x 64 lanes x 16 B
constexpr int kLcStepTable = 4 * 1024;                     // one k-step of a slab's table: 2 tiles x 2 limbs x 1 KiB
constexpr int kLcMaxSteps = 8;                             // A <= 256

__device__ __forceinline__ int lc_step_base(int s, int A) { return min(32 * s, A - 32); }

__device__ __forceinline__ void lc_waitcnt_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0) only

// Ring hand-off by LDS counters (no s_barrier per k-step: waves run decoupled).  full[slot] counts loader portions
// written, free[slot] counts consumer waves done reading; both only grow.  Relaxed LDS atomics plus explicit
// lgkmcnt waits and compiler-only fences: a release/acquire at workgroup scope would also wait vmcnt(0) and drain
// the loaders' loads in flight.  LDS operations of one wave execute in order, so a counter update issued after the
// data writes (waited for) is seen after them.
__device__ __forceinline__ void lc_signal(unsigned* ctr) {
  lc_waitcnt_lgkm0();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ __forceinline__ void lc_wait(const unsigned* ctr, unsigned target) {
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Per-workgroup item run: XCD x = blockIdx % 8 owns items [x n8, (x+1) n8) (n8 = ceil(B C / 8)); its L workgroups
// take them round-robin, so an XCD's resident workgroups stream adjacent channels of every antenna row.
struct LcRun {
  int first, stride, count;
};

__device__ __forceinline__ LcRun lc_run(int n) {
  LcRun r{0, 1, 0};
  const int G8 = (gridDim.x / 8) * 8;
  if (static_cast<int>(blockIdx.x) >= G8) return r;
  const int x = blockIdx.x & 7, l = blockIdx.x >> 3, L = G8 >> 3;
  const int n8 = (n + 7) / 8;
  const int lo = x * n8, hi = min(n, lo + n8);
  r.first = lo + l;
  r.stride = L;
  r.count = hi > r.first ? (hi - r.first + L - 1) / L : 0;
  return r;
}

// ---- loader -----------------------------------------------------------------------------------------------------
struct LcLoad {
  uint32_t d[2][4];  // antennas (2 qq, 2 qq + 1) of the loader's group: 4 samples x (p0 re, p0 im, p1 re, p1 im)
};

// Mode (diagnostics only): 1 constant table (no phasors), 2 no MFMA, 4 no stores, 8 loaders write without loading.
// The loader's issue cursor: the next k-step to load (wave-uniform, advanced one step per issue; clamped to the last
// step: the loads past the end are unconditional re-loads that are never written).
struct LcCursor {
  int t, s, q, k;       // global step, step in quarter, quarter, item in the run
  const uint8_t* item;  // the item's base: raw + ((b A + 0) C + c) T 4
};

__device__ __forceinline__ const uint8_t* lc_item_base(const FusedArgs& P, const LcRun& run, int k) {
  const int item = run.first + k * run.stride;
  const int b = item / P.C, c = item - b * P.C;
  return P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
}

__device__ __forceinline__ void lc_advance(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps,
                                           LcCursor& u) {
  if (u.t + 1 >= nsteps) return;  // stay on the last step
  ++u.t;
  if (++u.s == S) {
    u.s = 0;
    if (++u.q == NQ) {
      u.q = 0;
      ++u.k;
      u.item = lc_item_base(P, run, u.k);
    }
  }
}

template <int Mode = 0>
__device__ __forceinline__ void lc_issue(const FusedArgs& P, const LcCursor& u, int w, int tl, int qq, LcLoad& L) {
  if constexpr ((Mode & 8) != 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) L.d[0][j] = L.d[1][j] = static_cast<uint32_t>(u.t * 0x01010101 + j + tl + qq);
    return;
  }
  const int T4 = P.T >> 2;
  const int tq = min(16 * u.q + tl, T4 - 1);
  const int a = lc_step_base(u.s, P.A) + 8 * w + 2 * qq;
  const size_t ant_stride = static_cast<size_t>(P.C) * P.T * 4;
  const uint8_t* src = u.item + static_cast<size_t>(a) * ant_stride + static_cast<size_t>(tq) * 16;
  const u32x4_t v0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src));
  const u32x4_t v1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(src + ant_stride));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    L.d[0][j] = v0[j];
    L.d[1][j] = v1[j];
  }
}

// B fragment dword qq of consumer lane (tl, w) for every (sample i, pol p): antennas (2 qq, 2 qq + 1) of group w.
template <bool Signed>
__device__ __forceinline__ void lc_write(int8_t* slot, int w, int tl, int qq, const LcLoad& L) {
  uint32_t* base = reinterpret_cast<uint32_t*>(slot + (tl + 16 * w) * 16 + 4 * qq);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t v = __builtin_amdgcn_perm(L.d[1][i], L.d[0][i], p ? kSelP1 : kSelP0);
      if constexpr (!Signed) v ^= 0x80808080u;  // x - 128 as int8 (128 * column sum added back by the consumer)
      base[(i * 2 + p) * 256] = v;              // fragment (i, p) block is 1 KiB = 256 dwords
    }
}

template <bool Signed, int Mode = 0>
__device__ __forceinline__ void lc_loader(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps, int8_t* ring,
                                          unsigned* full, unsigned* free_, int nact, int w, int lane) {
  const int tl = lane & 15, qq = lane >> 4;
  LcLoad R[kLcDepth];
  LcCursor u{0, 0, 0, 0, lc_item_base(P, run, 0)};
#pragma unroll
  for (int d = 0; d < kLcDepth; ++d) {
    lc_issue<Mode>(P, u, w, tl, qq, R[d]);
    lc_advance(P, run, S, NQ, nsteps, u);
  }
  for (int t0 = 0; t0 < nsteps; t0 += kLcDepth) {
#pragma unroll
    for (int kk = 0; kk < kLcDepth; ++kk) {
      const int t = t0 + kk;
      if (t >= nsteps) break;
      const int slot = kk % kLcRing;  // t0 is a multiple of kLcRing
      // consumers are done with step t - kLcRing, the slot's previous contents
      lc_wait(free_ + slot, static_cast<unsigned>(nact * (t / kLcRing)));
      lc_write<Signed>(ring + slot * kLcSlot, w, tl, qq, R[kk]);
      lc_issue<Mode>(P, u, w, tl, qq, R[kk]);  // step t + kLcDepth (clamped)
      lc_advance(P, run, S, NQ, nsteps, u);
      lc_signal(full + slot);
    }
  }
}

// ---- consumer -----------------------------------------------------------------------------------------------------
// The slab's Q14 limb table for item (b, c): lane (row = 2 m' + r, h) of tile tt writes its own A-fragment entries
// (step s: antennas 8 h .. 8 h + 7, column row of the tile).  It evaluates 4 of those 8 phasors and takes the other
// 4 from lane ^ 1 (same beam, other column).  Column sums (all k) for the uint8 correction come back as corr.
template <bool Signed>
__device__ __forceinline__ void lc_table(const FusedArgs& P, int8_t* table, int S, int slab, int b, int c, int lane,
                                         int (&corr)[2][4]) {
  const int tl = lane & 15, h = lane >> 4;
  const int mloc = tl >> 1, r = tl & 1;
  const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
  const double ch = static_cast<double>(P.base_ch + c);
  const int cd = P.delay_channels == 1 ? 0 : c;
  int colsum[2] = {0, 0};
  // (tile, step) pairs e = tt S + s, the delay model of pair e + 1 in flight while pair e is evaluated (two register
  // sets, unrolled by 2: no copies, so the wait before each evaluation is counted, not vmcnt(0)).  The gain load is
  // unconditional (from the delay table when there are no gains, then ignored) to keep it branch-free.
  const int E = 2 * S;
  const float* gsrc = P.gain ? P.gain : reinterpret_cast<const float*>(P.dv);
  const bool has_gain = P.gain != nullptr;
  auto fetch = [&](int e, float4 (&dv)[4], float (&gv)[4]) {
    const int tt = e >= S ? 1 : 0, s = e - tt * S;
    const int m = min(16 * slab + 8 * tt + mloc, P.M - 1);
    const float4* dv_row = P.dv + (static_cast<size_t>(cd) * P.M + m) * P.A;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int a = min(lc_step_base(s, P.A) + 8 * h + 4 * r + j, P.A - 1);
      dv[j] = dv_row[a];
      gv[j] = gsrc[static_cast<size_t>(m) * P.A + a];
    }
  };
  auto eval = [&](int e, const float4 (&dv)[4], const float (&gv0)[4]) {
    const int tt = e >= S ? 1 : 0, s = e - tt * S;
    const int m = 16 * slab + 8 * tt + mloc;
    bool valid[4];
    float gv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // rows of antennas an earlier step covered stay zero
      valid[j] = m < P.M && lc_step_base(s, P.A) + 8 * h + 4 * r + j >= 32 * s;
      gv[j] = has_gain ? gv0[j] : 1.0f;
    }
    int wc[4], ws[4];
    q14_coeffs<4, true, false, true>(dv, gv, valid, ch, P.ctot, P.ts, P.k, dt, P.gain, wc, ws);
    int pc[4], ps[4];  // partner's 4 phasors (the other half of the 8 antennas)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pc[j] = __shfl_xor(wc[j], 1);
      ps[j] = __shfl_xor(ws[j], 1);
    }
    // antennas 8h + 0..3 are evaluated by r = 0, 8h + 4..7 by r = 1
    int C8[8], S8[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      C8[j] = r ? pc[j] : wc[j];
      S8[j] = r ? ps[j] : ws[j];
      C8[4 + j] = r ? wc[j] : pc[j];
      S8[4 + j] = r ? ws[j] : ps[j];
    }
    // column r = 0 (the beam's real part): k pair (c, -s); r = 1 (imaginary part): (s, c).  Balanced limbs
    // W = 256 hi + lo, lo in [-128, 127]: lo byte = W & 255, hi byte = ((W + 128) >> 8) & 255.
    uint32_t hi4[4], lo4[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      uint32_t hp[2], lp[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int j = 2 * e2 + f;
        const int w0 = r ? S8[j] : C8[j];
        const int w1 = r ? C8[j] : -S8[j];
        colsum[tt] += w0 + w1;
        hp[f] = __builtin_amdgcn_perm(static_cast<uint32_t>(w1 + 128), static_cast<uint32_t>(w0 + 128), 0x0c0c0501u);
        lp[f] = __builtin_amdgcn_perm(static_cast<uint32_t>(w1), static_cast<uint32_t>(w0), 0x0c0c0400u);
      }
      hi4[e2] = __builtin_amdgcn_perm(hp[1], hp[0], 0x05040100u);
      lo4[e2] = __builtin_amdgcn_perm(lp[1], lp[0], 0x05040100u);
    }
    int8_t* o = table + s * kLcStepTable + (tt * 2) * 1024 + lane * 16;
    *reinterpret_cast<u32x4_t*>(o) = u32x4_t{hi4[0], hi4[1], hi4[2], hi4[3]};
    *reinterpret_cast<u32x4_t*>(o + 1024) = u32x4_t{lo4[0], lo4[1], lo4[2], lo4[3]};
  };
  float4 dA[4], dB[4];
  float gA[4], gB[4];
  fetch(0, dA, gA);
  for (int e = 0; e < E; e += 2) {  // E = 2 S is even
    fetch(e + 1, dB, gB);
    eval(e, dA, gA);
    fetch(min(e + 2, E - 1), dA, gA);  // unconditional (a spare re-load at the end): no branch, no vmcnt(0)
    eval(e + 1, dB, gB);
  }
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    corr[tt][0] = corr[tt][1] = corr[tt][2] = corr[tt][3] = 0;
    if constexpr (!Signed) {
      int v = colsum[tt];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);  // column tl's sum over all k, in every lane (tl, *)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) corr[tt][rr] = 128 * __shfl(v, 4 * h + rr);
    }
  }
}

struct LcFrags {
  i32x4_t f[4][2];  // [sample i][pol]
};

__device__ __forceinline__ void lc_read_frags(const int8_t* slot, int lane, LcFrags& F) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int4 v = *reinterpret_cast<const int4*>(slot + (i * 2 + p) * 1024 + lane * 16);
      F.f[i][p] = i32x4_t{v.x, v.y, v.z, v.w};
    }
}

template <bool Signed>
__device__ __forceinline__ void lc_store_quarter(const FusedArgs& P, int b, int c, int q, int m0, int lane,
                                                 const i32x4_t (&hi)[2][4][2], const i32x4_t (&lo)[2][4][2],
                                                 const int (&corr)[2][4]) {
  const int tl = lane & 15, h = lane >> 4;
  const int T4 = P.T >> 2, tq = 16 * q + tl, M2 = 2 * P.M;
  const float s32 = P.out_scale * 0x1p-14f;
  const bool full = m0 + 16 <= P.M && (M2 & 15) == 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    uint32_t pk[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t qb[4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) qb[rr] = requant_bits((hi[p][i][t][rr] << 8) + lo[p][i][t][rr] + corr[t][rr], s32);
        pk[t][i] = pack_low_bytes(qb[0], qb[1], qb[2], qb[3]);
      }
    const size_t prow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T);
    if (full) {
#pragma unroll
      for (int t = 0; t < 2; ++t) transpose_rows4(pk[t]);  // lane (tl, h): row 4 tq + h, columns 16 t .. 16 t + 15
      if (tq < T4) {
        int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 4 * tq + h) * M2 + 2 * m0;
#pragma unroll
        for (int t = 0; t < 2; ++t)  // plain stores: L2 merges the four slab waves' 32-B row segments into lines
          *reinterpret_cast<u32x4_t*>(o + 16 * t) = u32x4_t{pk[t][0], pk[t][1], pk[t][2], pk[t][3]};
      }
    } else if (tq < T4) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + 4 * tq + i) * M2 + 2 * m0;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const int col = 16 * t + 4 * h + rr;
            if (2 * m0 + col < M2) o[col] = static_cast<int8_t>((pk[t][i] >> (8 * rr)) & 255);
          }
      }
    }
  }
}

// A consumer wave: per item its slab's table, then quarters x k-steps.  Step t starts past barrier B_t with slot t's
// fragments in registers (Fc); it reads its table fragments, prefetches slot t + 1 (written before B_t) into Fn,
// runs 32 MFMAs on Fc, and ends at B_{t+1}.  Every LDS read is unconditional (the last prefetch reads a stale slot
// and is never used), so the compiler's lgkmcnt waits stay counted.  The accumulators live only inside a quarter,
// so the table phase has the register file to itself.
template <bool Signed, int Mode = 0>
__device__ __forceinline__ void lc_consumer(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps,
                                            int8_t* ring, unsigned* full, unsigned* free_, int8_t* table, int slab,
                                            int lane) {
  LcFrags Fc, Fn;
  int corr[2][4];
  int t = 0;
  lc_wait(full, kLcLoaders);  // step 0's slot is written
  lc_read_frags(ring, lane, Fc);
  for (int k = 0; k < run.count; ++k) {
    const int item = run.first + k * run.stride;
    const int b = item / P.C, c = item - b * P.C;
    if constexpr ((Mode & 1) != 0) {
      if (k == 0)
        for (int e = 0; e < 2 * S; ++e)
          *reinterpret_cast<u32x4_t*>(table + e * 2048 + lane * 16) = u32x4_t{0x01020304u, 0x05060708u, 1u, 2u};
      corr[0][0] = corr[0][1] = corr[0][2] = corr[0][3] = corr[1][0] = corr[1][1] = corr[1][2] = corr[1][3] = 0;
    } else {
      lc_table<Signed>(P, table, S, slab, b, c, lane, corr);
    }
    for (int q = 0; q < NQ; ++q) {
      i32x4_t hi[2][4][2], lo[2][4][2];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) hi[p][i][tt] = lo[p][i][tt] = i32x4_t{0, 0, 0, 0};
      for (int s = 0; s < S; ++s, ++t) {
        i32x4_t chi[2], clo[2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int4 x0 = *reinterpret_cast<const int4*>(table + s * kLcStepTable + (tt * 2) * 1024 + lane * 16);
          const int4 x1 = *reinterpret_cast<const int4*>(table + s * kLcStepTable + (tt * 2 + 1) * 1024 + lane * 16);
          chi[tt] = i32x4_t{x0.x, x0.y, x0.z, x0.w};
          clo[tt] = i32x4_t{x1.x, x1.y, x1.z, x1.w};
        }
        lc_signal(free_ + t % kLcRing);  // Fc and the table fragments are in registers: slot t may be refilled
        const int tn = t + 1 < nsteps ? t + 1 : t;  // the last prefetch re-reads a slot it holds (never used)
        lc_wait(full + tn % kLcRing, static_cast<unsigned>(kLcLoaders * (tn / kLcRing + 1)));
        lc_read_frags(ring + (tn % kLcRing) * kLcSlot, lane, Fn);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) {
              if constexpr ((Mode & 2) != 0) {
                hi[p][i][tt] += chi[tt] ^ Fc.f[i][p];
                lo[p][i][tt] += clo[tt] ^ Fc.f[i][p];
              } else {
                hi[p][i][tt] = mfma_i8(chi[tt], Fc.f[i][p], hi[p][i][tt]);
                lo[p][i][tt] = mfma_i8(clo[tt], Fc.f[i][p], lo[p][i][tt]);
              }
            }
        Fc = Fn;
      }
      if constexpr ((Mode & 4) != 0) {
        int sum = 0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int tt = 0; tt < 2; ++tt) sum += hi[p][i][tt][0] ^ lo[p][i][tt][3];
        if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[lane] = sum;
      } else {
        lc_store_quarter<Signed>(P, b, c, q, 16 * slab, lane, hi, lo, corr);
      }
    }
  }
}

template <bool Signed, int Mode = 0>
__global__ __launch_bounds__(kLcThreads, 1) void beamform_fused_i8_wide_lc_kernel(FusedArgs P) {
  extern __shared__ __attribute__((aligned(16))) int4 lds_lc[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const LcRun run = lc_run(P.B * P.C);
  if (run.count == 0) return;  // the whole workgroup
  const int S = (P.A + 31) >> 5;
  const int NQ = (P.T + 63) >> 6;
  const int nsteps = run.count * NQ * S;
  const int nact = min(P.nslabs, kLcConsumers);
  int8_t* ring = reinterpret_cast<int8_t*>(lds_lc);
  unsigned* full = reinterpret_cast<unsigned*>(ring + kLcRing * kLcSlot);
  unsigned* free_ = full + 4;
  int8_t* tables = ring + kLcRing * kLcSlot + 64;
  if (threadIdx.x < 8) full[threadIdx.x] = 0;  // full[0..3], free[0..3]
  __syncthreads();                             // the only barrier
  if (wave >= kLcConsumers)
    lc_loader<Signed, Mode>(P, run, S, NQ, nsteps, ring, full, free_, nact, wave - kLcConsumers, lane);
  else if (wave < nact)
    lc_consumer<Signed, Mode>(P, run, S, NQ, nsteps, ring, full, free_,
                              tables + static_cast<size_t>(wave) * S * kLcStepTable, wave, lane);
}

size_t lc_lds_bytes(const FusedArgs& P) {
  const int S = (P.A + 31) >> 5;
  return static_cast<size_t>(kLcRing) * kLcSlot + 64 + static_cast<size_t>(kLcConsumers) * S * kLcStepTable;
}

int lc_grid() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
                                                hipSuccess && n >= 8)
      cus = n;
    else
      cus = 256;
  }
  return cus;
}

}  // namespace

bool i8_wide_lc_fits(const FusedArgs& P) {
  return P.A >= 32 && P.A <= 32 * kLcMaxSteps && P.M <= 16 * kLcConsumers && lc_lds_bytes(P) <= kMaxLds &&
         static_cast<long long>(P.B) * P.C < (1LL << 31) / (((P.T + 63) >> 6) * ((P.A + 31) >> 5));
}

template <bool Signed, int Mode>
int launch_lc(FusedArgs P, hipStream_t st) {
  BF_REQUIRE(i8_wide_lc_fits(P), "bf_beamform_fused: shape does not fit the loader/consumer integer wide kernel");
  P.nslabs = (P.M + 15) / 16;
  hipLaunchKernelGGL((beamform_fused_i8_wide_lc_kernel<Signed, Mode>), dim3(static_cast<unsigned>(lc_grid())),
                     dim3(kLcThreads), lc_lds_bytes(P), st, P);
  BF_LAUNCHED("beamform_fused_i8_wide_lc_kernel");
}

template <bool Signed>
int launch_i8_wide_lc(FusedArgs P, hipStream_t st) {
  return launch_lc<Signed, 0>(P, st);
}

template int launch_i8_wide_lc<false>(FusedArgs, hipStream_t);
template int launch_i8_wide_lc<true>(FusedArgs, hipStream_t);

}  // namespace bf

#ifdef BF_DIAG
// Diagnostics: the loader/consumer kernel's ablations (tools/diag_fused.py, DIAG_KERNELS=lc).
extern "C" int bf_diag_lc(int mode, const uint8_t* raw, const float* dv, void* y, int B, int C, int T, int A, int M,
                          int Ctot, double ts, void* stream) {
  bf::FusedArgs P{};
  P.raw = raw;
  P.dv = reinterpret_cast<const float4*>(dv);
  P.y = y;
  P.delay_channels = 1;
  P.B = B, P.C = C, P.T = T, P.A = A, P.M = M;
  P.ctot = Ctot;
  P.ts = ts;
  P.k = -3.141592653589793 / (Ctot * ts);
  P.batch_dt = 1e-3;
  P.out_scale = 1.0f / 64;
  hipStream_t st = bf::as_stream(stream);
  switch (mode) {
    case 0: return bf::launch_lc<true, 0>(P, st);
    case 1: return bf::launch_lc<true, 1>(P, st);
    case 2: return bf::launch_lc<true, 2>(P, st);
    case 3: return bf::launch_lc<true, 3>(P, st);
    case 4: return bf::launch_lc<true, 4>(P, st);
    case 8: return bf::launch_lc<true, 8>(P, st);
    case 9: return bf::launch_lc<true, 9>(P, st);
    case 11: return bf::launch_lc<true, 11>(P, st);
    case 15: return bf::launch_lc<true, 15>(P, st);
    default: return BF_ERR_ARG;
  }
}
#endif
