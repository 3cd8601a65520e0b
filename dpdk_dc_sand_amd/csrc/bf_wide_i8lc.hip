// Integer wide fused beamformer, loader/consumer form: many antennas x beams (config 4: 256 antennas, 64 beams),
// int8 beams, bit-exact to the integer contract (oracle.fused_beamform_int8).
//
// STATUS: an explicit path only (BF_FUSED_PATH_STAGED, tested bit-exact); measured slower than the 32-beam slab
// kernel of bf_wide_i8.hip, which is the default (827 vs ~520 us at config 4: one consumer wave per SIMD cannot
// overlap its own VALU with its MFMAs, and one loader wave per SIMD could not build the tables fast enough --
// per-phase s_memtime stamps in profiles/r2_lc_phase_stamps.txt).
//
// Why a second wide kernel.  The slab-per-workgroup kernel (bf_wide_i8.hip) reads each (batch, channel) item's
// 256 KiB of voltages once per 16-beam slab (4x, the later reads from L2), keeps at most two k-steps of loads in
// flight per wave and evaluates its phasors between its loads and its MFMAs; its load path alone (no coefficients, no
// MFMA) took 443 us at config 4 against a 217 us stream ceiling (profiles/r2_w8_ablation*.txt).  Here:
//
//   one persistent 512-thread workgroup per CU (LDS-limited), items (b, c) in XCD-contiguous runs;
//   waves 4..7 are LOADERS, wave 4 + w pairs with consumer w on one SIMD.  A loader
//     (1) streams its quarter of every k-step's voltages (2 antennas x 16 B per lane) through a 12-deep register
//         ring (ordinary global loads: nothing else sits in its vmcnt), builds the MFMA B fragments with one v_perm
//         per dword (+ the x - 128 flip for uint8) and writes them into a 3-slot LDS ring in consumer lane order;
//     (2) evaluates beam slab w's Q14 phasors for the NEXT item (fast float64 + exact fix-up) into the other half of
//         a double-buffered table, in between and while it waits for ring slots;
//   waves 0..3 are CONSUMERS: wave w contracts slab w of the current item: per k-step 32 v_mfma_i32_16x16x64_i8 on
//     fragments prefetched one step ahead, then requantises and stores each 64-sample quarter.
//   So one SIMD co-issues the consumer's MFMAs with its loader's VALU (phasors, perms), which a lone wave cannot.
//
// Half table.  A slab's table holds one column per beam, k = (2a, 2a + 1) -> (c, -s): y_re = sum x_re c - x_im s is
// one MFMA against B1 = (re, im); y_im = sum x_im c + x_re s against B2 = (im, ~re) (bitwise not: -re = ~re + 1 stays
// in int8 for re = -128), minus sum_a s.  That halves the table (16 KiB per slab at A = 256), which is what lets it be
// double-buffered beside the ring in 160 KiB of LDS.  uint8 samples run as x - 128: + 128 sum (c - s) for y_re and
// + 128 sum (c + s) for y_im (column sums kept with the table).
//
// Hand-offs are LDS counters that only grow (no s_barrier: waves run decoupled):
//   full[slot]  loader portions written to a ring slot        free[slot]  consumers done reading it
//   tready[buf] loader slabs written to a table buffer        tfree[buf]  consumers done with it
// Relaxed LDS atomics with explicit lgkmcnt waits and compiler-only fences: a workgroup-scope release/acquire would
// also wait vmcnt(0) and drain a loader's loads in flight.  LDS operations of one wave execute in order.
#include <algorithm>

#include "bf_fused.hpp"

namespace bf {

namespace {

constexpr int kLcConsumers = 4;                            // one 16-beam slab each
constexpr int kLcLoaders = 4;
constexpr int kLcThreads = 64 * (kLcConsumers + kLcLoaders);
constexpr int kLcRing = 3;                                 // LDS voltage slots
constexpr int kLcDepth = 12;                               // register slots in flight per loader (multiple of 3)
constexpr int kLcSlot = 8 * 1024;                          // (i, pol) fragments of one k-step: 8 x 64 lanes x 16 B
constexpr int kLcStepTable = 2 * 1024;                     // one k-step of a slab's half table: 2 limbs x 1 KiB
constexpr int kLcMaxSteps = 8;                             // A <= 256
constexpr int kLcCorr = 16 * 2 * 4;                        // per slab: 16 beams x (sum c, sum s) int32

__device__ __forceinline__ int lc_step_base(int s, int A) { return min(32 * s, A - 32); }

__device__ __forceinline__ void lc_waitcnt_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0) only

__device__ __forceinline__ void lc_add(unsigned* ctr) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// publish: the wave's LDS writes land, then the counter moves
__device__ __forceinline__ void lc_signal(unsigned* ctr) {
  lc_waitcnt_lgkm0();
  lc_add(ctr);
}

__device__ __forceinline__ bool lc_ready(const unsigned* ctr, unsigned target) {
  return __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target;
}

// Every spin is bounded (~0.1 s of sleeps): a hand-off bug then ends the kernel with wrong beams, never a hang.
constexpr int kLcSpinCap = 1 << 21;

__device__ __forceinline__ void lc_wait(const unsigned* ctr, unsigned target) {
  for (int n = 0; !lc_ready(ctr, target) && n < kLcSpinCap; ++n) __builtin_amdgcn_s_sleep(1);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Diagnostics (Mode & 16): per-wave cycle counters by phase, summed with s_memtime and written over the output
// buffer at the end (loader: 0 total, 1 table units, 2 slot waits, 3 ring writes; consumer: 0 total, 1 table waits,
// 2 slot waits, 3 steps, 4 stores).
struct LcStamps {
  unsigned long long v[5] = {0, 0, 0, 0, 0};
  unsigned long long t0 = 0;
  __device__ void start() { t0 = __builtin_amdgcn_s_memtime(); }
  __device__ void lap(int i) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    v[i] += t - t0;
    t0 = t;
  }
  __device__ void flush(void* y, int wave) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(y) + (blockIdx.x * 8 + wave) * 8;
    if ((threadIdx.x & 63) == 0)
      for (int i = 0; i < 5; ++i) o[i] = v[i];
  }
};

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

__device__ __forceinline__ void lc_item_bc(const FusedArgs& P, const LcRun& run, int k, int* b, int* c) {
  const int item = run.first + k * run.stride;
  *b = item / P.C;
  *c = item - *b * P.C;
}

struct LcLayout {  // LDS carve-up
  int8_t* ring;
  unsigned* ctr;  // full[0..3], free[4..7], tready[8..9], tfree[10..11]
  int8_t* table0;
  int tbytes;     // table buffer 1 = table0 + tbytes; the column sums follow both buffers
  // buffer selects by arithmetic, not by indexing a pointer array (that would live in scratch)
  __device__ int8_t* table(int buf) const { return table0 + buf * tbytes; }
  __device__ int* corr(int buf) const {
    return reinterpret_cast<int*>(table0 + 2 * tbytes) + buf * (kLcConsumers * kLcCorr / 4);
  }
};

__device__ __forceinline__ LcLayout lc_layout(int8_t* lds, int S) {
  LcLayout L;
  L.ring = lds;
  L.ctr = reinterpret_cast<unsigned*>(lds + kLcRing * kLcSlot);
  L.tbytes = kLcConsumers * S * kLcStepTable;
  L.table0 = lds + kLcRing * kLcSlot + 64;
  return L;
}

// ---- loader: voltage ring ------------------------------------------------------------------------------------------
// Mode (diagnostics only): 1 constant tables (no phasors), 2 no MFMA, 4 no stores, 8 loaders write without loading.
struct LcLoad {
  uint32_t d[2][4];  // antennas (2 qq, 2 qq + 1) of the loader's group: 4 samples x (p0 re, p0 im, p1 re, p1 im)
};

// The issue cursor: the next k-step to load (wave-uniform, one step per issue; clamped to the last step: the loads
// past the end are unconditional re-loads that are never written).
struct LcCursor {
  int t, s, q, k;
  const uint8_t* item;  // raw + (b A C + c) T 4
};

__device__ __forceinline__ const uint8_t* lc_item_base(const FusedArgs& P, const LcRun& run, int k) {
  int b, c;
  lc_item_bc(P, run, k, &b, &c);
  return P.raw + (static_cast<size_t>(b) * P.A * P.C + c) * static_cast<size_t>(P.T) * 4;
}

__device__ __forceinline__ void lc_advance(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps,
                                           LcCursor& u) {
  if (u.t + 1 >= nsteps) return;
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

template <int Mode>
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

// B1 fragment dword qq of consumer lane (tl, w) for every (sample i, pol p): antennas (2 qq, 2 qq + 1) of group w.
template <bool Signed>
__device__ __forceinline__ void lc_write(int8_t* slot, int w, int tl, int qq, const LcLoad& L) {
  uint32_t* base = reinterpret_cast<uint32_t*>(slot + (tl + 16 * w) * 16 + 4 * qq);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      uint32_t v = __builtin_amdgcn_perm(L.d[1][i], L.d[0][i], p ? kSelP1 : kSelP0);
      if constexpr (!Signed) v ^= 0x80808080u;  // x - 128 as int8
      base[(i * 2 + p) * 256] = v;              // fragment (i, p) block is 1 KiB = 256 dwords
    }
}

// ---- loader: phasor table of one slab -----------------------------------------------------------------------------
// Lane (m' = lane & 15, h = lane >> 4) owns the A-fragment entry of beam 16 w + m', antennas 8 h .. 8 h + 7 of every
// k-step s: 16 bytes per limb = 8 x (c, -s).  Work unit e = (s, half): 4 antennas 8 h + 4 half + j, the delay model
// of unit e + 1 in flight meanwhile.
struct LcTable {
  int e, E;          // next unit, units per item (2 S)
  int k;             // item being tabled
  int cs[4], ss[4];  // first half of the current step (Q14)
  int sumc, sums;    // the lane's partial column sums
  float4 dvn[4];
  float gn[4];
  bool done;
};

__device__ __forceinline__ void lc_tfetch(const FusedArgs& P, int slab, int c, int e, int lane, float4 (&dv)[4],
                                          float (&gv)[4]) {
  const int s = e >> 1, half = e & 1;
  const int m = min(16 * slab + (lane & 15), P.M - 1);
  const int cd = P.delay_channels == 1 ? 0 : c;
  const float4* dv_row = P.dv + (static_cast<size_t>(cd) * P.M + m) * P.A;
  const float* gsrc = P.gain ? P.gain : reinterpret_cast<const float*>(P.dv);  // unconditional load, ignored
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int a = min(lc_step_base(s, P.A) + 8 * (lane >> 4) + 4 * half + j, P.A - 1);
    dv[j] = dv_row[a];
    gv[j] = gsrc[static_cast<size_t>(m) * P.A + a];
  }
}

__device__ __forceinline__ void lc_tstart(const FusedArgs& P, const LcRun& run, int S, int slab, int k, int lane,
                                          LcTable& T) {
  T.k = k;
  T.e = 0;
  T.E = 2 * S;
  T.sumc = T.sums = 0;
  T.done = k >= run.count;
  if (T.done) return;
  int b, c;
  lc_item_bc(P, run, k, &b, &c);
  lc_tfetch(P, slab, c, 0, lane, T.dvn, T.gn);
}

// One unit of the table of item T.k into buffer `table`/`corr`; publishes tready after the last unit.
template <int Mode>
__device__ __forceinline__ void lc_tunit(const FusedArgs& P, const LcRun& run, int S, int slab, int lane,
                                         int8_t* table, int* corr, unsigned* tready, LcTable& T) {
  int b, c;
  lc_item_bc(P, run, T.k, &b, &c);
  const int e = T.e, s = e >> 1, half = e & 1;
  const int h = lane >> 4, mloc = lane & 15, m = 16 * slab + mloc;
  float4 dv[4];
  float gv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    dv[j] = T.dvn[j];
    gv[j] = P.gain ? T.gn[j] : 1.0f;
  }
  lc_tfetch(P, slab, c, min(e + 1, T.E - 1), lane, T.dvn, T.gn);  // unconditional (a spare re-load at the end)
  int wc[4], ws[4];
  if constexpr ((Mode & 1) != 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wc[j] = 16384 - 7 * j - mloc;
      ws[j] = 100 * j + h - half;
    }
  } else {
    bool valid[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)  // rows of antennas an earlier step covered stay zero
      valid[j] = m < P.M && lc_step_base(s, P.A) + 8 * h + 4 * half + j >= 32 * s;
    const double dt = P.t0 + static_cast<double>(b) * P.batch_dt;
    q14_coeffs<4, true, false, true>(dv, gv, valid, static_cast<double>(P.base_ch + c), P.ctot, P.ts, P.k, dt, P.gain,
                                     wc, ws);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    T.sumc += wc[j];
    T.sums += ws[j];
  }
  if (half == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T.cs[j] = wc[j];
      T.ss[j] = ws[j];
    }
  } else {
    // 16 bytes per limb: antennas q = 0..7 -> (c, -s).  Balanced limbs W = 256 hi + lo, lo in [-128, 127]:
    // lo byte = W & 255, hi byte = ((W + 128) >> 8) & 255.
    int C8[8], N8[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      C8[j] = T.cs[j];
      N8[j] = -T.ss[j];
      C8[4 + j] = wc[j];
      N8[4 + j] = -ws[j];
    }
    uint32_t hi4[4], lo4[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      uint32_t hp[2], lp[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int j = 2 * e2 + f;
        hp[f] = __builtin_amdgcn_perm(static_cast<uint32_t>(N8[j] + 128), static_cast<uint32_t>(C8[j] + 128),
                                      0x0c0c0501u);
        lp[f] = __builtin_amdgcn_perm(static_cast<uint32_t>(N8[j]), static_cast<uint32_t>(C8[j]), 0x0c0c0400u);
      }
      hi4[e2] = __builtin_amdgcn_perm(hp[1], hp[0], 0x05040100u);
      lo4[e2] = __builtin_amdgcn_perm(lp[1], lp[0], 0x05040100u);
    }
    int8_t* o = table + (slab * S + s) * kLcStepTable + lane * 16;
    *reinterpret_cast<u32x4_t*>(o) = u32x4_t{hi4[0], hi4[1], hi4[2], hi4[3]};
    *reinterpret_cast<u32x4_t*>(o + 1024) = u32x4_t{lo4[0], lo4[1], lo4[2], lo4[3]};
  }
  if (++T.e == T.E) {  // column sums over every antenna of beam m' (lanes m', m' + 16, + 32, + 48)
    int sc = T.sumc, sn = T.sums;
    sc += __shfl_xor(sc, 16);
    sn += __shfl_xor(sn, 16);
    sc += __shfl_xor(sc, 32);
    sn += __shfl_xor(sn, 32);
    if (h == 0) {
      corr[slab * 32 + 2 * mloc] = sc;
      corr[slab * 32 + 2 * mloc + 1] = sn;
    }
    lc_signal(tready);
    T.done = true;
  }
}

// Table work for item T.k (buffer T.k & 1) once the consumers have released that buffer (item T.k - 2).
template <int Mode>
__device__ __forceinline__ bool lc_try_table(const FusedArgs& P, const LcRun& run, int S, int slab, int lane,
                                             const LcLayout& L, int nact, LcTable& T) {
  if (T.done) return false;
  const int buf = T.k & 1;
  if (T.e == 0 && !lc_ready(L.ctr + 10 + buf, static_cast<unsigned>(nact * (T.k >> 1)))) return false;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  lc_tunit<Mode>(P, run, S, slab, lane, L.table(buf), L.corr(buf), L.ctr + 8 + buf, T);
  return true;
}

template <bool Signed, int Mode>
__device__ __forceinline__ void lc_loader(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps,
                                          const LcLayout& L, int nact, int w, int lane) {
  const int tl = lane & 15, qq = lane >> 4;
  const int per_item = NQ * S;
  LcStamps st;
  const unsigned long long tbeg = __builtin_amdgcn_s_memtime();
  if constexpr ((Mode & 16) != 0) st.start();
  LcLoad R[kLcDepth];
  LcCursor u{0, 0, 0, 0, lc_item_base(P, run, 0)};
#pragma unroll
  for (int d = 0; d < kLcDepth; ++d) {
    lc_issue<Mode>(P, u, w, tl, qq, R[d]);
    lc_advance(P, run, S, NQ, nsteps, u);
  }
  // item 0's table up front (its voltages are in flight meanwhile); later items' tables are interleaved with the
  // ring steps, each as soon as its buffer is released (item k waits for the consumers to finish item k - 2)
  LcTable T;
  lc_tstart(P, run, S, w, 0, lane, T);
  for (int n = 0; !T.done && n < kLcSpinCap; ++n) lc_try_table<Mode>(P, run, S, w, lane, L, nact, T);
  lc_tstart(P, run, S, w, 1, lane, T);
  // units tried per ring step before the slot check, so that an item's table keeps pace with the ring
  const int upt = (2 * S + per_item - 1) / per_item;
  for (int t0 = 0; t0 < nsteps; t0 += kLcDepth) {
#pragma unroll
    for (int kk = 0; kk < kLcDepth; ++kk) {
      const int t = t0 + kk;
      if (t >= nsteps) break;
      const int slot = kk % kLcRing;  // t0 is a multiple of kLcRing
      // One loop, one table call site (the unrolled ring keeps its register indices static).  Table work never
      // blocks the ring: a unit whose buffer is not yet released is skipped (the consumers that will release it may
      // be waiting for this very slot).
      int budget = upt;
      for (int n = 0; n < kLcSpinCap; ++n) {
        if (T.done && T.k + 1 < run.count) lc_tstart(P, run, S, w, T.k + 1, lane, T);
        if constexpr ((Mode & 16) != 0) st.lap(2);
        const bool did = lc_try_table<Mode>(P, run, S, w, lane, L, nact, T);
        if constexpr ((Mode & 16) != 0) st.lap(did ? 1 : 2);
        if (did && --budget > 0) continue;
        if (lc_ready(L.ctr + 4 + slot, static_cast<unsigned>(nact * (t / kLcRing)))) break;
        if (!did) __builtin_amdgcn_s_sleep(1);
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if constexpr ((Mode & 16) != 0) st.lap(2);
      lc_write<Signed>(L.ring + slot * kLcSlot, w, tl, qq, R[kk]);
      lc_issue<Mode>(P, u, w, tl, qq, R[kk]);  // step t + kLcDepth (clamped)
      lc_advance(P, run, S, NQ, nsteps, u);
      lc_signal(L.ctr + slot);
      if constexpr ((Mode & 16) != 0) st.lap(3);
    }
  }
  for (int n = 0; n < kLcSpinCap; ++n) {  // the remaining tables
    if (T.done) {
      if (T.k + 1 >= run.count) break;
      lc_tstart(P, run, S, w, T.k + 1, lane, T);
    }
    if (!lc_try_table<Mode>(P, run, S, w, lane, L, nact, T)) __builtin_amdgcn_s_sleep(1);
  }
  if constexpr ((Mode & 16) != 0) {
    st.v[0] = __builtin_amdgcn_s_memtime() - tbeg;
    st.flush(P.y, 4 + w);
  }
}

// ---- consumer ------------------------------------------------------------------------------------------------------
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

__device__ __forceinline__ void lc_read_table(const int8_t* step, int lane, i32x4_t& hi, i32x4_t& lo) {
  const int4 x0 = *reinterpret_cast<const int4*>(step + lane * 16);
  const int4 x1 = *reinterpret_cast<const int4*>(step + 1024 + lane * 16);
  hi = i32x4_t{x0.x, x0.y, x0.z, x0.w};
  lo = i32x4_t{x1.x, x1.y, x1.z, x1.w};
}

// B2 = (im, ~re) per antenna from B1 = (re, im): bytes [b1, ~b0, b3, ~b2]
__device__ __forceinline__ i32x4_t lc_b2(const i32x4_t& b1) {
  i32x4_t r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t v = static_cast<uint32_t>(b1[j]);
    r[j] = static_cast<int>(__builtin_amdgcn_perm(~v, v, 0x06030401u));
  }
  return r;
}

// Accumulators of one quarter: [pol][sample i][re / im], hi and lo limbs
struct LcAcc {
  i32x4_t hi[2][4][2], lo[2][4][2];
};

template <bool Signed>
__device__ __forceinline__ void lc_store_quarter(const FusedArgs& P, int b, int c, int q, int m0, int lane,
                                                 const LcAcc& acc, const int (&corr)[2][4]) {
  const int tl = lane & 15, h = lane >> 4;
  const int T4 = P.T >> 2, tq = 16 * q + tl, M2 = 2 * P.M;
  const float s32 = P.out_scale * 0x1p-14f;
  if (tq >= T4) return;
  const bool full = m0 + 4 * h + 4 <= P.M;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const size_t prow = ((static_cast<size_t>(b) * 2 + p) * P.C + c) * static_cast<size_t>(P.T) + 4 * tq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t qb[2][4];  // [re / im][beam 4 h + r]
#pragma unroll
      for (int ri = 0; ri < 2; ++ri)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          qb[ri][r] = requant_bits((acc.hi[p][i][ri][r] << 8) + acc.lo[p][i][ri][r] + corr[ri][r], s32);
      // output row bytes 2 m, 2 m + 1 = (re, im) of beam m: beams 4 h .. 4 h + 3 are 8 contiguous bytes
      const uint32_t w0 = pack_low_bytes(qb[0][0], qb[1][0], qb[0][1], qb[1][1]);
      const uint32_t w1 = pack_low_bytes(qb[0][2], qb[1][2], qb[0][3], qb[1][3]);
      int8_t* o = reinterpret_cast<int8_t*>(P.y) + (prow + i) * M2 + 2 * (m0 + 4 * h);
      if (full) {
        *reinterpret_cast<u32x2_t*>(o) = u32x2_t{w0, w1};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (m0 + 4 * h + r < P.M) {
            const uint32_t wr = r < 2 ? w0 : w1;
            o[2 * r] = static_cast<int8_t>((wr >> (16 * (r & 1))) & 255);
            o[2 * r + 1] = static_cast<int8_t>((wr >> (16 * (r & 1) + 8)) & 255);
          }
      }
    }
  }
}

template <bool Signed, int Mode>
__device__ __forceinline__ void lc_consumer(const FusedArgs& P, const LcRun& run, int S, int NQ, int nsteps,
                                            const LcLayout& L, int slab, int lane) {
  const int h = lane >> 4;
  LcStamps st;
  const unsigned long long tbeg = __builtin_amdgcn_s_memtime();
  if constexpr ((Mode & 16) != 0) st.start();
  LcFrags Fc, Fn;
  int t = 0;
  lc_wait(L.ctr, kLcLoaders);  // step 0's slot is written
  lc_read_frags(L.ring, lane, Fc);
  for (int k = 0; k < run.count; ++k) {
    int b, c;
    lc_item_bc(P, run, k, &b, &c);
    const int buf = k & 1;
    if constexpr ((Mode & 16) != 0) st.lap(3);
    lc_wait(L.ctr + 8 + buf, static_cast<unsigned>(kLcLoaders * ((k >> 1) + 1)));  // every slab of item k is tabled
    if constexpr ((Mode & 16) != 0) st.lap(1);
    const int8_t* table = L.table(buf) + slab * S * kLcStepTable;
    int corr[2][4];  // [re / im][beam 4 h + r]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int* cb = L.corr(buf);
      const int sc = cb[slab * 32 + 2 * (4 * h + r)], sn = cb[slab * 32 + 2 * (4 * h + r) + 1];
      corr[0][r] = Signed ? 0 : 128 * (sc - sn);
      corr[1][r] = -sn + (Signed ? 0 : 128 * (sc + sn));
    }
    i32x4_t ahi, alo;
    lc_read_table(table, lane, ahi, alo);
    for (int q = 0; q < NQ; ++q) {
      LcAcc acc;
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ri = 0; ri < 2; ++ri) acc.hi[p][i][ri] = acc.lo[p][i][ri] = i32x4_t{0, 0, 0, 0};
      for (int s = 0; s < S; ++s, ++t) {
        if (t > 0) lc_add(L.ctr + 4 + (t - 1) % kLcRing);  // slot t - 1 was consumed by the last step's MFMAs
        const int tn = t + 1 < nsteps ? t + 1 : t;          // the last prefetch re-reads a slot it holds (unused)
        if constexpr ((Mode & 16) != 0) st.lap(3);
        lc_wait(L.ctr + tn % kLcRing, static_cast<unsigned>(kLcLoaders * (tn / kLcRing + 1)));
        if constexpr ((Mode & 16) != 0) st.lap(2);
        lc_read_frags(L.ring + (tn % kLcRing) * kLcSlot, lane, Fn);
        i32x4_t nhi = ahi, nlo = alo;
        if (s + 1 < S) lc_read_table(table + (s + 1) * kLcStepTable, lane, nhi, nlo);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const i32x4_t b2 = lc_b2(Fc.f[i][p]);
            if constexpr ((Mode & 2) != 0) {
              acc.hi[p][i][0] += ahi ^ Fc.f[i][p];
              acc.lo[p][i][0] += alo ^ Fc.f[i][p];
              acc.hi[p][i][1] += ahi ^ b2;
              acc.lo[p][i][1] += alo ^ b2;
            } else {
              acc.hi[p][i][0] = mfma_i8(ahi, Fc.f[i][p], acc.hi[p][i][0]);
              acc.lo[p][i][0] = mfma_i8(alo, Fc.f[i][p], acc.lo[p][i][0]);
              acc.hi[p][i][1] = mfma_i8(ahi, b2, acc.hi[p][i][1]);
              acc.lo[p][i][1] = mfma_i8(alo, b2, acc.lo[p][i][1]);
            }
          }
        Fc = Fn;
        ahi = nhi;
        alo = nlo;
      }
      if constexpr ((Mode & 4) != 0) {
        int sum = 0;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ri = 0; ri < 2; ++ri) sum += acc.hi[p][i][ri][0] ^ acc.lo[p][i][ri][3];
        if (sum == 0x12345678) reinterpret_cast<int*>(P.y)[lane] = sum;
      } else {
        if constexpr ((Mode & 16) != 0) st.lap(3);
        lc_store_quarter<Signed>(P, b, c, q, 16 * slab, lane, acc, corr);
        if constexpr ((Mode & 16) != 0) st.lap(4);
      }
      if (q + 1 < NQ) lc_read_table(table, lane, ahi, alo);  // step 0 again for the next quarter
    }
    lc_signal(L.ctr + 10 + buf);  // the table buffer of item k is free
  }
  if constexpr ((Mode & 16) != 0) {
    st.v[0] = __builtin_amdgcn_s_memtime() - tbeg;
    st.flush(P.y, slab);
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
  const LcLayout L = lc_layout(reinterpret_cast<int8_t*>(lds_lc), S);
  if (threadIdx.x < 16) L.ctr[threadIdx.x] = 0;
  __syncthreads();  // the only barrier
  if (wave >= kLcConsumers)
    lc_loader<Signed, Mode>(P, run, S, NQ, nsteps, L, nact, wave - kLcConsumers, lane);
  else if (wave < nact)
    lc_consumer<Signed, Mode>(P, run, S, NQ, nsteps, L, wave, lane);
}

size_t lc_lds_bytes(const FusedArgs& P) {
  const int S = (P.A + 31) >> 5;
  return static_cast<size_t>(kLcRing) * kLcSlot + 64 + 2 * static_cast<size_t>(kLcConsumers) * S * kLcStepTable +
         2 * kLcConsumers * kLcCorr;
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

template <bool Signed, int Mode>
int launch_lc(FusedArgs P, hipStream_t st);

}  // namespace

bool i8_wide_lc_fits(const FusedArgs& P) {
  return P.A >= 32 && P.A <= 32 * kLcMaxSteps && P.M <= 16 * kLcConsumers && lc_lds_bytes(P) <= kMaxLds &&
         static_cast<long long>(P.B) * P.C < (1LL << 31) / (((P.T + 63) >> 6) * ((P.A + 31) >> 5));
}

namespace {
template <bool Signed, int Mode>
int launch_lc(FusedArgs P, hipStream_t st) {
  BF_REQUIRE(i8_wide_lc_fits(P), "bf_beamform_fused: shape does not fit the loader/consumer integer wide kernel");
  P.nslabs = (P.M + 15) / 16;
  hipLaunchKernelGGL((beamform_fused_i8_wide_lc_kernel<Signed, Mode>), dim3(static_cast<unsigned>(lc_grid())),
                     dim3(kLcThreads), lc_lds_bytes(P), st, P);
  BF_LAUNCHED("beamform_fused_i8_wide_lc_kernel");
}
}  // namespace

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
    case 16: return bf::launch_lc<true, 16>(P, st);
    case 17: return bf::launch_lc<true, 17>(P, st);
    default: return BF_ERR_ARG;
  }
}
#endif
