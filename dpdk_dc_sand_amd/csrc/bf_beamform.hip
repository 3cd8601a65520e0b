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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "bf_mfma.hpp"

namespace bf {

// ---------------------------------------------------------------------------------------------------------
// Stage W[b,p,c][:, slab columns] (rows k < Sp*32, zero past 2A and past 2M) -> hi/lo fragments in LDS.  A thread
// takes 8 consecutive k of one column (a fragment lane's 8 halves): 8 dword loads down the column (32 threads read
// 128 contiguous bytes of each row), all issued before any conversion, then one ds_write_b128 per limb.  (Round 1
// staged float4 rows with a runtime division per element and two 2-byte LDS writes per value: at 256 antennas the
// staging alone cost ~540 us of a 2 ms launch.)
template <int NTS>
__device__ __forceinline__ void stage_table(_Float16* lh, const float* __restrict__ wp, int K2, int M2, int Sp,
                                            int tau0, int nts, int tid) {
  constexpr int cols = NTS * 16;
  const int npairs = Sp * 4 * cols;  // (k block of 8, column)
  for (int e0 = 0; e0 < npairs; e0 += 2 * kThreads) {
    float v[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = min(e0 + u * kThreads + tid, npairs - 1);
      const int kb = e / cols, cl = e % cols;  // cols is a power of two: shifts
      const int col = min(tau0 * 16 + cl, M2 - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[u][j] = wp[static_cast<size_t>(min(8 * kb + j, K2 - 1)) * M2 + col];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = e0 + u * kThreads + tid;
      if (e >= npairs) break;
      const int kb = e / cols, cl = e % cols;
      if (cl >= 16 * nts) continue;  // past the slab's last tile (partial slab)
      const bool colok = tau0 * 16 + cl < M2;
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float w = (colok && 8 * kb + j < K2) ? v[u][j] : 0.0f;
        hi[j] = static_cast<_Float16>(w);
        lo[j] = static_cast<_Float16>(w - static_cast<float>(hi[j]));  // exact difference, then rounded
      }
      const int e8 = coef_elem(8 * kb, cl, nts);  // 8 consecutive halves of one lane's fragment
      *reinterpret_cast<half8*>(lh + e8) = hi;
      *reinterpret_cast<half8*>(lh + e8 + 64 * 8) = lo;
    }
  }
}

// Workgroup -> (item bpc, slab).  xcd: the slabs of one item run back to back on one XCD (workgroups are dealt to
// the 8 XCDs round-robin), so the slabs after the first re-read the item's voltages from that XCD's L2; the grid is
// padded to whole groups of 8 items and the padding workgroups return at once.
__device__ __forceinline__ bool table_coords(int nslabs, long long nbpc, int xcd, int& slab, size_t& bpc) {
  if (xcd) {
    const int x = blockIdx.x & 7, local = blockIdx.x >> 3;
    slab = local % nslabs;
    bpc = static_cast<size_t>(local / nslabs) * 8 + x;
    return static_cast<long long>(bpc) < nbpc;
  }
  slab = blockIdx.x % nslabs;
  bpc = blockIdx.x / nslabs;
  return true;
}

// ---------------------------------------------------------------------------------------------------------
// MatrixMultiply drop-in.  grid = B*P*C*nslabs; a slab is NTS 16-column tiles of the 2M outputs.
// Vec8: A % 4 == 0, so a lane's 8 bytes are one aligned 8-byte load; otherwise 2-byte antenna granules.
template <bool Signed, int NTS, bool Vec8>
__global__ __launch_bounds__(kThreads) void beamform_table_kernel(const uint8_t* __restrict__ x,
                                                                  const float* __restrict__ w,
                                                                  float* __restrict__ y, int NB, int A, int M, int S,
                                                                  int NT, int nslabs, long long nbpc, int xcd) {
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int slab;
  size_t bpc;
  if (!table_coords(nslabs, nbpc, xcd, slab, bpc)) return;
  const int tau0 = slab * NTS;
  const int nts = min(NTS, NT - tau0);
  const int K2 = 2 * A, M2 = 2 * M;

  stage_table<NTS>(reinterpret_cast<_Float16*>(lds), w + bpc * static_cast<size_t>(K2) * M2, K2, M2, S, tau0, nts,
                   tid);
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

// Streaming variant for A % 4 == 0 (8-byte fragment loads): a wave's k-step fragments of all its row groups form one
// stream that runs through a register ring of R steps x G row groups, refilled R steps ahead by unconditional loads
// (address clamped inside the table; steps past S meet zero coefficients).  The loop body is identical every
// iteration, so the compiler's vmcnt waits stay exact and R G loads stay in flight -- the per-step load-then-use of
// the basic kernel paid one memory latency per k-step (32 per row at 256 antennas).
//
// W16 (A % 8 == 0, x 16-byte aligned): one 16-byte load per lane covers two k-steps -- lane group h reads bytes
// [64 s2 + 16 h, + 16) of its row, i.e. halves (A_h, B_h) -- and two permlane swaps per dword rebuild both steps'
// fragments exactly:  permlane16_swap(A, B) -> ([A0 B0 A2 B2], [A1 B1 A3 B3]) over lane groups 0..3, then
// permlane32_swap -> step 2 s2 = [A0 B0 A1 B1] (k = 8 h + j) and step 2 s2 + 1 = [A2 B2 A3 B3].  Half the load
// instructions (each still touches 16 row segments), the same per-step fragments and MFMA order (bitwise the same
// sums as the 8-byte form, and as the fused kernels).
template <bool Signed, int NTS, int R, int Mode = 0, bool W16 = false>
__global__ __launch_bounds__(kThreads) void beamform_table_ring_kernel(const uint8_t* __restrict__ x,
                                                                       const float* __restrict__ w,
                                                                       float* __restrict__ y, int NB, int A, int M,
                                                                       int S, int NT, int nslabs, long long nbpc,
                                                                       int xcd) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int slab;
  size_t bpc;
  if (!table_coords(nslabs, nbpc, xcd, slab, bpc)) return;
  const int tau0 = slab * NTS;
  const int nts = min(NTS, NT - tau0);
  const int K2 = 2 * A, M2 = 2 * M;
  const int Sp = (S + R - 1) / R * R;  // padded steps per row group

  const int T = NB * kSamplesPerBlock;
  const uint8_t* xp = x + bpc * static_cast<size_t>(T) * K2;
  float* yp = y + bpc * static_cast<size_t>(T) * M2;
  const int h = lane >> 4, tl = lane & 15;
  const int nrg = (NB - wave + kWaves - 1) / kWaves;  // this wave's row groups (rg = wave + 4 j)
  // G row groups are contracted together (each LDS table fragment feeds G x 2 MFMAs, 2 G NTS accumulator chains);
  // the lane's row pointer of row group j is computed once per row group (round 1 recomputed a division and a
  // 64-bit product per load: ~1.3 ms of a 2 ms launch went to streaming x at 256 antennas)
  constexpr int G = 2;
  auto rowp = [&](int j) -> const uint8_t* {  // clamped inside the item even for row-less waves
    return xp + static_cast<size_t>(min((wave + kWaves * j) * kSamplesPerBlock + tl, T - 1)) * K2;
  };
  // (the fused kernels' bitwise equality with this chain rests on the per-step fragments: the 16-byte form below
  // re-deals its loads into exactly the one-step fragments)
  const int kh = 8 * h;
  auto ld = [&](const uint8_t* row, int s) -> uint2 {
    if constexpr (Mode & 8) return uint2{static_cast<uint32_t>(s + tl), static_cast<uint32_t>(s)};
    return *reinterpret_cast<const uint2*>(row + min(32 * s + kh, K2 - 8));
  };
  auto ld16 = [&](const uint8_t* row, int s2) -> uint4 {  // W16: steps 2 s2, 2 s2 + 1
    if constexpr (Mode & 8)
      return uint4{static_cast<uint32_t>(s2 + tl), static_cast<uint32_t>(s2), static_cast<uint32_t>(s2 - tl), 7u};
    return *reinterpret_cast<const uint4*>(row + min(64 * s2 + 2 * kh, K2 - 16));
  };
  const uint8_t* cur_rows[G];
  const uint8_t* next_rows[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    cur_rows[g] = rowp(g);
    next_rows[g] = rowp(G + g);
  }
  // the ring's first R steps are requested BEFORE the coefficient table: vmcnt counts in order, so the table
  // conversion's wait then covers both, and the voltage latency overlaps the table's
  constexpr int R8 = W16 ? 1 : R, R16 = W16 ? R / 2 : 1;
  uint2 ring[R8][G];
  uint4 ring16[R16][G];
  if constexpr (W16) {
#pragma unroll
    for (int r = 0; r < R16; ++r)
#pragma unroll
      for (int g = 0; g < G; ++g) ring16[r][g] = ld16(cur_rows[g], r);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int g = 0; g < G; ++g) ring[r][g] = ld(cur_rows[g], r);
  }
  __builtin_amdgcn_sched_barrier(0);
  // Mode (diagnostics only): 1 no table staging, 2 no MFMA, 4 no stores, 8 no voltage loads
  if constexpr (!(Mode & 1))
    stage_table<NTS>(reinterpret_cast<_Float16*>(lds), w + bpc * static_cast<size_t>(K2) * M2, K2, M2, Sp, tau0, nts,
                     tid);  // padded steps zero
  __syncthreads();
  if (nrg <= 0) return;

  const int npair = (nrg + G - 1) / G;
  for (int pi = 0; pi < npair; ++pi) {
    f32x4 acc[G][NTS];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) acc[g][tau] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s0 = 0; s0 < Sp; s0 += R) {  // R divides Sp
      const bool nx = s0 + R >= Sp;      // this ring turn prefetches the next row groups' first steps
      const int sb = nx ? 0 : s0 + R;
      auto contract = [&](int s, const half8 (&v)[G]) {
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) {
          if (tau < nts) {
            const int slot = ((s * nts + tau) * 2) * 64;
            const half8 chi = lds[slot + lane], clo = lds[slot + 64 + lane];
#pragma unroll
            for (int g = 0; g < G; ++g) {
              if constexpr (Mode & 2) {
                acc[g][tau] += __builtin_bit_cast(f32x4, v[g]) + __builtin_bit_cast(f32x4, chi);
              } else {
                acc[g][tau] = mfma(chi, v[g], acc[g][tau]);
                acc[g][tau] = mfma(clo, v[g], acc[g][tau]);
              }
            }
          }
        }
      };
      if constexpr (W16) {
#pragma unroll
        for (int r = 0; r < R16; ++r) {
          half8 v0[G], v1[G];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint4 cur = ring16[r][g];
            ring16[r][g] = ld16(nx ? next_rows[g] : cur_rows[g], sb / 2 + r);
            auto x0 = __builtin_amdgcn_permlane16_swap(cur.x, cur.z, false, false);
            auto x1 = __builtin_amdgcn_permlane16_swap(cur.y, cur.w, false, false);
            auto y0 = __builtin_amdgcn_permlane32_swap(x0[0], x0[1], false, false);
            auto y1 = __builtin_amdgcn_permlane32_swap(x1[0], x1[1], false, false);
            v0[g] = bytes8_to_frag<Signed>(y0[0], y1[0]);
            v1[g] = bytes8_to_frag<Signed>(y0[1], y1[1]);
          }
          contract(s0 + 2 * r, v0);
          contract(s0 + 2 * r + 1, v1);
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          half8 v[G];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint2 cur = ring[r][g];
            ring[r][g] = ld(nx ? next_rows[g] : cur_rows[g], sb + r);
            v[g] = bytes8_to_frag<Signed>(cur.x, cur.y);
          }
          contract(s0 + r, v);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int j = pi * G + g;
      if (j >= nrg) break;
      float* orow = yp + static_cast<size_t>((wave + kWaves * j) * kSamplesPerBlock + tl) * M2;
#pragma unroll
      for (int tau = 0; tau < NTS; ++tau) {
        if constexpr (Mode & 4) {
          if (acc[g][tau][0] == 1234.5f) orow[tau] = acc[g][tau][1];
        } else {
          if (tau < nts) store_f32<NTS>(orow, 16 * (tau0 + tau) + 4 * h, M2, acc[g][tau]);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      cur_rows[g] = next_rows[g];
      next_rows[g] = rowp((pi + 2) * G + g);
    }
  }
}

// Persistent form of the 16-byte ring kernel (256-antenna rows: UPT = 8 table units per thread): a workgroup walks
// its (item, slab) list, and the next item's coefficient slab is loaded into registers (64 floats per thread) while
// the current item is contracted, so the table read -- half the algorithmic bytes at config 4 -- no longer sits
// between the workgroup's start and its first MFMA.  The ring's last turn of an item prefetches the next item's
// first steps.  Per item: convert the registers into the LDS slab, barrier, request the next slab, contract, barrier.
// The MFMA sequence per output is the ring kernel's (bitwise the same results).
template <bool Signed, int NTS, int R, int UPT, int Mode = 0, int G = 2>
__global__ __launch_bounds__(kThreads, 2) void beamform_table_persist_kernel(
    const uint8_t* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int NB, int A, int M, int S,
    int NT, int nslabs, long long nbpc, int xcd, long long nitems) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const int K2 = 2 * A, M2 = 2 * M;
  const int Sp = (S + R - 1) / R * R;
  const int T = NB * kSamplesPerBlock;
  constexpr int R16 = R / 2, cols = NTS * 16;
  const long long stride = gridDim.x;  // a multiple of 8: an item's XCD is its workgroup's
  // item -> (slab, bpc), the table_coords mapping; padding items (xcd groups past nbpc) are skipped
  auto coords = [&](long long it, int& slab, size_t& bpc) -> bool {
    if (xcd) {
      const long long local = it >> 3;
      slab = static_cast<int>(local % nslabs);
      bpc = static_cast<size_t>(local / nslabs) * 8 + static_cast<size_t>(it & 7);
    } else {
      slab = static_cast<int>(it % nslabs);
      bpc = static_cast<size_t>(it / nslabs);
    }
    return static_cast<long long>(bpc) < nbpc;
  };
  auto next_valid = [&](long long it) -> long long {  // the first valid item >= it on this workgroup's list, or -1
    int sl;
    size_t bp;
    for (; it < nitems; it += stride)
      if (coords(it, sl, bp)) return it;
    return -1;
  };
  float tv[UPT][8];
  auto table_load = [&](int slab, size_t bpc) {
    if constexpr (Mode & 16) {  // diagnostics: no table loads
#pragma unroll
      for (int u = 0; u < UPT; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) tv[u][j] = 1e-3f * static_cast<float>(j + u + slab);
      return;
    }
    const float* wp = w + bpc * static_cast<size_t>(K2) * M2;
    const int tau0 = slab * NTS;
    // rows past 2A only occur as whole 8-row units (A % 8 == 0): clamp the unit's first row, zeroed at the store
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int e = u * kThreads + tid, kb = e / cols, cl = e % cols;
      const float* pu = wp + static_cast<size_t>(min(8 * kb, K2 - 8)) * M2 + min(tau0 * 16 + cl, M2 - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) tv[u][j] = pu[static_cast<size_t>(j) * M2];
    }
  };
  auto table_store = [&](int slab) {
    const int tau0 = slab * NTS, nts = min(NTS, NT - tau0);
    _Float16* lh = reinterpret_cast<_Float16*>(lds);
#pragma unroll
    for (int u = 0; u < UPT; ++u) {
      const int e = u * kThreads + tid, kb = e / cols, cl = e % cols;
      if (cl >= 16 * nts) continue;
      const bool colok = tau0 * 16 + cl < M2;
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float wv = (colok && 8 * kb + j < K2) ? tv[u][j] : 0.0f;
        hi[j] = static_cast<_Float16>(wv);
        lo[j] = static_cast<_Float16>(wv - static_cast<float>(hi[j]));
      }
      const int e8 = coef_elem(8 * kb, cl, nts);
      *reinterpret_cast<half8*>(lh + e8) = hi;
      *reinterpret_cast<half8*>(lh + e8 + 64 * 8) = lo;
    }
  };
  const int nrg = (NB - wave + kWaves - 1) / kWaves;
  const int npair = (nrg + G - 1) / G;
  // row pointer of the wave's row group j of item bpc (clamped inside the item)
  auto rowp = [&](size_t bpc, int j) -> const uint8_t* {
    return x + bpc * static_cast<size_t>(T) * K2 +
           static_cast<size_t>(min((wave + kWaves * j) * kSamplesPerBlock + tl, T - 1)) * K2;
  };
  const int kh2 = 16 * h;
  auto ld16 = [&](const uint8_t* row, int s2) -> uint4 {
    if constexpr (Mode & 8)
      return uint4{static_cast<uint32_t>(s2 + tl), static_cast<uint32_t>(s2), static_cast<uint32_t>(s2 - tl), 7u};
    return *reinterpret_cast<const uint4*>(row + min(64 * s2 + kh2, K2 - 16));
  };

  long long it = next_valid(blockIdx.x);
  if (it < 0) return;  // workgroup-uniform
  int slab;
  size_t bpc;
  coords(it, slab, bpc);
  long long itn = next_valid(it + stride);
  int slab_n = slab;
  size_t bpc_n = bpc;
  if (itn >= 0) coords(itn, slab_n, bpc_n);
  table_load(slab, bpc);
  const uint8_t* cur_rows[G];
  const uint8_t* next_rows[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    cur_rows[g] = rowp(bpc, g);
    next_rows[g] = npair > 1 ? rowp(bpc, G + g) : rowp(bpc_n, g);
  }
  uint4 ring16[R16][G];
#pragma unroll
  for (int r = 0; r < R16; ++r)
#pragma unroll
    for (int g = 0; g < G; ++g) ring16[r][g] = ld16(cur_rows[g], r);

  while (true) {
    __syncthreads();  // every wave is done reading the previous slab
    if constexpr (!(Mode & 1)) table_store(slab);
    __syncthreads();
    if (itn >= 0) table_load(slab_n, bpc_n);  // in flight during this item's contraction
    const int tau0 = slab * NTS, nts = min(NTS, NT - tau0);
    float* yp = y + bpc * static_cast<size_t>(T) * M2;
    for (int pi = 0; pi < npair; ++pi) {
      f32x4 acc[G][NTS];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) acc[g][tau] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < Sp; s0 += R) {
        const bool nx = s0 + R >= Sp;
        const int sb = nx ? 0 : s0 + R;
#pragma unroll
        for (int r = 0; r < R16; ++r) {
          half8 v0[G], v1[G];
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint4 cur = ring16[r][g];
            ring16[r][g] = ld16(nx ? next_rows[g] : cur_rows[g], sb / 2 + r);
            auto x0 = __builtin_amdgcn_permlane16_swap(cur.x, cur.z, false, false);
            auto x1 = __builtin_amdgcn_permlane16_swap(cur.y, cur.w, false, false);
            auto y0 = __builtin_amdgcn_permlane32_swap(x0[0], x0[1], false, false);
            auto y1 = __builtin_amdgcn_permlane32_swap(x1[0], x1[1], false, false);
            v0[g] = bytes8_to_frag<Signed>(y0[0], y1[0]);
            v1[g] = bytes8_to_frag<Signed>(y0[1], y1[1]);
          }
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int s = s0 + 2 * r + half;
#pragma unroll
            for (int tau = 0; tau < NTS; ++tau) {
              if (tau < nts) {
                const int slot = ((s * nts + tau) * 2) * 64;
                const half8 chi = lds[slot + lane], clo = lds[slot + 64 + lane];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                  const half8 vv = half ? v1[g] : v0[g];
                  acc[g][tau] = mfma(chi, vv, acc[g][tau]);
                  acc[g][tau] = mfma(clo, vv, acc[g][tau]);
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int j = pi * G + g;
        if (j >= nrg) break;
        float* orow = yp + static_cast<size_t>((wave + kWaves * j) * kSamplesPerBlock + tl) * M2;
#pragma unroll
        for (int tau = 0; tau < NTS; ++tau) {
          if constexpr (Mode & 4) {
            if (acc[g][tau][0] == 1234.5f) orow[tau] = acc[g][tau][1];
          } else {
            if (tau < nts) store_f32<NTS>(orow, 16 * (tau0 + tau) + 4 * h, M2, acc[g][tau]);
          }
        }
      }
      // rows of pair pi + 2: this item's, or (past its last pair) the next item's first pairs
#pragma unroll
      for (int g = 0; g < G; ++g) {
        cur_rows[g] = next_rows[g];
        const int q = pi + 2;
        next_rows[g] = q < npair ? rowp(bpc, q * G + g) : rowp(bpc_n, (q - npair) * G + g);
      }
    }
    if (itn < 0) break;  // workgroup-uniform
    it = itn;
    slab = slab_n;
    bpc = bpc_n;
    itn = next_valid(it + stride);
    if (itn >= 0) coords(itn, slab_n, bpc_n);
    if (npair == 1) {  // the pair-end update above already moved to this item; its next pair is the following item's
#pragma unroll
      for (int g = 0; g < G; ++g) next_rows[g] = rowp(bpc_n, g);
    }
  }
}

// Output-stationary form for config 4's item shape (2M = 128 output columns, T = 256 samples, A % 64 == 0): one
// workgroup of NW waves per (b, p, c) item holds the whole Y[256 x 128] in accumulators (wave w: 16 RG rows, RG =
// 16 / NW row groups, all 8 column tiles) and streams K = 2A through LDS in chunks of 64 rows (two k-steps): the
// chunk's table rows are read as whole 512-byte rows (thread = 8 rows x 16 / NW columns, converted to one hi and one
// lo fragment per column), double-buffered, and each coefficient fragment feeds RG row groups x 2 MFMAs.  Against
// the 32-column slab kernels this reads every item's voltages once instead of once per slab (4x at config 4) and the
// table in whole rows instead of 128-byte row pieces.  Per output the MFMA sequence is the slab kernels' (k-steps in
// order, hi then lo): bitwise the same sums.  NW = 8: 2 row groups per wave, 128 VGPRs, two workgroups (16 waves)
// per CU; NW = 4: 4 row groups, 256 VGPRs, two workgroups (8 waves).  Mode (diagnostics): 4 no stores, 8 no voltage
// loads, 16 no table loads.
constexpr int kOsCols = 128, kOsRows = 256;
constexpr size_t kOsLds = 2 * 2 * 8 * 2 * 64 * 16;  // 2 buffers x 2 steps x 8 tiles x 2 limbs x 64 lanes x 16 B

template <bool Signed, int Mode, int NW, int Occ = NW / 2>
__global__ __launch_bounds__(NW * 64, Occ) void beamform_table_os_kernel(const uint8_t* __restrict__ x,
                                                                      const float* __restrict__ w,
                                                                      float* __restrict__ y, int A) {
  static_assert(kDiagBuild || Mode == 0, "diagnostic Mode bits in a product instantiation");
  extern __shared__ __attribute__((aligned(16))) half8 lds[];
  constexpr int NTL = kOsCols / 16, RG = 16 / NW, M2 = kOsCols, T = kOsRows;
  constexpr int CPT = 16 / NW;            // table columns per thread
  constexpr int UPR = kOsCols / CPT;      // threads per row octet
  constexpr int kBuf = 2 * NTL * 2 * 64;  // half8 per buffer
  typedef float fvec __attribute__((ext_vector_type(CPT)));
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 4, tl = lane & 15;
  const size_t bpc = blockIdx.x;
  const int K2 = 2 * A, nk = K2 / 64;  // chunks (even: A % 64 == 0)
  const uint8_t* xp = x + bpc * static_cast<size_t>(T) * K2;
  const float* wp = w + bpc * static_cast<size_t>(K2) * M2;
  float* yp = y + bpc * static_cast<size_t>(T) * M2;

  const int ro = tid / UPR, cq = tid % UPR;  // rows 8 ro .. 8 ro + 7 of a chunk x columns CPT cq ..
  fvec tv[8];
  auto tload = [&](int kc) __attribute__((always_inline)) {
    if constexpr (Mode & 16) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < CPT; ++i) tv[j][i] = 1e-3f * (j + i) + 3e-3f * kc;
      return;
    }
    // a uniform base + one 32-bit lane offset (the item's table is 2A x 128 floats)
    const uint32_t off = static_cast<uint32_t>(((kc * 64 + 8 * ro) * M2 + CPT * cq) * 4);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      tv[j] = *reinterpret_cast<const fvec*>(reinterpret_cast<const char*>(wp) + off + j * M2 * 4);
  };
  auto tstore = [&](int buf) __attribute__((always_inline)) {
    half8* L = lds + buf * kBuf;
    const int sl = ro >> 2, hh = ro & 3;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int col = CPT * cq + i;
      half8 hi, lo;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float wv = tv[j][i];
        hi[j] = static_cast<_Float16>(wv);
        lo[j] = static_cast<_Float16>(wv - static_cast<float>(hi[j]));  // exact difference, then rounded
      }
      const int slot = ((sl * NTL + (col >> 4)) * 2) * 64 + (col & 15) + 16 * hh;
      L[slot] = hi;
      L[slot + 64] = lo;
    }
  };
  // voltages: row group rg of this wave = rows (RG wave + rg) 16 + tl; one 16-byte load = both k-steps of a chunk
  const uint32_t xoff = static_cast<uint32_t>((RG * wave * 16 + tl) * K2 + 16 * h);  // lane offset in the item
  auto xload = [&](int kc, uint4 (&xr)[RG]) __attribute__((always_inline)) {
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {
      if constexpr (Mode & 8)
        xr[rg] = uint4{static_cast<uint32_t>(kc + tl), static_cast<uint32_t>(rg), static_cast<uint32_t>(kc - tl), 7u};
      else
        xr[rg] = *reinterpret_cast<const uint4*>(xp + (xoff + static_cast<uint32_t>(rg * 16 * K2 + 64 * kc)));
    }
  };
  f32x4 acc[RG][NTL];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[rg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // contract the chunk in LDS buffer `buf` from the voltages in xr, then (next >= 0) reload xr with chunk `next`:
  // the registers are free once re-dealt, so one voltage buffer keeps a chunk in flight
  auto contract = [&](int buf, uint4 (&xr)[RG], int next) __attribute__((always_inline)) {
    const half8* L = lds + buf * kBuf;
    half8 v[RG];
    uint32_t r1[RG][2];  // step 1's re-dealt dwords, converted after step 0
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) {  // the ring kernel's re-deal: both steps' 8-byte fragments from one load
      auto x0 = __builtin_amdgcn_permlane16_swap(xr[rg].x, xr[rg].z, false, false);
      auto x1 = __builtin_amdgcn_permlane16_swap(xr[rg].y, xr[rg].w, false, false);
      auto y0 = __builtin_amdgcn_permlane32_swap(x0[0], x0[1], false, false);
      auto y1 = __builtin_amdgcn_permlane32_swap(x1[0], x1[1], false, false);
      v[rg] = bytes8_to_frag<Signed>(y0[0], y1[0]);
      r1[rg][0] = y0[1];
      r1[rg][1] = y1[1];
    }
    if (next >= 0) xload(next, xr);  // uniform
#pragma unroll
    for (int sl = 0; sl < 2; ++sl) {
      if (sl == 1) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) v[rg] = bytes8_to_frag<Signed>(r1[rg][0], r1[rg][1]);
      }
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int slot = ((sl * NTL + t) * 2) * 64 + lane;
        const half8 chi = L[slot], clo = L[slot + 64];
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) {
          acc[rg][t] = mfma(chi, v[rg], acc[rg][t]);
          acc[rg][t] = mfma(clo, v[rg], acc[rg][t]);
        }
      }
    }
  };

  uint4 xr[RG];
  tload(0);
  xload(0, xr);
  tstore(0);
  __syncthreads();
  // chunk pairs: kc in LDS buffer 0, kc + 1 in buffer 1; each chunk's successor table is requested before the chunk
  // is contracted (its voltages right after the re-deal: vmcnt is in order, so the table conversion waits for the
  // table only).  The last pair requests nothing past the item: a uniform branch in the one loop -- peeled, the last
  // pair kept its own copies of the loop's thread-index offsets live across the loop (spills).
  for (int kc = 0; kc < nk; kc += 2) {  // one loop, the last pair's successor requests skipped by a uniform branch
    tload(min(kc + 1, nk - 1));
    contract(0, xr, kc + 1);
    tstore(1);
    __syncthreads();
    const bool more = kc + 2 < nk;
    if (more) tload(kc + 2);
    contract(1, xr, more ? kc + 2 : -1);
    if (more) tstore(0);
    __syncthreads();
  }

#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    float* orow = yp + static_cast<size_t>((RG * wave + rg) * 16 + tl) * M2 + 4 * h;
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      if constexpr (Mode & 4) {
        if (acc[rg][t][0] == 1234.5f) orow[t] = acc[rg][t][1];
      } else {
        *reinterpret_cast<f32x4*>(orow + 16 * t) = acc[rg][t];
      }
    }
  }
}

// The output-stationary kernel's shape conditions (the caller's buffers: 16-byte aligned x and w rows).
inline bool table_os_fits(int NB, int A, int M, const uint8_t* x, const float* w) {
  return 2 * M == kOsCols && NB * kSamplesPerBlock == kOsRows && A % 64 == 0 && A >= 64 &&
         (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
}

template <bool Signed, int Mode = 0, int NW = 8, int Occ = NW / 2>
int launch_table_os(const uint8_t* x, const float* w, float* y, long long bpc, int A, hipStream_t st) {
  BF_REQUIRE(bpc < (1LL << 31), "bf_beamform: grid too large");
  hipLaunchKernelGGL((beamform_table_os_kernel<Signed, Mode, NW, Occ>), dim3(static_cast<unsigned>(bpc)), dim3(NW * 64),
                     kOsLds, st, x, w, y, A);
  BF_LAUNCHED("beamform_table_os_kernel");
}

template <bool Signed, int NTS, bool Vec8>
int launch_table(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                 hipStream_t st) {
  const int nslabs = (NT + NTS - 1) / NTS;
  const size_t lds = coef_lds_bytes(S, NTS);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform: n_ants=%d too large for one coefficient slab", A);
  const int xcd = nslabs > 1;
  const long long grid = xcd ? (bpc + 7) / 8 * 8 * nslabs : bpc * nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform: grid too large");
  hipLaunchKernelGGL((beamform_table_kernel<Signed, NTS, Vec8>), dim3(static_cast<unsigned>(grid)), dim3(kThreads),
                     lds, st, x, w, y, NB, A, M, S, NT, nslabs, bpc, xcd);
  BF_LAUNCHED("beamform_table_kernel");
}

template <bool Signed, int NTS, int R, int Mode = 0, int Form = 0>
int launch_ring(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                hipStream_t st) {
  const int nslabs = (NT + NTS - 1) / NTS;
  const int Sp = (S + R - 1) / R * R;
  const size_t lds = coef_lds_bytes(Sp, NTS);
  BF_REQUIRE(lds <= kMaxLds, "bf_beamform: n_ants=%d too large for one coefficient slab", A);
  const int xcd = nslabs > 1;
  const long long grid = xcd ? (bpc + 7) / 8 * 8 * nslabs : bpc * nslabs;
  BF_REQUIRE(grid < (1LL << 31), "bf_beamform: grid too large");
  // Form 0: 16-byte loads when the rows allow them (A % 8 == 0, x 16-byte aligned); 1 (diagnostics): 8-byte loads
  const bool w16 = Form == 0 && A % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (w16)
    hipLaunchKernelGGL((beamform_table_ring_kernel<Signed, NTS, R, Mode, true>), dim3(static_cast<unsigned>(grid)),
                       dim3(kThreads), lds, st, x, w, y, NB, A, M, S, NT, nslabs, bpc, xcd);
  else
    hipLaunchKernelGGL((beamform_table_ring_kernel<Signed, NTS, R, Mode>), dim3(static_cast<unsigned>(grid)),
                       dim3(kThreads), lds, st, x, w, y, NB, A, M, S, NT, nslabs, bpc, xcd);
  BF_LAUNCHED("beamform_table_ring_kernel");
}

// The persistent ring kernel: UPT table units per thread (Sp * NTS / 4 == UPT), two workgroups per CU.
template <bool Signed, int NTS, int R, int UPT, int Mode = 0, int G = 2>
int launch_persist(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                   hipStream_t st) {
  const int nslabs = (NT + NTS - 1) / NTS;
  const int Sp = (S + R - 1) / R * R;
  const size_t lds = coef_lds_bytes(Sp, NTS);
  BF_REQUIRE(lds <= kMaxLds / 2 && Sp * NTS == 4 * UPT && A % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0,
             "bf_beamform: shape does not fit the persistent table kernel");
  const int xcd = nslabs > 1;
  const long long nitems = xcd ? (bpc + 7) / 8 * 8 * nslabs : bpc * nslabs;
  // two workgroups per CU; with the XCD item order the grid is a multiple of 8 (an item's XCD is its workgroup's:
  // nitems is then a multiple of 8 too), otherwise any size
  const int n_cu = cu_count();
  const long long grid = std::min<long long>(nitems, xcd ? 2LL * n_cu / 8 * 8 : 2LL * n_cu);
  BF_REQUIRE(grid > 0 && (!xcd || grid % 8 == 0), "bf_beamform: persistent grid");
  hipLaunchKernelGGL((beamform_table_persist_kernel<Signed, NTS, R, UPT, Mode, G>), dim3(static_cast<unsigned>(grid)),
                     dim3(kThreads), lds, st, x, w, y, NB, A, M, S, NT, nslabs, bpc, xcd, nitems);
  BF_LAUNCHED("beamform_table_persist_kernel");
}

template <bool Signed, int NTS>
int dispatch_vec(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                 hipStream_t st) {
  const char* e = diag_env("BF_TABLE_BASIC");  // tests: force the basic kernel
  if (A % 4 == 0 && !(e && e[0] == '1')) {
    // ring depth: the k-steps of a row, up to 16 (the steps are padded to a multiple of R); long rows only
    if (S >= 16 && coef_lds_bytes((S + 15) / 16 * 16, NTS) <= kMaxLds) {
      // 256-antenna rows in two-workgroup slabs (config 4): the persistent form, the next slab loaded under the
      // current item's contraction
      if constexpr (NTS == 2)
        if ((S + 15) / 16 == 1 && A % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
            (bpc >= 8))
          return launch_persist<Signed, 2, 16, 8>(x, w, y, bpc, NB, A, M, S, NT, st);
      return launch_ring<Signed, NTS, 16>(x, w, y, bpc, NB, A, M, S, NT, st);
    }
    if (S >= 8 && coef_lds_bytes((S + 7) / 8 * 8, NTS) <= kMaxLds)
      return launch_ring<Signed, NTS, 8>(x, w, y, bpc, NB, A, M, S, NT, st);
    // 4..7 k-steps (64 antennas: config 3): a 4-deep ring
    const char* r4 = diag_env("BF_TABLE_RING4");  // measurement: 0 keeps the basic kernel
    if (S >= 4 && !(r4 && r4[0] == '0') && coef_lds_bytes((S + 3) / 4 * 4, NTS) <= kMaxLds)
      return launch_ring<Signed, NTS, 4>(x, w, y, bpc, NB, A, M, S, NT, st);
  }
  if (A % 4 == 0) return launch_table<Signed, NTS, true>(x, w, y, bpc, NB, A, M, S, NT, st);
  return launch_table<Signed, NTS, false>(x, w, y, bpc, NB, A, M, S, NT, st);
}

template <bool Signed>
int dispatch_table(const uint8_t* x, const float* w, float* y, long long bpc, int NB, int A, int M, int S, int NT,
                   hipStream_t st) {
  const char* os = diag_env("BF_TABLE_OS");  // measurement: 0 keeps the slab kernels
  // 4 waves per item (256 VGPRs, two workgroups per CU), spill-free in the one-loop form: 791 us at config 4 against
  // 853 for the 8-wave form (128 VGPRs, spills 24-40 B/lane) and 933 for the 8-wave form bounded to 3 waves per
  // SIMD (no spill, one workgroup per CU), profiles/r4_s_table_os_ab.txt
  if (table_os_fits(NB, A, M, x, w) && !(os && os[0] == '0')) return launch_table_os<Signed, 0, 4>(x, w, y, bpc, A, st);
  // Long rows (>= 16 k-steps: 256+ antennas): the widest slab whose staged fragments leave room for a second
  // workgroup per CU, so one workgroup's table staging overlaps the other's contraction (cfg4: a 128 KiB slab held
  // one workgroup per CU and ran 3.1 ms); the slabs' re-reads of x hit L2 (XCD-grouped slabs).
  if (S >= 16) {
    const size_t half = kMaxLds / 2;
    if (NT >= 4 && coef_lds_bytes((S + 15) / 16 * 16, 4) <= half)
      return dispatch_vec<Signed, 4>(x, w, y, bpc, NB, A, M, S, NT, st);
    if (NT >= 2 && coef_lds_bytes((S + 15) / 16 * 16, 2) <= half)
      return dispatch_vec<Signed, 2>(x, w, y, bpc, NB, A, M, S, NT, st);
  }
  // Otherwise the widest slab whose fragments fit LDS (fewer slabs = fewer re-reads of x).
  if (NT >= 8 && coef_lds_bytes(S, 8) <= kMaxLds) return dispatch_vec<Signed, 8>(x, w, y, bpc, NB, A, M, S, NT, st);
  if (NT >= 4 && coef_lds_bytes(S, 4) <= kMaxLds) return dispatch_vec<Signed, 4>(x, w, y, bpc, NB, A, M, S, NT, st);
  if (NT >= 2 && coef_lds_bytes(S, 2) <= kMaxLds) return dispatch_vec<Signed, 2>(x, w, y, bpc, NB, A, M, S, NT, st);
  return dispatch_vec<Signed, 1>(x, w, y, bpc, NB, A, M, S, NT, st);
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

#ifdef BF_DIAG
#include "diag/beamform_diag.inc"
#endif
