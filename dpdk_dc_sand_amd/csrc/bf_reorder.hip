// Pre-beamform reorder: u16 (B, A, C, T, P) -> (B, P, C, T/16, 16, A), bit-exact.
// Replaces the mako/PyCUDA kernel prebeamform_reorder (beamforming/kernels/prebeamform_reorder_kernel.mako:37-93),
// contract = beamforming/reorder.py:40-42.
//
// The reference kernel moves one u16 per thread with A-strided scattered stores.  Here one workgroup owns a
// (b, c, time-chunk) tile: every antenna's contiguous run of TT*4 bytes is loaded with 16-byte coalesced
// loads into an LDS image [A][TT*4 (+4 pad)], and the output -- which for a fixed (b, p, c) and time chunk
// is ONE contiguous run of TT*A u16 -- is written with 16-byte coalesced stores (8 antennas per lane).
// Loads are issued in batches of 8 per thread before their LDS writes (a load-then-write loop paid one HBM latency
// per iteration).  For A % 8 == 0 a thread reads the 8 antennas' dwords of one time sample (both pols) and splits
// them with v_perm into the two pols' outputs; other A use 2-byte transposed reads.  The odd dword pitch (TT + 1)
// keeps the transposed LDS reads (nearly) bank-conflict-free.
#include <cstdlib>

#include "bf_common.hpp"

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

namespace bf {

// Cache: bit 1 non-temporal voltage loads, bit 2 non-temporal stores (both streams are touched once).
template <bool Oct, int Cache>
__global__ __launch_bounds__(256) void reorder_kernel(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                      int A, int C, int T, int TT, int nchunk, int xcd_range) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_u32[];
  // XCD-range order (grid % 8 == 0): workgroups are dealt round-robin to the 8 XCDs, so XCD x takes the contiguous
  // tile range [x N/8, (x+1) N/8) and streams one contiguous window per antenna (as the fused item kernels)
  const long long tile = xcd_range ? (blockIdx.x & 7) * static_cast<long long>(gridDim.x >> 3) + (blockIdx.x >> 3)
                                   : static_cast<long long>(blockIdx.x);
  const int chunk = static_cast<int>(tile % nchunk);
  const long long bc = tile / nchunk;
  const long long b = bc / C;
  const int c = static_cast<int>(bc % C);
  const int t0 = chunk * TT;
  const int pitch = TT + 1;  // dwords per antenna row
  const int quads = TT >> 2;
  const int nq = A * quads;

  // 1. antenna runs -> LDS.  in[b][a][c][t][p][ri], one 16-byte load = 4 time samples x 2 pols x (re, im).  Batches
  // of 8 loads per thread are all issued (unconditional, clamped) before their LDS writes.
  for (int base = 0; base < nq; base += 8 * 256) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = min(base + k * 256 + static_cast<int>(threadIdx.x), nq - 1);
      const int a = idx / quads;
      const int tq = idx - a * quads;
      const size_t src = ((static_cast<size_t>(b) * A + a) * C + c) * static_cast<size_t>(T) * 4 +
                         static_cast<size_t>(t0 + 4 * tq) * 4;
      const uint4* ps = reinterpret_cast<const uint4*>(in + src);
      if constexpr (Cache & 1) {
        const u32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(ps));
        v[k] = make_uint4(t[0], t[1], t[2], t[3]);
      } else {
        v[k] = *ps;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = base + k * 256 + static_cast<int>(threadIdx.x);
      if (idx < nq) {
        const int a = idx / quads;
        const int tq = idx - a * quads;
        uint32_t* row = lds_u32 + a * pitch + 4 * tq;
        row[0] = v[k].x;
        row[1] = v[k].y;
        row[2] = v[k].z;
        row[3] = v[k].w;
      }
    }
  }
  __syncthreads();

  // 2. LDS -> out[b][p][c][t][a][ri]: for each pol the chunk is TT*A contiguous u16 (16-byte aligned).
  uint8_t* dst0 = out + ((static_cast<size_t>(b) * 2 + 0) * C + c) * static_cast<size_t>(T) * A * 2 +
                  static_cast<size_t>(t0) * A * 2;
  uint8_t* dst1 = out + ((static_cast<size_t>(b) * 2 + 1) * C + c) * static_cast<size_t>(T) * A * 2 +
                  static_cast<size_t>(t0) * A * 2;
  if constexpr (Oct) {
    // A % 8 == 0: a thread owns (t, 8 antennas a0..a0+7): 8 dword reads give both pols' (re, im) of the 8 antennas
    // and one v_perm per output dword splits them into the pol-0 and pol-1 16-byte outputs (antenna group fastest
    // across lanes, so the stores are contiguous; the odd row pitch keeps the reads at most 2-way conflicted)
    const int ngrp = A >> 3;
    const int n_items = TT * ngrp;
    for (int it = threadIdx.x; it < n_items; it += 256) {
      const int t = it / ngrp;
      const int a0 = (it - t * ngrp) * 8;
      uint32_t d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = lds_u32[(a0 + j) * pitch + t];
      uint4 w0, w1;  // pol 0: low halves (u16 0) of each antenna's dword; pol 1: high halves
      w0.x = __builtin_amdgcn_perm(d[1], d[0], 0x05040100u);
      w0.y = __builtin_amdgcn_perm(d[3], d[2], 0x05040100u);
      w0.z = __builtin_amdgcn_perm(d[5], d[4], 0x05040100u);
      w0.w = __builtin_amdgcn_perm(d[7], d[6], 0x05040100u);
      w1.x = __builtin_amdgcn_perm(d[1], d[0], 0x07060302u);
      w1.y = __builtin_amdgcn_perm(d[3], d[2], 0x07060302u);
      w1.z = __builtin_amdgcn_perm(d[5], d[4], 0x07060302u);
      w1.w = __builtin_amdgcn_perm(d[7], d[6], 0x07060302u);
      const size_t off = (static_cast<size_t>(t) * A + a0) * 2;
      if constexpr (Cache & 2) {
        __builtin_nontemporal_store(u32x4_t{w0.x, w0.y, w0.z, w0.w}, reinterpret_cast<u32x4_t*>(dst0 + off));
        __builtin_nontemporal_store(u32x4_t{w1.x, w1.y, w1.z, w1.w}, reinterpret_cast<u32x4_t*>(dst1 + off));
      } else {
        *reinterpret_cast<uint4*>(dst0 + off) = w0;
        *reinterpret_cast<uint4*>(dst1 + off) = w1;
      }
    }
  } else {
    const uint16_t* lds_u16 = reinterpret_cast<const uint16_t*>(lds_u32);
    const int n_u16 = TT * A;
    for (int p = 0; p < 2; ++p) {
      uint8_t* dst = p ? dst1 : dst0;
      for (int e0 = threadIdx.x * 8; e0 < n_u16; e0 += blockDim.x * 8) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t pair = 0;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            const int e = e0 + 2 * j + half;
            const int t = e / A;
            const int a = e - t * A;
            // element (a, t, p) of the LDS image, in u16 units: a*pitch*2 + t*2 + p
            pair |= static_cast<uint32_t>(lds_u16[a * pitch * 2 + t * 2 + p]) << (16 * half);
          }
          w[j] = pair;
        }
        if constexpr (Cache & 2)
          __builtin_nontemporal_store(u32x4_t{w[0], w[1], w[2], w[3]},
                                      reinterpret_cast<u32x4_t*>(dst + static_cast<size_t>(e0) * 2));
        else
          *reinterpret_cast<uint4*>(dst + static_cast<size_t>(e0) * 2) = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
}

template <bool Oct>
void launch_reorder(int cache, dim3 grid, size_t lds, hipStream_t st, const uint8_t* in, uint8_t* out, int A, int C,
                    int T, int TT, int nchunk, int xcd_range) {
  switch (cache) {
    case 0: hipLaunchKernelGGL((reorder_kernel<Oct, 0>), grid, dim3(256), lds, st, in, out, A, C, T, TT, nchunk, xcd_range); break;
    case 1: hipLaunchKernelGGL((reorder_kernel<Oct, 1>), grid, dim3(256), lds, st, in, out, A, C, T, TT, nchunk, xcd_range); break;
    case 2: hipLaunchKernelGGL((reorder_kernel<Oct, 2>), grid, dim3(256), lds, st, in, out, A, C, T, TT, nchunk, xcd_range); break;
    default: hipLaunchKernelGGL((reorder_kernel<Oct, 3>), grid, dim3(256), lds, st, in, out, A, C, T, TT, nchunk, xcd_range); break;
  }
}

}  // namespace bf

namespace {
// the product's cache policy: non-temporal loads and stores (cfg3 831 -> 723 us, cfg4 447 -> 413 us;
// profiles/r3_j_ops_ab.txt)
constexpr int kReorderCache = 3;
}

extern "C" int bf_reorder(const uint8_t* in, uint8_t* out, int B, int A, int C, int T, void* stream) {
  BF_REQUIRE(in && out, "bf_reorder: null pointer");
  BF_REQUIRE(B > 0 && A > 0 && C > 0 && T > 0, "bf_reorder: bad shape B=%d A=%d C=%d T=%d", B, A, C, T);
  // the reference's check `T % (T // 16)` does not enforce this; the layout needs it.
  BF_REQUIRE(T % bf::kSamplesPerBlock == 0, "bf_reorder: n_samples_per_channel=%d must be a multiple of 16", T);
  BF_REQUIRE((reinterpret_cast<uintptr_t>(in) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0,
             "bf_reorder: buffers must be 16-byte aligned");
  // Largest power-of-two time chunk (>= 8, dividing T) whose LDS image fits 64 KiB.
  const char* ttc = bf::diag_env("BF_REORDER_TT");  // measurement: cap the time chunk
  const int tt_cap = ttc ? atoi(ttc) : 1 << 30;
  int TT = 1;
  while (TT * 2 <= T && T % (TT * 2) == 0 && TT * 2 <= tt_cap) TT *= 2;
  while (TT > 8 && static_cast<long long>(A) * (TT * 4 + 4) > 65536) TT /= 2;
  BF_REQUIRE(static_cast<long long>(A) * (TT * 4 + 4) <= 65536, "bf_reorder: n_ants=%d too large", A);
  const int nchunk = T / TT;
  const long long grid = static_cast<long long>(B) * C * nchunk;
  BF_REQUIRE(grid < (1LL << 31), "bf_reorder: grid too large");
  const size_t lds = static_cast<size_t>(A) * (TT + 1) * 4;
  const char* e = bf::diag_env("BF_REORDER_ORDER");  // measurement: "channel" keeps the plain order
  const int xcd_range = grid % 8 == 0 && !(e && e[0] == 'c');
  const char* nt = bf::diag_env("BF_REORDER_NT");  // measurement: cache policy bits (1 loads, 2 stores)
  const int cache = nt ? atoi(nt) : kReorderCache;
  if (A % 8 == 0)
    bf::launch_reorder<true>(cache, dim3(static_cast<unsigned>(grid)), lds, bf::as_stream(stream), in, out, A, C, T,
                             TT, nchunk, xcd_range);
  else
    bf::launch_reorder<false>(cache, dim3(static_cast<unsigned>(grid)), lds, bf::as_stream(stream), in, out, A, C, T,
                              TT, nchunk, xcd_range);
  BF_LAUNCHED("reorder_kernel");
}
