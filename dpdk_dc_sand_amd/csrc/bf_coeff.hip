// Steering-coefficient generators.
//
// bf_coeff_gen      -- Python layout (B, P, C, 2A, 2M) f32, bit-exact to CoeffGenerator.cpu_coeffs
//                      (unit_test/coeff_generator_cpu.py:78-187); replaces run_coeff_gen
//                      (beamforming/coeff_generator.py:12-103) without its ant/beam transposition.
// bf_coeff_gen_time -- compact time-dependent form (n_times, C, A, M) complex f32 or f16, the C++ study's
//                      grouped_channels_and_timestamps / b16BitOutput modes (BeamformerKernels.cu:121-189)
//                      with the Python sign convention.
//
// Work is C*A*M phasors (tiny next to the beamform); the kernels are write-bound.  One thread per (c, a, m),
// m fastest, so the (cos, sin) / (-sin, cos) float2 pairs of consecutive threads are contiguous in a row of
// the 2M-wide output.
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cstdlib>

#include "bf_common.hpp"
#include "bf_phase.hpp"

namespace bf {

// One thread per (c, a, m): grid (ceil(A*M / 256), C), 32-bit index math (the grid-stride form with 64-bit
// divisions spent more time on index arithmetic and serial load latency than on the phasor or the writes).
__global__ __launch_bounds__(256) void coeff_gen_kernel(const float4* __restrict__ dv, float* __restrict__ out,
                                                        int B, int P, int C, int A, int M, long long base_ch,
                                                        double ctot, double ts) {
  const int am = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  if (am >= A * M) return;
  const int c = static_cast<int>(blockIdx.y);
  const int a = am / M, m = am - a * M;
  const float4 d = dv[(static_cast<size_t>(c) * M + m) * A + a];  // delay_vals[c][m][a]
  float re, im;
  steering_coeff(d, static_cast<double>(base_ch + c), make_phase(ctot, ts), 0.0, &re, &im);
  const float2 row0 = make_float2(re, im);   // W[2a][2m], W[2a][2m+1]
  const float2 row1 = make_float2(-im, re);  // W[2a+1][2m], W[2a+1][2m+1]
  const size_t plane = static_cast<size_t>(2 * A) * (2 * M);  // one (b, p, c) coefficient matrix
  float* w = out + static_cast<size_t>(c) * plane + static_cast<size_t>(2 * a) * (2 * M) + 2 * m;
  const size_t bp_stride = static_cast<size_t>(C) * plane;
  for (int bp = 0; bp < B * P; ++bp) {
    *reinterpret_cast<float2*>(w + bp * bp_stride) = row0;
    *reinterpret_cast<float2*>(w + bp * bp_stride + 2 * M) = row1;
  }
}

// Tiled form (32 antennas x 32 beams per workgroup): the delay model is [c][m][a] (antenna fastest) and the table
// [c][2a][2m] (beam fastest), so the one-thread-per-(a, m) kernel above reads the model with a 4 KiB lane stride at
// 256 antennas (a 64-byte line per 16-byte entry: 4x over-fetch of a 1 GiB model at config 4).  Here the tile's
// model rows are read coalesced (antenna fastest) into LDS, and each thread then takes its entries beam-fastest
// for the phasor and the coalesced table stores.
constexpr int kCoefTile = 32;
__global__ __launch_bounds__(256) void coeff_gen_tile_kernel(const float4* __restrict__ dv, float* __restrict__ out,
                                                             int B, int P, int C, int A, int M, long long base_ch,
                                                             double ctot, double ts) {
  __shared__ float4 tile[kCoefTile][kCoefTile + 1];  // [a][m], padded row
  const int c = static_cast<int>(blockIdx.y);
  const int ntm = (M + kCoefTile - 1) / kCoefTile;
  const int a0 = static_cast<int>(blockIdx.x) / ntm * kCoefTile, m0 = static_cast<int>(blockIdx.x) % ntm * kCoefTile;
  const int t = static_cast<int>(threadIdx.x);
  {
    const int la = t & 31;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int lm = (t >> 5) + 8 * j;
      const int a = min(a0 + la, A - 1), m = min(m0 + lm, M - 1);
      tile[la][lm] = dv[(static_cast<size_t>(c) * M + m) * A + a];  // delay_vals[c][m][a]
    }
  }
  __syncthreads();
  const int lm = t & 31, m = m0 + lm;
  const size_t plane = static_cast<size_t>(2 * A) * (2 * M);  // one (b, p, c) coefficient matrix
  const size_t bp_stride = static_cast<size_t>(C) * plane;
  const PhaseK k = make_phase(ctot, ts);
  const double ch = static_cast<double>(base_ch + c);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int la = (t >> 5) + 8 * j, a = a0 + la;
    if (a >= A || m >= M) continue;
    float re, im;
    steering_coeff(tile[la][lm], ch, k, 0.0, &re, &im);
    const float2 row0 = make_float2(re, im);   // W[2a][2m], W[2a][2m+1]
    const float2 row1 = make_float2(-im, re);  // W[2a+1][2m], W[2a+1][2m+1]
    float* w = out + static_cast<size_t>(c) * plane + static_cast<size_t>(2 * a) * (2 * M) + 2 * m;
    for (int bp = 0; bp < B * P; ++bp) {
      *reinterpret_cast<float2*>(w + bp * bp_stride) = row0;
      *reinterpret_cast<float2*>(w + bp * bp_stride + 2 * M) = row1;
    }
  }
}

// Block form (the default): one workgroup per (c, run of na antennas).  The run's 2 na rows of a (2A, 2M) plane are
// ONE contiguous 16 na M-byte piece of every (b, p) plane, so the workgroup evaluates its na M phasors once (model
// rows read antenna-fastest, coalesced), lays the piece out in LDS (one 16-byte pad per antenna pair of rows), and
// then streams it to the B P planes with 16-byte stores -- whole contiguous runs, no partial lines (the per-(a, m)
// kernels above store 8-byte pairs into rows 2M floats apart).  Cache & 2: non-temporal stores (the table is
// written once and read by the multiply much later).
constexpr int kCoefBlockLds = 32 * 1024;
__host__ __device__ inline int coef_block_ants(int A, int M) {
  int na = kCoefBlockLds / 16 / (M + 1);
  if (na >= 16) na &= ~15;
  return na < A ? na : A;
}

template <int Cache>
__global__ __launch_bounds__(256) void coeff_gen_block_kernel(const float4* __restrict__ dv, float* __restrict__ out,
                                                              int BP, int C, int A, int M, int na, int bpg,
                                                              long long base_ch, double ctot, double ts) {
  extern __shared__ __attribute__((aligned(16))) float4 img4[];  // [antenna][M + 1] float4 (rows 2a, 2a + 1 + pad)
  float* img = reinterpret_cast<float*>(img4);
  const int c = static_cast<int>(blockIdx.y);
  const int a0 = static_cast<int>(blockIdx.x) * na;
  const int nb = min(na, A - a0);
  const int pitch = 4 * (M + 1);  // floats per antenna
  const PhaseK k = make_phase(ctot, ts);
  const double ch = static_cast<double>(base_ch + c);
  for (int e = static_cast<int>(threadIdx.x); e < nb * M; e += 256) {
    const int m = e / nb, la = e - m * nb;
    const float4 d = dv[(static_cast<size_t>(c) * M + m) * A + a0 + la];  // delay_vals[c][m][a]
    float re, im;
    steering_coeff(d, ch, k, 0.0, &re, &im);
    float* r = img + la * pitch + 2 * m;
    *reinterpret_cast<float2*>(r) = make_float2(re, im);           // W[2a][2m], W[2a][2m+1]
    *reinterpret_cast<float2*>(r + 2 * M) = make_float2(-im, re);  // W[2a+1][2m], W[2a+1][2m+1]
  }
  __syncthreads();
  const size_t plane = static_cast<size_t>(2 * A) * (2 * M);
  const size_t bp_stride = static_cast<size_t>(C) * plane;
  float4* dst = reinterpret_cast<float4*>(out + static_cast<size_t>(c) * plane + static_cast<size_t>(2 * a0) * (2 * M));
  for (int j = static_cast<int>(threadIdx.x); j < nb * M; j += 256) {  // 16-byte pieces of the run
    const int la = j / M;
    const float4 v = img4[la * (M + 1) + (j - la * M)];
    const int bp1 = min(BP, (static_cast<int>(blockIdx.z) + 1) * bpg);
    for (int bp = static_cast<int>(blockIdx.z) * bpg; bp < bp1; ++bp) {
      float4* o = dst + static_cast<size_t>(bp) * (bp_stride >> 2) + j;
      if constexpr (Cache & 2) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<f4v*>(o));
      } else {
        *o = v;
      }
    }
  }
}

template <bool F16>
__global__ __launch_bounds__(256) void coeff_gen_time_kernel(const float4* __restrict__ dv, int delay_channels,
                                                             void* __restrict__ out, int n_times, int C, int A, int M,
                                                             long long base_ch, double ctot, double ts, double t0,
                                                             double dt_step) {
  const long long n = static_cast<long long>(n_times) * C * A * M;
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  for (long long idx = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += stride) {
    const int m = static_cast<int>(idx % M);
    long long r = idx / M;
    const int a = static_cast<int>(r % A);
    r /= A;
    const int c = static_cast<int>(r % C);
    const int t = static_cast<int>(r / C);
    const int cd = delay_channels == 1 ? 0 : c;
    const float4 d = dv[(static_cast<size_t>(cd) * M + m) * A + a];
    float re, im;
    steering_coeff(d, static_cast<double>(base_ch + c), make_phase(ctot, ts), t0 + t * dt_step, &re, &im);
    if constexpr (F16) {
      reinterpret_cast<__half2*>(out)[idx] = __floats2half2_rn(re, im);
    } else {
      reinterpret_cast<float2*>(out)[idx] = make_float2(re, im);
    }
  }
}

// The C++ study's own time-dependent convention (calculate_beamweights_grouped_channels_and_timestamps,
// BeamformerKernels.cu:155-170), restated operation for operation in float32: the delay RATE in the channel term and
// the opposite sign of the Python path, dt = t * Ts * fft_size, precise sincosf (the reference's
// __sincosf is its fast-math form; its own golden, BeamformerCoefficientTest.cu:294-337, uses cos / sin).  Delay
// model [a * M + m] as 4 floats (delay_s, delay_rate, phase_rad, phase_rate) -- the study's struct delay_vals
// (BeamformerParameters.h:61-66) with its antenna-major (a, beam) index -- output [t][c][a][m] complex.
template <bool F16>
__global__ __launch_bounds__(256) void coeff_gen_time_study_kernel(const float4* __restrict__ dv,
                                                                   void* __restrict__ out, int n_times, int C, int A,
                                                                   int M, float ts, int fft_size) {
  const long long n = static_cast<long long>(n_times) * C * A * M;
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  const float pi = 3.14159265358979323846f;
  for (long long idx = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; idx < n; idx += stride) {
#pragma clang fp contract(off)  // separate roundings, as the study's float expressions
    const int am = static_cast<int>(idx % (static_cast<long long>(A) * M));
    long long r = idx / (static_cast<long long>(A) * M);
    const int c = static_cast<int>(r % C);
    const int t = static_cast<int>(r / C);
    const float4 d = dv[am];
    const float delta_time = t * ts * fft_size;
    const float delta_delay = d.y * delta_time;
    const float delta_phase = d.w * delta_time;
    const float delay_n2 = (d.x + delta_delay) * (static_cast<float>(C) / 2.0f) * pi / (ts * C);  // C / 2.0f: odd C too
    const float delay_n = (d.y + delta_delay) * c * pi / (ts * C);
    const float phase0 = d.z - delay_n2 + delta_phase;
    const float rotation = delay_n + phase0;
    float sn, cs;
    sincosf(rotation, &sn, &cs);
    if constexpr (F16) {
      reinterpret_cast<__half2*>(out)[idx] = __floats2half2_rn(cs, sn);
    } else {
      reinterpret_cast<float2*>(out)[idx] = make_float2(cs, sn);
    }
  }
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 256LL * 16) g = 256LL * 16;  // grid-stride beyond 16 blocks per CU
  return static_cast<int>(g < 1 ? 1 : g);
}

}  // namespace bf

extern "C" int bf_coeff_gen(const float* delay_vals, float* out, int B, int P, int C, int Ctot, int A, int M,
                            int xeng_id, double sample_period, void* stream) {
  BF_REQUIRE(delay_vals && out, "bf_coeff_gen: null pointer");
  BF_REQUIRE(B > 0 && P > 0 && C > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_coeff_gen: bad shape B=%d P=%d C=%d A=%d M=%d Ctot=%d xeng_id=%d", B, P, C, A, M, Ctot, xeng_id);
  BF_REQUIRE(sample_period > 0.0, "bf_coeff_gen: sample_period must be > 0");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 7) == 0,
             "bf_coeff_gen: misaligned buffer");
  BF_REQUIRE(static_cast<long long>(A) * M < (1LL << 31) && C < 65536, "bf_coeff_gen: shape too large");
  const char* form = bf::diag_env("BF_COEFF_FORM");  // measurement: "thread" / "tile" = the per-(a, m) kernels
  const int na = bf::coef_block_ants(A, M);
  // the block form stores 16-byte pieces (every antenna pair's rows start 16 M bytes apart): it needs a 16-byte
  // aligned table; an 8-byte aligned one (a C-ABI caller's offset pointer) takes the per-(a, m) kernels below
  if (!form && na >= 1 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    const unsigned gx = static_cast<unsigned>((A + na - 1) / na);
    const size_t lds = static_cast<size_t>(na) * (M + 1) * 16;
    const char* nt = bf::diag_env("BF_COEFF_NT");
    const char* bg = bf::diag_env("BF_COEFF_BPG");  // measurement: (b, p) planes per workgroup
    // up to 4 (b, p) planes per workgroup: cfg3 (16 planes) 245 -> 189 us, non-temporal (plain 245 us); one plane
    // per workgroup recomputes the phasors too often (300 us) -- profiles/r3_k_ops_ab.txt
    const int bpg = bg ? std::max(1, atoi(bg)) : std::min(B * P, 4);
    const unsigned gz = static_cast<unsigned>((B * P + bpg - 1) / bpg);
    const auto dv = reinterpret_cast<const float4*>(delay_vals);
    const long long base = static_cast<long long>(C) * xeng_id;
    if (nt && nt[0] == '0')
      hipLaunchKernelGGL(bf::coeff_gen_block_kernel<0>, dim3(gx, static_cast<unsigned>(C), gz), dim3(256), lds,
                         bf::as_stream(stream), dv, out, B * P, C, A, M, na, bpg, base, static_cast<double>(Ctot),
                         sample_period);
    else
      hipLaunchKernelGGL(bf::coeff_gen_block_kernel<2>, dim3(gx, static_cast<unsigned>(C), gz), dim3(256), lds,
                         bf::as_stream(stream), dv, out, B * P, C, A, M, na, bpg, base, static_cast<double>(Ctot),
                         sample_period);
    BF_LAUNCHED("coeff_gen_block_kernel");
  }
  if (A >= 32 && M >= 32 && !(form && form[0] == 't' && form[1] == 'h')) {  // many antennas and beams: the tiled, coalesced-read form
    const unsigned gx = static_cast<unsigned>(((A + bf::kCoefTile - 1) / bf::kCoefTile) *
                                              ((M + bf::kCoefTile - 1) / bf::kCoefTile));
    hipLaunchKernelGGL(bf::coeff_gen_tile_kernel, dim3(gx, static_cast<unsigned>(C)), dim3(256), 0,
                       bf::as_stream(stream), reinterpret_cast<const float4*>(delay_vals), out, B, P, C, A, M,
                       static_cast<long long>(C) * xeng_id, static_cast<double>(Ctot), sample_period);
    BF_LAUNCHED("coeff_gen_tile_kernel");
  }
  const unsigned gx = static_cast<unsigned>((static_cast<long long>(A) * M + 255) / 256);
  hipLaunchKernelGGL(bf::coeff_gen_kernel, dim3(gx, static_cast<unsigned>(C)), dim3(256), 0, bf::as_stream(stream),
                     reinterpret_cast<const float4*>(delay_vals), out, B, P, C, A, M,
                     static_cast<long long>(C) * xeng_id, static_cast<double>(Ctot), sample_period);
  BF_LAUNCHED("coeff_gen_kernel");
}

extern "C" int bf_coeff_gen_time(const float* delay_vals, int delay_channels, void* out, int out_fp16,
                                 int n_times, int C, int Ctot, int A, int M, int xeng_id, double sample_period,
                                 double t0, double dt_step, void* stream) {
  BF_REQUIRE(delay_vals && out, "bf_coeff_gen_time: null pointer");
  BF_REQUIRE(n_times > 0 && C > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_coeff_gen_time: bad shape");
  BF_REQUIRE(delay_channels == 1 || delay_channels == C, "bf_coeff_gen_time: delay_channels must be 1 or C");
  BF_REQUIRE(sample_period > 0.0, "bf_coeff_gen_time: sample_period must be > 0");
  const long long n = static_cast<long long>(n_times) * C * A * M;
  const auto dv = reinterpret_cast<const float4*>(delay_vals);
  const long long base = static_cast<long long>(C) * xeng_id;
  if (out_fp16) {
    hipLaunchKernelGGL(bf::coeff_gen_time_kernel<true>, dim3(bf::grid_for(n)), dim3(256), 0, bf::as_stream(stream),
                       dv, delay_channels, out, n_times, C, A, M, base, static_cast<double>(Ctot), sample_period, t0,
                       dt_step);
  } else {
    hipLaunchKernelGGL(bf::coeff_gen_time_kernel<false>, dim3(bf::grid_for(n)), dim3(256), 0,
                       bf::as_stream(stream), dv, delay_channels, out, n_times, C, A, M, base,
                       static_cast<double>(Ctot), sample_period, t0, dt_step);
  }
  BF_LAUNCHED("coeff_gen_time_kernel");
}

extern "C" int bf_coeff_gen_time_study(const float* delay_vals, void* out, int out_fp16, int n_times, int C, int A,
                                       int M, float sample_period, int fft_size, void* stream) {
  BF_REQUIRE(delay_vals && out, "bf_coeff_gen_time_study: null pointer");
  BF_REQUIRE(n_times > 0 && C > 0 && A > 0 && M > 0 && fft_size > 0, "bf_coeff_gen_time_study: bad shape");
  BF_REQUIRE(sample_period > 0.0f, "bf_coeff_gen_time_study: sample_period must be > 0");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0, "bf_coeff_gen_time_study: misaligned delay_vals");
  const long long n = static_cast<long long>(n_times) * C * A * M;
  const auto dv = reinterpret_cast<const float4*>(delay_vals);
  if (out_fp16)
    hipLaunchKernelGGL(bf::coeff_gen_time_study_kernel<true>, dim3(bf::grid_for(n)), dim3(256), 0,
                       bf::as_stream(stream), dv, out, n_times, C, A, M, sample_period, fft_size);
  else
    hipLaunchKernelGGL(bf::coeff_gen_time_study_kernel<false>, dim3(bf::grid_for(n)), dim3(256), 0,
                       bf::as_stream(stream), dv, out, n_times, C, A, M, sample_period, fft_size);
  BF_LAUNCHED("coeff_gen_time_study_kernel");
}
