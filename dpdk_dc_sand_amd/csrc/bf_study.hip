// The C++ study's fused coefficient + beamform kernel in the study's OWN semantics:
// calculate_beamweights_and_beamform_single_channel (beamformer_coefficient_generator/BeamformerKernels.cu:192-367)
// as its harness checks it (BeamformerCoeffTest::verify_output, BeamformerCoefficientTest.cu:356-400).
//
// Per channel c, time t = 16 t_ex + t_in and beam m:
//   y_re = sum_a cos(rot) * x_re,   y_im = sum_a sin(rot) * x_im
// -- NOT a complex product (the study multiplies real by real and imaginary by imaginary, :313-316, and its
// golden mirrors that, :391-392) -- with rot the study's time-dependent phasor at (t, c, a, m): the delay RATE in the
// channel term and the sign opposite to the Python path, exactly bf_coeff_gen_time_study's expression
// (BeamformerKernels.cu:300-306).  The beam sum runs over the antennas in order, one float32 rounding per product and
// per addition, as the golden's loop (:385-394).
//
// What is NOT reproduced: the kernel's shadowed prefetch (:277-282 declare a new u32PrefetchedAntData inside the `if`,
// so every 16-sample chunk after the first beamforms the first chunk's voltages again) and its fixed 64 x 16 shape and
// 1024-thread block.  The golden, which reads every chunk, is the contract.
//
// Layouts (the study's, BeamformerParameters.h:36-45 and the golden's indices :378-383):
//   delay_vals f32 (M*A, 4), index m*A + a (the combined kernel's beam-major order, :307-316)
//   x          int8 [C][T/16][A][16][2]   (char2 [channels][time/16][station][16])
//   out        f32  [C][T/16][M][16][2]
//
// MI355X form: one workgroup per (channel, 16-sample chunk); the chunk's A x 16 complex samples are staged in LDS
// once; each lane owns (beam, sample) pairs and walks the antennas.  The phasor count is C T A M (16.7M at the study's
// default shape) -- a small kernel; it exists for parity with the study, the product beamformer is bf_beamform_fused.
#include <algorithm>
#include <cmath>

#include "bf_common.hpp"

namespace bf {

namespace {

constexpr int kStudyThreads = 256;
constexpr int kStudyMaxAnts = 2048;  // 64 KiB of LDS: A x 16 complex int8 samples

__global__ __launch_bounds__(kStudyThreads) void study_beamform_single_channel_kernel(
    const float4* __restrict__ dv, const int8_t* __restrict__ x, float2* __restrict__ out, int C, int T, int A, int M,
    float ts, int fft_size) {
#pragma clang fp contract(off)  // separate float32 roundings, as the study's expressions and the golden's sums
  extern __shared__ __attribute__((aligned(16))) int8_t xs[];  // [A][16][2]
  const int c = blockIdx.x, tex = blockIdx.y;
  const int nchunk = T / 16;
  const size_t chunk_bytes = static_cast<size_t>(A) * 32;
  const int8_t* src = x + (static_cast<size_t>(c) * nchunk + tex) * chunk_bytes;
  for (size_t i = threadIdx.x * 4; i < chunk_bytes; i += kStudyThreads * 4)
    *reinterpret_cast<uint32_t*>(xs + i) = *reinterpret_cast<const uint32_t*>(src + i);
  __syncthreads();
  const int tin = threadIdx.x & 15;
  const int t = tex * 16 + tin;
  const float pi = 3.14159265358979323846f;
  const float delta_time = t * ts * fft_size;
  const float tsc = ts * C;
  const float half = static_cast<float>(C) / 2.0f;  // NR_CHANNELS / 2.0f (:301)
  for (int m = threadIdx.x >> 4; m < M; m += kStudyThreads / 16) {
    const float4* d = dv + static_cast<size_t>(m) * A;
    float re = 0.0f, im = 0.0f;
    for (int a = 0; a < A; ++a) {
      const float4 v = d[a];
      const float delta_delay = v.y * delta_time;
      const float delta_phase = v.w * delta_time;
      const float delay_n2 = (v.x + delta_delay) * half * pi / tsc;
      const float delay_n = (v.y + delta_delay) * c * pi / tsc;
      const float phase0 = v.z - delay_n2 + delta_phase;
      const float rotation = delay_n + phase0;
      float sn, cs;
      sincosf(rotation, &sn, &cs);
      const int8_t* s = xs + (a * 16 + tin) * 2;
      re = re + cs * static_cast<float>(s[0]);
      im = im + sn * static_cast<float>(s[1]);
    }
    out[((static_cast<size_t>(c) * nchunk + tex) * M + m) * 16 + tin] = make_float2(re, im);
  }
}

}  // namespace

}  // namespace bf

extern "C" int bf_beamform_study_single_channel(const float* delay_vals, const int8_t* x, float* out, int C, int T,
                                                int A, int M, float sample_period, int fft_size, void* stream) {
  BF_REQUIRE(delay_vals && x && out, "bf_beamform_study_single_channel: null pointer");
  BF_REQUIRE(C > 0 && T > 0 && T % 16 == 0 && A > 0 && M > 0 && fft_size > 0,
             "bf_beamform_study_single_channel: bad shape C=%d T=%d (a multiple of 16) A=%d M=%d", C, T, A, M);
  BF_REQUIRE(A <= bf::kStudyMaxAnts, "bf_beamform_study_single_channel: A=%d above %d", A, bf::kStudyMaxAnts);
  BF_REQUIRE(C < 65536 && T / 16 < 65536, "bf_beamform_study_single_channel: shape too large");
  BF_REQUIRE(sample_period > 0.0f, "bf_beamform_study_single_channel: sample_period must be > 0");
  BF_REQUIRE((reinterpret_cast<uintptr_t>(delay_vals) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 3) == 0 &&
                 (reinterpret_cast<uintptr_t>(out) & 7) == 0,
             "bf_beamform_study_single_channel: misaligned buffer");
  const size_t lds = static_cast<size_t>(A) * 32;
  hipLaunchKernelGGL(bf::study_beamform_single_channel_kernel, dim3(static_cast<unsigned>(C), static_cast<unsigned>(T / 16)),
                     dim3(bf::kStudyThreads), lds, bf::as_stream(stream), reinterpret_cast<const float4*>(delay_vals),
                     x, reinterpret_cast<float2*>(out), C, T, A, M, sample_period, fft_size);
  BF_LAUNCHED("study_beamform_single_channel_kernel");
}
