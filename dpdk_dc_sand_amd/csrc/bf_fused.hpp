// Shared declarations of the fused beamform kernels (bf_fused.hip: item / pipe / generic / int8 kernels;
// bf_wide.hip: the wide kernel for many antennas x beams).
#pragma once

#include "bf_mfma.hpp"
#include "bf_phase.hpp"

namespace bf {

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct FusedArgs {
  const uint8_t* raw;
  const float4* dv;
  const float* gain;  // optional (M, A) real per-input beam weights (?beam-weights), folded into the phasors
  void* y;
  int delay_channels, B, C, T, A, M, S, NT, nslabs, xcd_order;
  long long base_ch;
  double ctot, ts, k, t0, batch_dt;
  float out_scale;
};

// Per-(a, m) real beam weight applied to the float32 phasor (one rounding per component, as the oracle).
__device__ __forceinline__ void apply_gain(float g, float* re, float* im) {
  *re = __fmul_rn(*re, g);
  *im = __fmul_rn(*im, g);
}

// BF_FUSED_KERNEL = item (default) | pipe | generic | wide; BF_FUSED_GENERIC=1 is shorthand for generic.
int fused_kernel_choice();

// Wide kernel (bf_wide.hip): returns BF_ERR_ARG without launching when the shape does not fit it.
bool wide_fits(const FusedArgs& P);
template <bool Signed, bool Exact>
int launch_wide(FusedArgs P, hipStream_t st);

}  // namespace bf
