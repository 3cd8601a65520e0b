// Shared helpers for libbf: thread-local error state, HIP error mapping, argument checks.
// The reference's C++ harness calls exit() from GPU_ERRCHK (common/Utils.cpp:8-16); here every failure is a
// negative status plus a message retrievable through bf_last_error().
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/bf.h"

namespace bf {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

inline int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
  return e == hipErrorNoDevice ? BF_ERR_NODEV : BF_ERR_HIP;
}

#define BF_HIP(call)                                                  \
  do {                                                                \
    hipError_t bf_e_ = (call);                                        \
    if (bf_e_ != hipSuccess) return ::bf::hip_fail(bf_e_, #call);     \
  } while (0)

#define BF_REQUIRE(cond, ...)          \
  do {                                 \
    if (!(cond)) {                     \
      ::bf::set_error(__VA_ARGS__);    \
      return BF_ERR_ARG;               \
    }                                  \
  } while (0)

// After a kernel launch: report launch-configuration errors without synchronising.
#define BF_LAUNCHED(name)                                            \
  do {                                                               \
    hipError_t bf_e_ = hipGetLastError();                            \
    if (bf_e_ != hipSuccess) return ::bf::hip_fail(bf_e_, name);     \
    ::bf::clear_error();                                             \
    return BF_OK;                                                    \
  } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Measurement knobs (load forms, slab widths, launch orders) are read from the environment only in the diagnostic
// build (`make diag`, -DBF_DIAG, used by tools/diag_*.py).  The product library never reads the environment: kernel
// paths and contract switches are explicit bf_beamform_fused flags (include/bf.h).
inline const char* diag_env(const char* name) {
#ifdef BF_DIAG
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// The kernels' compile-time `Mode` ablation bits (skip a phase, stamp, re-route a stream) exist for the diagnostic
// build only: a product instantiation carrying one fails to compile (static_assert(kDiagBuild || ...) per kernel).
#ifdef BF_DIAG
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif

constexpr int kSamplesPerBlock = 16;  // matrix_multiply.py:76 (128 // 8)

// Launch flags of bf_beamform_fused* and bf_pipeline_create (include/bf.h): only known bits, a defined kernel
// path, a defined workgroup order.  Returns nullptr when valid, else what is wrong.
inline const char* fused_flags_error(int flags) {
  if (flags & ~(BF_FUSED_SIGNED | BF_FUSED_OUT_INT8 | BF_FUSED_EXACT_COEFF | BF_FUSED_INT8_VIA_F32 |
                BF_FUSED_PATH_MASK | BF_FUSED_ORDER_MASK))
    return "unknown flags";
  const int path = flags & BF_FUSED_PATH_MASK;
  if (path != 0 && path != BF_FUSED_PATH_ITEM && path != BF_FUSED_PATH_GENERIC && path != BF_FUSED_PATH_WIDE)
    return "unknown kernel path";
  if ((flags & BF_FUSED_ORDER_MASK) == BF_FUSED_ORDER_MASK) return "unknown workgroup order";
  return nullptr;
}

// The Q14 integer path's int32 beam sums: |y| <= A * max|x| * (sqrt(2) * rne(max|g| * 2^14) + 1) must stay below
// 2^31 (max|x| = 128 for int8 samples, 255 for uint8), and the high limb of rne(g * 2^14) must stay int8
// (|g| <= 1.992).  The oracle sums in int64; beyond the bound the int32 accumulators would wrap.
inline bool q14_sum_bound_ok(int A, bool sample_signed, double max_gain) {
  if (__builtin_rint(max_gain * 16384.0) > 32639.0) return false;
  return static_cast<double>(A) * (sample_signed ? 128 : 255) * (1.4142135623730951 * 16384.0 * max_gain + 1.0) <
         2147483648.0;
}

// Compute units of the current device (cached per device index; sizes persistent grids only).
int cu_count();

#ifdef BF_DIAG
// A second stream on the current device for work a call forks off its caller's stream and joins back (the int8
// wide path's coefficient generator running beside the contraction), and a pool of events for the hand-offs.
// Thread-local per device: concurrent callers on other host threads never serialise on one another's helper.
// Returns nullptr (and sets the error) if the stream or events cannot be created.
struct AuxStream {
  hipStream_t stream = nullptr;
  hipEvent_t ev[17] = {};  // [0] fork, [1 + k] chunk k done
};
AuxStream* aux_stream();
#endif

}  // namespace bf
