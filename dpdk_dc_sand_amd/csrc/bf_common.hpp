// Shared helpers for libbf: thread-local error state, HIP error mapping, argument checks.
// The reference's C++ harness calls exit() from GPU_ERRCHK (common/Utils.cpp:8-16); here every failure is a
// negative status plus a message retrievable through bf_last_error().
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
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

constexpr int kSamplesPerBlock = 16;  // matrix_multiply.py:76 (128 // 8)

}  // namespace bf
