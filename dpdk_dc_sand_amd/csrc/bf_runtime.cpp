// Runtime helpers of the C ABI: device memory, pinned host memory, streams and events over HIP.
// These stand in for katsdpsigproc.accel's context/queue/DeviceArray (beamform_op_sequence_test.py:105-163)
// and the CUDA-runtime calls of the C++ harness (common/UnitTest.cpp:28-111).
#include <algorithm>
#include <atomic>
#include <cstring>

#include "bf_common.hpp"

namespace bf {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

void clear_error() { g_last_error.clear(); }

// An empty kernel whose dispatches delimit a region in a profiler's kernel trace (bench.py: the timed steps).
__global__ void bf_trace_mark_kernel(int tag) { (void)tag; }

// splitmix64 of (seed, 16-byte chunk index): two words per lane, one 16-byte store.
__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void bf_fill_random_kernel(uint8_t* dst, size_t bytes, unsigned long long seed) {
  const size_t n16 = bytes / 16;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += static_cast<size_t>(gridDim.x) * 256) {
    const unsigned long long a = splitmix64(seed ^ (2 * i)), b = splitmix64(seed ^ (2 * i + 1));
    *reinterpret_cast<ulonglong2*>(dst + 16 * i) = ulonglong2{a, b};
  }
  const size_t tail = bytes - 16 * n16;  // the last < 16 bytes: one thread
  if (blockIdx.x == 0 && threadIdx.x == 0 && tail) {
    const unsigned long long a = splitmix64(seed ^ (2 * n16)), b = splitmix64(seed ^ (2 * n16 + 1));
    for (size_t k = 0; k < tail; ++k) dst[16 * n16 + k] = static_cast<uint8_t>((k < 8 ? a >> (8 * k) : b >> (8 * (k - 8))));
  }
}

// Position-weighted checksum of a 2-D region of 4-byte words (rows x run_words, row pitch pitch_words): the sum
// over packed word index i of splitmix64(splitmix64(i) ^ w_i), mod 2^64.  The same value for a contiguous slice and
// for the strided band region it was packed from (bf_channel_scatter verification).
__global__ __launch_bounds__(256) void bf_checksum_kernel(const uint32_t* p, size_t run_words, size_t pitch_words,
                                                          size_t rows, unsigned long long* out) {
  unsigned long long h = 0;
  for (size_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const uint32_t* row = p + r * pitch_words;
    for (size_t j = blockIdx.x * 256ull + threadIdx.x; j < run_words; j += static_cast<size_t>(gridDim.x) * 256) {
      const unsigned long long i = r * run_words + j;
      h += splitmix64(splitmix64(i) ^ row[j]);
    }
  }
  for (int o = 32; o >= 1; o >>= 1) h += __shfl_xor(h, o);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, h);
}

int cu_count() {
  static std::atomic<int> cache[64];  // per device index; 0 = not looked up yet
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < 64 && (n = cache[dev].load(std::memory_order_relaxed)) > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  if (dev >= 0 && dev < 64) cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

#ifdef BF_DIAG  // the generator/contraction overlap measurement (bf_wide_i8.hip)
AuxStream* aux_stream() {
  static thread_local AuxStream per_device[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    set_error("aux stream: no current device");
    return nullptr;
  }
  AuxStream& a = per_device[dev];
  if (!a.stream) {
    hipError_t e = hipStreamCreateWithFlags(&a.stream, hipStreamNonBlocking);
    for (auto& ev : a.ev)
      if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      set_error("aux stream: %s", hipGetErrorString(e));
      return nullptr;
    }
  }
  return &a;
}
#endif

}  // namespace bf

extern "C" {

const char* bf_last_error(void) { return bf::g_last_error.c_str(); }

// 3.0: 0x0500 (BF_FUSED_PATH_WIDE16), accepted by 2.0, is rejected; bf_coeff_gen_time_study, bf_comm_stats,
// bf_comm_load and bf_checksum added; the root's own scatter slice is a 2-D copy at N > 1 (include/bf.h).
int bf_abi_version(void) { return 302; }

int bf_device_count(int* count) {
  BF_REQUIRE(count != nullptr, "bf_device_count: null pointer");
  *count = 0;
  hipError_t e = hipGetDeviceCount(count);
  if (e == hipErrorNoDevice) {
    *count = 0;
    return bf::hip_fail(e, "hipGetDeviceCount");
  }
  BF_HIP(e);
  return BF_OK;
}

int bf_set_device(int device) {
  BF_HIP(hipSetDevice(device));
  return BF_OK;
}

int bf_get_device(int* device) {
  BF_REQUIRE(device != nullptr, "bf_get_device: null pointer");
  BF_HIP(hipGetDevice(device));
  return BF_OK;
}

int bf_device_name(int device, char* buf, size_t len) {
  BF_REQUIRE(buf != nullptr && len > 0, "bf_device_name: empty buffer");
  hipDeviceProp_t prop;
  BF_HIP(hipGetDeviceProperties(&prop, device));
  const char* name = prop.name[0] ? prop.name : "AMD Instinct GPU";  // the marketing name can be empty
  snprintf(buf, len, "%s (%s, %d CUs)", name, prop.gcnArchName, prop.multiProcessorCount);
  return BF_OK;
}

int bf_malloc(void** ptr, size_t bytes) {
  BF_REQUIRE(ptr != nullptr, "bf_malloc: null pointer");
  *ptr = nullptr;
  if (bytes == 0) return BF_OK;
  BF_HIP(hipMalloc(ptr, bytes));
  return BF_OK;
}

int bf_free(void* ptr) {
  if (ptr) BF_HIP(hipFree(ptr));
  return BF_OK;
}

int bf_host_alloc(void** ptr, size_t bytes) {
  BF_REQUIRE(ptr != nullptr, "bf_host_alloc: null pointer");
  *ptr = nullptr;
  if (bytes == 0) return BF_OK;
  BF_HIP(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
  return BF_OK;
}

int bf_host_free(void* ptr) {
  if (ptr) BF_HIP(hipHostFree(ptr));
  return BF_OK;
}

int bf_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return BF_OK;
  BF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, bf::as_stream(stream)));
  return BF_OK;
}

int bf_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return BF_OK;
  BF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, bf::as_stream(stream)));
  return BF_OK;
}

int bf_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
  if (bytes == 0) return BF_OK;
  BF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, bf::as_stream(stream)));
  return BF_OK;
}

int bf_memset(void* dst, int value, size_t bytes, void* stream) {
  if (bytes == 0) return BF_OK;
  BF_HIP(hipMemsetAsync(dst, value, bytes, bf::as_stream(stream)));
  return BF_OK;
}

int bf_stream_create(void** stream) {
  BF_REQUIRE(stream != nullptr, "bf_stream_create: null pointer");
  hipStream_t s;
  BF_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return BF_OK;
}

int bf_stream_destroy(void* stream) {
  if (stream) BF_HIP(hipStreamDestroy(bf::as_stream(stream)));
  return BF_OK;
}

int bf_stream_synchronize(void* stream) {
  BF_HIP(hipStreamSynchronize(bf::as_stream(stream)));
  return BF_OK;
}

int bf_stream_wait_event(void* stream, void* event) {
  BF_HIP(hipStreamWaitEvent(bf::as_stream(stream), reinterpret_cast<hipEvent_t>(event), 0));
  return BF_OK;
}

int bf_device_synchronize(void) {
  BF_HIP(hipDeviceSynchronize());
  return BF_OK;
}

int bf_event_create(void** event) {
  BF_REQUIRE(event != nullptr, "bf_event_create: null pointer");
  hipEvent_t e;
  BF_HIP(hipEventCreate(&e));
  *event = e;
  return BF_OK;
}

int bf_event_destroy(void* event) {
  if (event) BF_HIP(hipEventDestroy(reinterpret_cast<hipEvent_t>(event)));
  return BF_OK;
}

int bf_event_record(void* event, void* stream) {
  BF_HIP(hipEventRecord(reinterpret_cast<hipEvent_t>(event), bf::as_stream(stream)));
  return BF_OK;
}

int bf_event_synchronize(void* event) {
  BF_HIP(hipEventSynchronize(reinterpret_cast<hipEvent_t>(event)));
  return BF_OK;
}

int bf_fill_random(void* dst, size_t bytes, unsigned long long seed, void* stream) {
  if (bytes == 0) return BF_OK;
  BF_REQUIRE(dst != nullptr && (reinterpret_cast<uintptr_t>(dst) & 15) == 0, "bf_fill_random: null or misaligned");
  const size_t chunks = (bytes + 15) / 16;
  const unsigned grid = static_cast<unsigned>(std::min<size_t>((chunks + 255) / 256, 8192));
  hipLaunchKernelGGL(bf::bf_fill_random_kernel, dim3(grid), dim3(256), 0, bf::as_stream(stream),
                     static_cast<uint8_t*>(dst), bytes, seed);
  BF_LAUNCHED("bf_fill_random_kernel");
}

int bf_checksum(const void* src, size_t run_bytes, size_t pitch_bytes, size_t rows, unsigned long long* out,
                void* stream) {
  BF_REQUIRE(out != nullptr, "bf_checksum: null output");
  *out = 0;
  if (rows == 0 || run_bytes == 0) return BF_OK;
  BF_REQUIRE(src != nullptr && (reinterpret_cast<uintptr_t>(src) & 3) == 0 && run_bytes % 4 == 0 &&
                 pitch_bytes % 4 == 0 && (rows == 1 || pitch_bytes >= run_bytes),
             "bf_checksum: need 4-byte aligned words (run %zu, pitch %zu)", run_bytes, pitch_bytes);
  hipStream_t st = bf::as_stream(stream);
  unsigned long long* d = nullptr;
  BF_HIP(hipMalloc(reinterpret_cast<void**>(&d), sizeof(*d)));
  hipError_t e = hipMemsetAsync(d, 0, sizeof(*d), st);
  if (e == hipSuccess) {
    const size_t words = run_bytes / 4;
    const unsigned gx = static_cast<unsigned>(std::min<size_t>((words + 255) / 256, 1024));
    const unsigned gy = static_cast<unsigned>(std::min<size_t>(rows, std::max<size_t>(1, 8192 / gx)));
    hipLaunchKernelGGL(bf::bf_checksum_kernel, dim3(gx, gy), dim3(256), 0, st, static_cast<const uint32_t*>(src),
                       words, pitch_bytes / 4, rows, d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(*d), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d);
  BF_HIP(e);
  return BF_OK;
}

int bf_trace_mark(int tag, void* stream) {
  hipLaunchKernelGGL(bf::bf_trace_mark_kernel, dim3(1), dim3(64), 0, bf::as_stream(stream), tag);
  BF_LAUNCHED("bf_trace_mark_kernel");
}

int bf_event_elapsed_ms(float* ms, void* start, void* stop) {
  BF_REQUIRE(ms != nullptr, "bf_event_elapsed_ms: null pointer");
  BF_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
  return BF_OK;
}

}  // extern "C"
