// Runtime helpers of the C ABI: device memory, pinned host memory, streams and events over HIP.
// These stand in for katsdpsigproc.accel's context/queue/DeviceArray (beamform_op_sequence_test.py:105-163)
// and the CUDA-runtime calls of the C++ harness (common/UnitTest.cpp:28-111).
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

}  // namespace bf

extern "C" {

const char* bf_last_error(void) { return bf::g_last_error.c_str(); }

int bf_abi_version(void) { return 100; }

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

int bf_event_elapsed_ms(float* ms, void* start, void* stop) {
  BF_REQUIRE(ms != nullptr, "bf_event_elapsed_ms: null pointer");
  BF_HIP(hipEventElapsedTime(ms, reinterpret_cast<hipEvent_t>(start), reinterpret_cast<hipEvent_t>(stop)));
  return BF_OK;
}

}  // extern "C"
