// Streaming ingest pipeline: pinned host frames -> H2D copy stream -> fused
// beamform (+ int8 requantisation) on the compute stream -> D2H copy stream -> pinned host beams.
//
// The reference's equivalents are the event-chained PCIe test (utilities/pcie_bandwidth_tests/cudaPcieRateTest.cpp:
// 63-123) and the HtoD / kernel / DtoH phases of its unit-test harness (common/UnitTest.cpp:28-57), which run the
// phases back to back.  Here the three phases of successive frames overlap on three HIP streams (two DMA engines
// and the CUs) over a ring of `depth` device slots:
//   frame n uses slot n % depth;
//   H2D(n)     waits for compute(n - depth) (the slot's input buffer is free again);
//   compute(n) waits for H2D(n) and for D2H(n - depth) (the slot's output buffer has been drained);
//   D2H(n)     waits for compute(n).
// Delay-model and beam-weight updates are staged through a ring of pinned buffers and uploaded on the compute
// stream, so a frame submitted before an update uses the old model and every later frame the new one (stream
// order), with no host synchronisation on the data path (an update waits only when kStage earlier updates are
// still queued behind in-flight frames).
#include <cmath>
#include <cstring>
#include <vector>

#include "bf_common.hpp"

constexpr int kStage = 4;  // control-update staging buffers per table

struct bf_pipeline {
  int B, C, T, A, M, Ctot, xeng_id, flags, delay_channels, depth, device;
  double ts;
  float out_scale;
  size_t in_bytes, out_bytes, delay_bytes, gain_bytes;
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<void*> d_in, d_out;
  // per slot: [0] h2d start, [1] h2d end, [2] compute start, [3] compute end, [4] d2h start, [5] d2h end
  std::vector<hipEvent_t> ev;
  float* d_delays = nullptr;
  float* d_gains = nullptr;
  void* d_workspace = nullptr;  // the fused call's workspace (int8 wide path's Q14 table), used on s_comp only
  size_t workspace_bytes = 0;
  // pinned staging rings for control updates: update u uses stage u % kStage, whose previous upload must have
  // retired (its event) -- so only kStage updates in flight at once can make the caller wait
  float* h_delays[kStage] = {};
  float* h_gains[kStage] = {};
  hipEvent_t ev_delays[kStage] = {}, ev_gains[kStage] = {};
  long long n_delay_updates = 0, n_gain_updates = 0;
  bool delays_set = false, gains_set = false;
  long long next = 0;
};

namespace {

constexpr int kEvents = 6;

// Make the pipeline's device current for the duration of a call; restore the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  hipError_t err;
  explicit DeviceGuard(int dev) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

hipEvent_t& slot_event(bf_pipeline* p, long long frame, int which) {
  return p->ev[static_cast<size_t>(frame % p->depth) * kEvents + which];
}

void release(bf_pipeline* p) {
  if (p->s_h2d) (void)hipStreamSynchronize(p->s_h2d);
  if (p->s_comp) (void)hipStreamSynchronize(p->s_comp);
  if (p->s_d2h) (void)hipStreamSynchronize(p->s_d2h);
  for (void* x : p->d_in) (void)hipFree(x);
  for (void* x : p->d_out) (void)hipFree(x);
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  for (int i = 0; i < kStage; ++i) {
    if (p->ev_delays[i]) (void)hipEventDestroy(p->ev_delays[i]);
    if (p->ev_gains[i]) (void)hipEventDestroy(p->ev_gains[i]);
    if (p->h_delays[i]) (void)hipHostFree(p->h_delays[i]);
    if (p->h_gains[i]) (void)hipHostFree(p->h_gains[i]);
  }
  if (p->d_delays) (void)hipFree(p->d_delays);
  if (p->d_gains) (void)hipFree(p->d_gains);
  if (p->d_workspace) (void)hipFree(p->d_workspace);
  if (p->s_h2d) (void)hipStreamDestroy(p->s_h2d);
  if (p->s_comp) (void)hipStreamDestroy(p->s_comp);
  if (p->s_d2h) (void)hipStreamDestroy(p->s_d2h);
  delete p;
}

}  // namespace

#define BF_GUARD(p)                                   \
  DeviceGuard bf_guard_((p)->device);                 \
  if (bf_guard_.err != hipSuccess) return ::bf::hip_fail(bf_guard_.err, "hipSetDevice")

extern "C" {

int bf_pipeline_create(bf_pipeline** out, int B, int C, int T, int A, int M, int Ctot, int xeng_id,
                       double sample_period, int flags, float out_scale, int delay_channels, int depth) {
  BF_REQUIRE(out != nullptr, "bf_pipeline_create: null pointer");
  *out = nullptr;
  BF_REQUIRE(B > 0 && C > 0 && T > 0 && A > 0 && M > 0 && Ctot > 0 && xeng_id >= 0,
             "bf_pipeline_create: bad shape B=%d C=%d T=%d A=%d M=%d Ctot=%d", B, C, T, A, M, Ctot);
  BF_REQUIRE(T % bf::kSamplesPerBlock == 0, "bf_pipeline_create: n_samples_per_channel=%d must be a multiple of 16",
             T);
  BF_REQUIRE(delay_channels == 1 || delay_channels == C, "bf_pipeline_create: delay_channels must be 1 or C");
  BF_REQUIRE(depth >= 1 && depth <= 64, "bf_pipeline_create: depth=%d out of [1, 64]", depth);
  BF_REQUIRE(sample_period > 0.0, "bf_pipeline_create: sample_period must be > 0");
  const char* ferr = bf::fused_flags_error(flags);
  BF_REQUIRE(ferr == nullptr, "bf_pipeline_create: %s (flags 0x%x)", ferr, flags);
  const bool q14 = (flags & BF_FUSED_OUT_INT8) && !(flags & BF_FUSED_INT8_VIA_F32);
  BF_REQUIRE(!q14 || bf::q14_sum_bound_ok(A, flags & BF_FUSED_SIGNED, 1.0),
             "bf_pipeline_create: n_ants=%d overflows the int8 path's int32 beam sums", A);
  auto* p = new bf_pipeline();
  p->B = B, p->C = C, p->T = T, p->A = A, p->M = M, p->Ctot = Ctot, p->xeng_id = xeng_id, p->flags = flags;
  p->delay_channels = delay_channels, p->depth = depth, p->ts = sample_period, p->out_scale = out_scale;
  p->in_bytes = static_cast<size_t>(B) * A * C * T * 4;
  p->out_bytes = static_cast<size_t>(B) * 2 * C * T * 2 * M * ((flags & BF_FUSED_OUT_INT8) ? 1 : 4);
  p->delay_bytes = static_cast<size_t>(delay_channels) * M * A * 4 * sizeof(float);
  p->gain_bytes = static_cast<size_t>(M) * A * sizeof(float);
  hipError_t e = hipGetDevice(&p->device);
  auto fail = [&](hipError_t err, const char* what) {
    const int st = bf::hip_fail(err, what);
    release(p);
    return st;
  };
  if (e != hipSuccess) return fail(e, "hipGetDevice");
  if ((e = hipStreamCreateWithFlags(&p->s_h2d, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
  if ((e = hipStreamCreateWithFlags(&p->s_comp, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
  if ((e = hipStreamCreateWithFlags(&p->s_d2h, hipStreamNonBlocking)) != hipSuccess) return fail(e, "stream");
  p->d_in.assign(depth, nullptr);
  p->d_out.assign(depth, nullptr);
  p->ev.assign(static_cast<size_t>(depth) * kEvents, nullptr);
  for (int i = 0; i < depth; ++i) {
    if ((e = hipMalloc(&p->d_in[i], p->in_bytes)) != hipSuccess) return fail(e, "hipMalloc(frame in)");
    if ((e = hipMalloc(&p->d_out[i], p->out_bytes)) != hipSuccess) return fail(e, "hipMalloc(frame out)");
  }
  for (auto& ev : p->ev)
    if ((e = hipEventCreate(&ev)) != hipSuccess) return fail(e, "hipEventCreate");
  for (int i = 0; i < kStage; ++i) {
    if ((e = hipEventCreateWithFlags(&p->ev_delays[i], hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipEventCreateWithFlags(&p->ev_gains[i], hipEventDisableTiming)) != hipSuccess) return fail(e, "event");
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&p->h_delays[i]), p->delay_bytes, hipHostMallocDefault)) !=
        hipSuccess)
      return fail(e, "hipHostMalloc");
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&p->h_gains[i]), p->gain_bytes, hipHostMallocDefault)) !=
        hipSuccess)
      return fail(e, "hipHostMalloc");
  }
  if ((e = hipMalloc(reinterpret_cast<void**>(&p->d_delays), p->delay_bytes)) != hipSuccess) return fail(e, "malloc");
  if ((e = hipMalloc(reinterpret_cast<void**>(&p->d_gains), p->gain_bytes)) != hipSuccess) return fail(e, "malloc");
  if (bf_fused_workspace_bytes(B, C, T, A, M, flags, &p->workspace_bytes) == BF_OK && p->workspace_bytes > 0 &&
      (e = hipMalloc(&p->d_workspace, p->workspace_bytes)) != hipSuccess)
    return fail(e, "hipMalloc(workspace)");
  *out = p;
  bf::clear_error();
  return BF_OK;
}

int bf_pipeline_destroy(bf_pipeline* p) {
  if (!p) return BF_OK;
  DeviceGuard g(p->device);
  release(p);
  return BF_OK;
}

int bf_pipeline_frame_bytes(const bf_pipeline* p, size_t* in_bytes, size_t* out_bytes) {
  BF_REQUIRE(p != nullptr, "bf_pipeline_frame_bytes: null pipeline");
  if (in_bytes) *in_bytes = p->in_bytes;
  if (out_bytes) *out_bytes = p->out_bytes;
  return BF_OK;
}

// Stage a host table through pinned memory and upload it on the compute stream (after every frame already
// submitted, before every later one).  Update u uses staging buffer u % kStage; the caller waits only when that
// buffer's previous upload (kStage updates ago) is still queued behind in-flight frames.
static int upload(bf_pipeline* p, const float* host, float* const (&staging)[kStage], float* dev, size_t bytes,
                  hipEvent_t (&done)[kStage], long long* count) {
  const int i = static_cast<int>(*count % kStage);
  BF_HIP(hipEventSynchronize(done[i]));
  std::memcpy(staging[i], host, bytes);
  BF_HIP(hipMemcpyAsync(dev, staging[i], bytes, hipMemcpyHostToDevice, p->s_comp));
  BF_HIP(hipEventRecord(done[i], p->s_comp));
  ++*count;
  return BF_OK;
}

int bf_pipeline_set_delays(bf_pipeline* p, const float* host_delay_vals) {
  BF_REQUIRE(p != nullptr && host_delay_vals != nullptr, "bf_pipeline_set_delays: null pointer");
  BF_GUARD(p);
  const int st = upload(p, host_delay_vals, p->h_delays, p->d_delays, p->delay_bytes, p->ev_delays,
                        &p->n_delay_updates);
  if (st == BF_OK) p->delays_set = true;
  return st;
}

int bf_pipeline_set_gains(bf_pipeline* p, const float* host_gains) {
  BF_REQUIRE(p != nullptr, "bf_pipeline_set_gains: null pipeline");
  BF_GUARD(p);
  if (!host_gains) {  // back to unit weights: frames submitted from now on do not read the gain table
    p->gains_set = false;
    bf::clear_error();
    return BF_OK;
  }
  if ((p->flags & BF_FUSED_OUT_INT8) && !(p->flags & BF_FUSED_INT8_VIA_F32)) {
    // the Q14 integer path: the weights must keep the high limb int8 and the int32 sums from wrapping
    double gmax = 0.0;
    const size_t n = static_cast<size_t>(p->M) * p->A;
    for (size_t i = 0; i < n; ++i) {
      const double g = std::fabs(static_cast<double>(host_gains[i]));
      BF_REQUIRE(std::isfinite(g), "bf_pipeline_set_gains: weight %zu is not finite", i);
      gmax = g > gmax ? g : gmax;
    }
    BF_REQUIRE(bf::q14_sum_bound_ok(p->A, p->flags & BF_FUSED_SIGNED, gmax),
               "bf_pipeline_set_gains: weight magnitude %g out of range for int8 beams with %d inputs", gmax, p->A);
  }
  const int st = upload(p, host_gains, p->h_gains, p->d_gains, p->gain_bytes, p->ev_gains, &p->n_gain_updates);
  if (st == BF_OK) p->gains_set = true;
  return st;
}

int bf_pipeline_submit(bf_pipeline* p, const void* host_in, void* host_out, double t0, double batch_dt,
                       long long* ticket) {
  BF_REQUIRE(p != nullptr && host_in != nullptr && host_out != nullptr, "bf_pipeline_submit: null pointer");
  BF_REQUIRE(p->delays_set, "bf_pipeline_submit: no delay model (call bf_pipeline_set_delays first)");
  BF_GUARD(p);
  const long long n = p->next;
  const int slot = static_cast<int>(n % p->depth);
  if (n >= p->depth) {  // slot reuse: its input must have been consumed, its output drained
    BF_HIP(hipStreamWaitEvent(p->s_h2d, slot_event(p, n, 3), 0));
    BF_HIP(hipStreamWaitEvent(p->s_comp, slot_event(p, n, 5), 0));
  }
  BF_HIP(hipEventRecord(slot_event(p, n, 0), p->s_h2d));
  BF_HIP(hipMemcpyAsync(p->d_in[slot], host_in, p->in_bytes, hipMemcpyHostToDevice, p->s_h2d));
  BF_HIP(hipEventRecord(slot_event(p, n, 1), p->s_h2d));

  BF_HIP(hipStreamWaitEvent(p->s_comp, slot_event(p, n, 1), 0));
  BF_HIP(hipEventRecord(slot_event(p, n, 2), p->s_comp));
  const int st = bf_beamform_fused_ws(static_cast<const uint8_t*>(p->d_in[slot]), p->d_delays, p->delay_channels,
                                      p->gains_set ? p->d_gains : nullptr, p->d_out[slot], p->B, p->C, p->T, p->A,
                                      p->M, p->Ctot, p->xeng_id, p->ts, t0, batch_dt, p->flags, p->out_scale,
                                      p->d_workspace, p->workspace_bytes, p->s_comp);
  if (st != BF_OK) return st;
  BF_HIP(hipEventRecord(slot_event(p, n, 3), p->s_comp));

  BF_HIP(hipStreamWaitEvent(p->s_d2h, slot_event(p, n, 3), 0));
  BF_HIP(hipEventRecord(slot_event(p, n, 4), p->s_d2h));
  BF_HIP(hipMemcpyAsync(host_out, p->d_out[slot], p->out_bytes, hipMemcpyDeviceToHost, p->s_d2h));
  BF_HIP(hipEventRecord(slot_event(p, n, 5), p->s_d2h));
  p->next = n + 1;
  if (ticket) *ticket = n;
  bf::clear_error();
  return BF_OK;
}

// stage 0: the frame's input has been copied (its host buffer may be refilled); 1: its beams are in host_out.
// A slot's events are re-recorded by later frames; waiting on a later frame's event is still correct (in-order
// streams), only conservative.
int bf_pipeline_wait(bf_pipeline* p, long long ticket, int stage) {
  BF_REQUIRE(p != nullptr, "bf_pipeline_wait: null pipeline");
  BF_REQUIRE(ticket >= 0 && ticket < p->next, "bf_pipeline_wait: ticket %lld was never submitted", ticket);
  BF_REQUIRE(stage == 0 || stage == 1, "bf_pipeline_wait: stage must be 0 (input) or 1 (output)");
  BF_GUARD(p);
  BF_HIP(hipEventSynchronize(slot_event(p, ticket, stage ? 5 : 1)));
  return BF_OK;
}

int bf_pipeline_query(bf_pipeline* p, long long ticket, int stage, int* done) {
  BF_REQUIRE(p != nullptr && done != nullptr, "bf_pipeline_query: null pointer");
  BF_REQUIRE(ticket >= 0 && ticket < p->next, "bf_pipeline_query: ticket %lld was never submitted", ticket);
  BF_REQUIRE(stage == 0 || stage == 1, "bf_pipeline_query: stage must be 0 (input) or 1 (output)");
  BF_GUARD(p);
  const hipError_t e = hipEventQuery(slot_event(p, ticket, stage ? 5 : 1));
  if (e == hipErrorNotReady) {
    *done = 0;
    return BF_OK;
  }
  BF_HIP(e);
  *done = 1;
  return BF_OK;
}

int bf_pipeline_flush(bf_pipeline* p) {
  BF_REQUIRE(p != nullptr, "bf_pipeline_flush: null pipeline");
  BF_GUARD(p);
  BF_HIP(hipStreamSynchronize(p->s_h2d));
  BF_HIP(hipStreamSynchronize(p->s_comp));
  BF_HIP(hipStreamSynchronize(p->s_d2h));
  return BF_OK;
}

// Per-stage durations of the most recent use of `ticket`'s slot (valid once the ticket's output stage is done
// and while no later frame has reused the slot).
int bf_pipeline_stage_ms(bf_pipeline* p, long long ticket, float* h2d_ms, float* compute_ms, float* d2h_ms) {
  BF_REQUIRE(p != nullptr, "bf_pipeline_stage_ms: null pipeline");
  BF_REQUIRE(ticket >= 0 && ticket < p->next && ticket + p->depth >= p->next,
             "bf_pipeline_stage_ms: ticket %lld is not among the last %d frames", ticket, p->depth);
  BF_GUARD(p);
  BF_HIP(hipEventSynchronize(slot_event(p, ticket, 5)));
  float v[3];
  for (int k = 0; k < 3; ++k)
    BF_HIP(hipEventElapsedTime(&v[k], slot_event(p, ticket, 2 * k), slot_event(p, ticket, 2 * k + 1)));
  if (h2d_ms) *h2d_ms = v[0];
  if (compute_ms) *compute_ms = v[1];
  if (d2h_ms) *d2h_ms = v[2];
  return BF_OK;
}

}  // extern "C"
