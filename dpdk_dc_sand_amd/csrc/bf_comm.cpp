// Multi-GPU channel scatter over RCCL: the only collective of the channel-sharded beamformer.
//
// The reference has no multi-GPU path: each X-engine (xeng_id) owns a contiguous block of channels whose absolute
// index is c + C * xeng_id (beamformer/beamforming/coeff_generator.py:49-53), and its one multi-device pattern is a
// host thread per device (utilities/pcie_bandwidth_tests/main.cpp:193-224, cudaPcieRateTest.cpp:9).  Here one
// process drives one GPU (rank r = X-engine r) and the root hands every rank its channel slice of a full-band
// voltage cube once, device to device over xGMI:
//   root: every peer's slice (B * A strided runs of C*T*4 bytes in the (B, A, C*N, T, 2, 2) band) is packed into a
//         contiguous staging block by 2-D copies, then RCCL groups of one ncclSend per peer -- each peer's bytes on
//         their own xGMI link at once; the root's own slice is a 2-D copy straight into `slice`.  At one rank the
//         root's slice instead goes pack -> self ncclSend/ncclRecv, so the one-GPU box exercises the same RCCL
//         point-to-point path the N-rank node runs;
//   peers: ncclRecv of the slice into the (B, A, C, T, 2, 2) input buffer of the fused beamformer.
// The slice moves in pieces of at most 256 MiB (whole rows, or segments of a row longer than that), one RCCL group
// per piece.
// Everything is ordered on the caller's stream; nothing on the beamforming hot path touches RCCL.  Every rank
// records `done` after its part of each scatter; bf_comm_destroy waits for it before tearing the communicator down.
// bf_checksum (position-weighted 64-bit sum of a 2-D byte region) lets the ranks verify what they received against
// the root's band without moving it to the host.
//
// RCCL is loaded at first use (dlopen of /opt/rocm's librccl.so.1, the ROCm release libbf is built against), so a
// single-GPU user of libbf never maps it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "bf_common.hpp"

namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  std::string load_error;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      r.handle = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.handle) break;
    }
    if (!r.handle) {
      const char* e = dlerror();
      r.load_error = e ? e : "dlopen(librccl.so.1) failed";
      return;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(r.handle, name));
      if (!fn && r.load_error.empty()) r.load_error = std::string("librccl lacks ") + name;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.all_reduce, "ncclAllReduce");
    sym(r.error_string, "ncclGetErrorString");
  });
  return r;
}

int rccl_fail(ncclResult_t e, const char* what) {
  const Rccl& r = rccl();
  bf::set_error("%s: %s (%d)", what, r.error_string ? r.error_string(e) : "RCCL error", static_cast<int>(e));
  return BF_ERR_COMM;
}

#define BF_RCCL(call)                                              \
  do {                                                             \
    ncclResult_t bf_r_ = (call);                                   \
    if (bf_r_ != ncclSuccess) return rccl_fail(bf_r_, #call);      \
  } while (0)

#define BF_RCCL_LOADED()                                                                        \
  do {                                                                                          \
    if (!rccl().load_error.empty()) {                                                           \
      ::bf::set_error("RCCL unavailable: %s", rccl().load_error.c_str());                       \
      return BF_ERR_COMM;                                                                       \
    }                                                                                           \
  } while (0)

}  // namespace

// Bytes per RCCL group of a scatter.  A piece is a block of whole (b, a) rows, or a segment of one row when a row is
// longer than this: no group moves more.  Why: RCCL 2.27.7's point-to-point drops bytes of large messages -- a
// single self ncclSend/ncclRecv of more than 1 GiB leaves every byte past 2^30 unwritten, while the 2-D pack of the
// same slice (hipMemcpy2DAsync) is intact; attributed stage by stage on the device (tools/diag_scatter.py
// --attribute, profiles/r5_a_scatter_attribution.txt: 1 GiB ok; 2047 and 2048 MiB wrong from byte 2^30 on, pack ok).
// With 256 MiB pieces every size verifies (tests/test_gpu_multi_rank.py: 2 GiB slices, rows over 256 MiB).
constexpr size_t kScatterChunk = size_t(256) << 20;
#ifdef BF_DIAG
size_t g_scatter_chunk = kScatterChunk;  // measurement knob (bf_diag_scatter_chunk): attribute the truncation
inline size_t scatter_chunk() { return g_scatter_chunk; }
#else
constexpr size_t scatter_chunk() { return kScatterChunk; }
#endif

namespace {
// One piece of a slice: `nrows` rows from `row0`, bytes [off, off + width) of each.  Either width == run (whole rows,
// contiguous in the packed slice) or nrows == 1 (a row segment): a piece is always one contiguous run of nrows * width
// bytes of the packed slice, at row0 * run + off.
struct Piece {
  size_t row0, nrows, off, width;
};

// Calls f(piece) for every piece of a slice of `rows` runs of `run` bytes, in the same order on every rank (the
// root's sends and each peer's receives pair up group by group); stops at the first non-zero status.
template <class F>
int for_each_piece(size_t rows, size_t run, size_t chunk, F&& f) {
  if (run <= chunk) {
    const size_t per = chunk / run;
    for (size_t r0 = 0; r0 < rows; r0 += per)
      if (const int st = f(Piece{r0, std::min(per, rows - r0), 0, run})) return st;
  } else {
    for (size_t r = 0; r < rows; ++r)
      for (size_t off = 0; off < run; off += chunk)
        if (const int st = f(Piece{r, 1, off, std::min(chunk, run - off)})) return st;
  }
  return BF_OK;
}

bf_scatter_op make_op(int kind, int peer, int group, int src_space, size_t src_off, size_t src_pitch, int dst_space,
                      size_t dst_off, size_t dst_pitch, size_t width, size_t height) {
  bf_scatter_op o{};
  o.kind = kind;
  o.peer = peer;
  o.group = group;
  o.src_space = src_space;
  o.dst_space = dst_space;
  o.src_off = src_off;
  o.src_pitch = src_pitch;
  o.dst_off = dst_off;
  o.dst_pitch = dst_pitch;
  o.width = width;
  o.height = height;
  return o;
}

// The operation list of one rank's part of a scatter (bf_scatter_plan): the root 2-D packs every peer's slice of
// each piece into its staging slot -- peer r at slot r < root ? r : r - 1, N - 1 slots -- and its own rows straight
// into `slice`, then one RCCL group sends each peer its piece; at one rank the root's own piece is packed and moved by
// a self send/receive instead.  A peer receives each piece from the root in the same group order, so the k-th send
// root -> r pairs with r's k-th receive.
std::vector<bf_scatter_op> scatter_plan(int nranks, int rank, int root, size_t rows, size_t run, size_t chunk,
                                        size_t* staging_bytes) {
  std::vector<bf_scatter_op> ops;
  const size_t pitch = run * static_cast<size_t>(nranks);  // the band's (b, a) row
  const size_t slice_bytes = run * rows;
  const bool self_p2p = nranks == 1;
  const int npeers = self_p2p ? 1 : nranks - 1;
  *staging_bytes = rank == root ? slice_bytes * static_cast<size_t>(npeers) : 0;
  auto slot = [&](int r) { return slice_bytes * static_cast<size_t>(self_p2p ? 0 : (r < root ? r : r - 1)); };
  int group = 0;
  (void)for_each_piece(rows, run, chunk, [&](const Piece& pc) -> int {
    const size_t off = pc.row0 * run + pc.off, bytes = pc.nrows * pc.width;
    if (rank == root) {
      for (int r = 0; r < nranks; ++r) {
        const bool direct = r == root && !self_p2p;
        ops.push_back(make_op(BF_SCATTER_COPY2D, r, group, BF_SPACE_BAND,
                              pc.row0 * pitch + pc.off + run * static_cast<size_t>(r), pitch,
                              direct ? BF_SPACE_SLICE : BF_SPACE_STAGING, direct ? off : slot(r) + off, run, pc.width,
                              pc.nrows));
      }
      for (int r = 0; r < nranks; ++r) {
        if (r == root && !self_p2p) continue;
        ops.push_back(make_op(BF_SCATTER_SEND, r, group, BF_SPACE_STAGING, slot(r) + off, 0, 0, 0, 0, bytes, 1));
        if (r == root)
          ops.push_back(make_op(BF_SCATTER_RECV, root, group, 0, 0, 0, BF_SPACE_SLICE, off, 0, bytes, 1));
      }
    } else {
      ops.push_back(make_op(BF_SCATTER_RECV, root, group, 0, 0, 0, BF_SPACE_SLICE, off, 0, bytes, 1));
    }
    ++group;
    return BF_OK;
  });
  return ops;
}
}  // namespace

struct bf_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  void* staging = nullptr;  // root: the packed peer slices (N - 1 of them; at one rank the root's own, for the self path)
  size_t staging_bytes = 0;
  double* d_scalar = nullptr;  // allreduce scratch
  hipStream_t stream = nullptr;
  hipEvent_t sent = nullptr;   // root: recorded after the last scatter's sends (the staging buffer's last reader)
  hipEvent_t done = nullptr;   // every rank: recorded after its part of the last scatter (teardown waits for it)
  bool pending = false;        // a scatter was enqueued since the last wait on `done`
  unsigned long long p2p_sent = 0, p2p_received = 0;  // bytes handed to ncclSend / ncclRecv
};

namespace {
// The communicator's device for the duration of a call (the caller's device restored on return).
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
}  // namespace

extern "C" {

int bf_comm_unique_id(void* id, size_t len) {
  BF_REQUIRE(id != nullptr && len >= BF_COMM_ID_BYTES, "bf_comm_unique_id: need a %d-byte buffer",
             BF_COMM_ID_BYTES);
  static_assert(sizeof(ncclUniqueId) == BF_COMM_ID_BYTES, "ncclUniqueId size");
  BF_RCCL_LOADED();
  ncclUniqueId u;
  BF_RCCL(rccl().get_unique_id(&u));
  std::memcpy(id, &u, sizeof(u));
  bf::clear_error();
  return BF_OK;
}

int bf_comm_create(bf_comm** out, const void* id, size_t len, int nranks, int rank) {
  BF_REQUIRE(out != nullptr && id != nullptr, "bf_comm_create: null pointer");
  *out = nullptr;
  BF_REQUIRE(len == BF_COMM_ID_BYTES, "bf_comm_create: the unique id has %d bytes", BF_COMM_ID_BYTES);
  BF_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bf_comm_create: rank %d of %d", rank, nranks);
  BF_RCCL_LOADED();
  auto* c = new bf_comm();
  c->nranks = nranks;
  c->rank = rank;
  hipError_t e = hipGetDevice(&c->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->d_scalar), sizeof(double));
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->sent, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    if (c->d_scalar) (void)hipFree(c->d_scalar);
    if (c->sent) (void)hipEventDestroy(c->sent);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return bf::hip_fail(e, "bf_comm_create");
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  const ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    (void)hipFree(c->d_scalar);
    (void)hipEventDestroy(c->sent);
    (void)hipEventDestroy(c->done);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return rccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  bf::clear_error();
  return BF_OK;
}

int bf_comm_destroy(bf_comm* c) {
  if (!c) return BF_OK;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->device);
  // every scatter this rank enqueued (sends, receives, the staging reads) has finished before RCCL is torn down
  if (c->pending) (void)hipEventSynchronize(c->done);
  if (c->staging) (void)hipEventSynchronize(c->sent);
  (void)hipStreamSynchronize(c->stream);
  const ncclResult_t r = c->comm ? rccl().comm_destroy(c->comm) : ncclSuccess;
  if (c->staging) (void)hipFree(c->staging);
  (void)hipFree(c->d_scalar);
  (void)hipEventDestroy(c->sent);
  (void)hipEventDestroy(c->done);
  (void)hipStreamDestroy(c->stream);
  delete c;
  if (prev >= 0) (void)hipSetDevice(prev);
  if (r != ncclSuccess) return rccl_fail(r, "ncclCommDestroy");
  return BF_OK;
}

int bf_comm_allreduce_max(bf_comm* c, double* value) {
  BF_REQUIRE(c != nullptr && value != nullptr, "bf_comm_allreduce_max: null pointer");
  DeviceGuard dg(c->device);
  BF_HIP(hipMemcpyAsync(c->d_scalar, value, sizeof(double), hipMemcpyHostToDevice, c->stream));
  BF_RCCL(rccl().all_reduce(c->d_scalar, c->d_scalar, 1, ncclFloat64, ncclMax, c->comm, c->stream));
  BF_HIP(hipMemcpyAsync(value, c->d_scalar, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  BF_HIP(hipStreamSynchronize(c->stream));
  return BF_OK;
}

int bf_scatter_plan(int nranks, int rank, int root, int B, int A, int C, int T, size_t chunk, bf_scatter_op* ops,
                    size_t capacity, size_t* n_ops, size_t* staging_bytes) {
  BF_REQUIRE(n_ops != nullptr && staging_bytes != nullptr, "bf_scatter_plan: null pointer");
  BF_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks && root >= 0 && root < nranks,
             "bf_scatter_plan: rank %d, root %d of %d ranks", rank, root, nranks);
  BF_REQUIRE(B > 0 && A > 0 && C > 0 && T > 0, "bf_scatter_plan: bad shape B=%d A=%d C=%d T=%d", B, A, C, T);
  const size_t run = static_cast<size_t>(C) * T * 4;
  const auto plan = scatter_plan(nranks, rank, root, static_cast<size_t>(B) * A, run, chunk ? chunk : scatter_chunk(),
                                 staging_bytes);
  *n_ops = plan.size();
  if (ops == nullptr) return BF_OK;
  BF_REQUIRE(capacity >= plan.size(), "bf_scatter_plan: %zu ops need a capacity of at least that", plan.size());
  std::copy(plan.begin(), plan.end(), ops);
  bf::clear_error();
  return BF_OK;
}

int bf_channel_scatter(bf_comm* c, const uint8_t* band, uint8_t* slice, int B, int A, int C, int T, int root,
                       void* stream) {
  BF_REQUIRE(c != nullptr && slice != nullptr, "bf_channel_scatter: null pointer");
  BF_REQUIRE(B > 0 && A > 0 && C > 0 && T > 0, "bf_channel_scatter: bad shape B=%d A=%d C=%d T=%d", B, A, C, T);
  BF_REQUIRE(root >= 0 && root < c->nranks, "bf_channel_scatter: root %d of %d ranks", root, c->nranks);
  BF_REQUIRE(c->rank != root || band != nullptr, "bf_channel_scatter: the root needs the band");
  DeviceGuard dg(c->device);
  hipStream_t st = bf::as_stream(stream);
  size_t need = 0;
  const auto plan = scatter_plan(c->nranks, c->rank, root, static_cast<size_t>(B) * A, static_cast<size_t>(C) * T * 4,
                                 scatter_chunk(), &need);
  if (need > c->staging_bytes) {
    if (c->staging) {
      BF_HIP(hipEventSynchronize(c->sent));
      BF_HIP(hipFree(c->staging));
      c->staging = nullptr;
      c->staging_bytes = 0;
    }
    BF_HIP(hipMalloc(&c->staging, need));
    c->staging_bytes = need;
  }
  // the previous scatter's sends may still read the staging buffer on another stream
  if (c->rank == root) BF_HIP(hipStreamWaitEvent(st, c->sent, 0));
  auto at = [&](int space, unsigned long long off) -> uint8_t* {
    uint8_t* base = space == BF_SPACE_BAND      ? const_cast<uint8_t*>(band)
                    : space == BF_SPACE_STAGING ? static_cast<uint8_t*>(c->staging)
                                                : slice;
    return base + off;
  };
  unsigned long long sent = 0, received = 0;
  for (size_t i = 0; i < plan.size();) {
    const int group = plan[i].group;
    for (; i < plan.size() && plan[i].group == group && plan[i].kind == BF_SCATTER_COPY2D; ++i) {
      const bf_scatter_op& o = plan[i];
      BF_HIP(hipMemcpy2DAsync(at(o.dst_space, o.dst_off), o.dst_pitch, at(o.src_space, o.src_off), o.src_pitch, o.width,
                              o.height, hipMemcpyDeviceToDevice, st));
    }
    BF_RCCL(rccl().group_start());
    for (; i < plan.size() && plan[i].group == group; ++i) {
      const bf_scatter_op& o = plan[i];
      const ncclResult_t e =
          o.kind == BF_SCATTER_SEND ? rccl().send(at(o.src_space, o.src_off), o.width, ncclUint8, o.peer, c->comm, st)
          : o.kind == BF_SCATTER_RECV ? rccl().recv(at(o.dst_space, o.dst_off), o.width, ncclUint8, o.peer, c->comm, st)
                                      : ncclInvalidUsage;  // a copy after the group's sends: not a plan this file makes
      if (e != ncclSuccess) {
        (void)rccl().group_end();
        return rccl_fail(e, o.kind == BF_SCATTER_SEND ? "ncclSend" : "ncclRecv");
      }
      (o.kind == BF_SCATTER_SEND ? sent : received) += o.width;
    }
    BF_RCCL(rccl().group_end());
  }
  if (c->rank == root) BF_HIP(hipEventRecord(c->sent, st));
  c->p2p_sent += sent;
  c->p2p_received += received;
  BF_HIP(hipEventRecord(c->done, st));
  c->pending = true;
  bf::clear_error();
  return BF_OK;
}

int bf_comm_stats(const bf_comm* c, unsigned long long* sent, unsigned long long* received) {
  BF_REQUIRE(c != nullptr && sent != nullptr && received != nullptr, "bf_comm_stats: null pointer");
  *sent = c->p2p_sent;
  *received = c->p2p_received;
  return BF_OK;
}

int bf_comm_load(void) {
  BF_RCCL_LOADED();
  bf::clear_error();
  return BF_OK;
}

#ifdef BF_DIAG
// ---- diagnostic build: attributing the round-4 2 GiB truncation (tools/diag_scatter.py --attribute) ----
// The scatter's piece size; 0 restores the product's.
int bf_diag_scatter_chunk(size_t bytes) {
  g_scatter_chunk = bytes ? bytes : kScatterChunk;
  return BF_OK;
}
// The pack stage alone: one hipMemcpy2DAsync of `height` rows of `width` bytes (pitches as given).
int bf_diag_memcpy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height,
                     void* stream) {
  BF_HIP(hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToDevice, bf::as_stream(stream)));
  return BF_OK;
}
// The RCCL stage alone: one group of a self ncclSend(src) + ncclRecv(dst) of `bytes` on a one-rank communicator.
int bf_diag_p2p_self(bf_comm* c, const void* src, void* dst, size_t bytes, void* stream) {
  BF_REQUIRE(c != nullptr && c->nranks == 1, "bf_diag_p2p_self: needs a one-rank communicator");
  DeviceGuard dg(c->device);
  hipStream_t st = bf::as_stream(stream);
  BF_RCCL(rccl().group_start());
  ncclResult_t e = rccl().send(src, bytes, ncclUint8, 0, c->comm, st);
  if (e == ncclSuccess) e = rccl().recv(dst, bytes, ncclUint8, 0, c->comm, st);
  if (e != ncclSuccess) {
    (void)rccl().group_end();
    return rccl_fail(e, "bf_diag_p2p_self");
  }
  BF_RCCL(rccl().group_end());
  return BF_OK;
}
#endif  // BF_DIAG

}  // extern "C"
