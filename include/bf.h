/*
 * bf.h -- C ABI of libbf.so, the MI355X-native (gfx950) beamformer hot path.
 *
 * Drop-in boundary for the reference's operator package `beamformer/beamforming` (magnate3/dpdk_dc_sand).
 * Every entry point below states the reference interface it replaces (file:line, relative to the reference
 * repository root).  Conventions:
 *   - every function returns int: 0 = OK, negative = error; bf_last_error() gives a thread-local message;
 *   - compute entry points take caller-owned DEVICE pointers plus a stream (hipStream_t passed as void*,
 *     NULL = the default stream), never allocate, are asynchronous and stream-ordered, and are reentrant
 *     across streams;
 *   - shapes are the reference's (B = batches, P = pols = 2, C = channels on this engine, Ctot = channels
 *     in the band, A = antennas, M = beams, T = samples per channel, NB = T / 16);
 *   - 8-bit voltages are complex (re, im) byte pairs; sample_signed = 0 reads them as uint8 (the reference
 *     slots' dtype, matrix_multiply.py:145-147), 1 as int8 (the C++ study's char2, BeamformerKernels.cu:196).
 */
#ifndef DPDK_DC_SAND_AMD_BF_H
#define DPDK_DC_SAND_AMD_BF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------------------------------------- */
#define BF_OK 0
#define BF_ERR_ARG (-1)     /* invalid shape / argument (reference: template ValueError, prebeamform_reorder.py:62-65) */
#define BF_ERR_HIP (-2)     /* HIP runtime error (reference: GPU_ERRCHK, common/Utils.hpp:8, common/Utils.cpp:8-16) */
#define BF_ERR_NODEV (-3)   /* no GPU visible */
#define BF_ERR_COMM (-4)    /* RCCL unavailable or a collective failed (multi-GPU channel scatter) */

/* Thread-local message of the last failing call on this thread (replaces GPU_ERRCHK's stderr print). */
const char* bf_last_error(void);
/* ABI version: major * 100 + minor.  300: ABI 3.0 -- 0x0500 (BF_FUSED_PATH_WIDE16, accepted by 2.0) is rejected as an
 * unknown path, and bf_coeff_gen_time_study, bf_comm_stats, bf_comm_load and bf_checksum were added.  301: ABI 3.1 --
 * bf_scatter_plan added (the channel scatter's operation list as a pure host function).  302: ABI 3.2 --
 * bf_beamform_study_single_channel added (the C++ study's fused kernel in its own semantics). */
int bf_abi_version(void);

/* ---- runtime helpers (device memory, streams, events) -------------------------------------------------
 * The reference gets these from katsdpsigproc.accel / PyCUDA (accel.create_some_context,
 * ctx.create_command_queue, DeviceArray.set/get: beamform_op_sequence_test.py:105-163) and, in the C++
 * harness, from the CUDA runtime (common/UnitTest.cpp:28-111).  Thin HIP wrappers so the Python shim needs
 * no other GPU runtime. */
int bf_device_count(int* count);
int bf_set_device(int device);
int bf_get_device(int* device);
int bf_device_name(int device, char* buf, size_t len);
int bf_malloc(void** ptr, size_t bytes);
int bf_free(void* ptr);
int bf_host_alloc(void** ptr, size_t bytes);   /* pinned host memory (streaming ring, cudaPcieRateTest.cpp:63-123) */
int bf_host_free(void* ptr);
int bf_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int bf_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
int bf_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);
int bf_memset(void* dst, int value, size_t bytes, void* stream);
int bf_stream_create(void** stream);
int bf_stream_destroy(void* stream);
int bf_stream_synchronize(void* stream);
int bf_stream_wait_event(void* stream, void* event);
int bf_device_synchronize(void);
int bf_event_create(void** event);
int bf_event_destroy(void* event);
int bf_event_record(void* event, void* stream);
int bf_event_synchronize(void* event);
int bf_event_elapsed_ms(float* ms, void* start, void* stop);
/* Launch one empty kernel (`bf_trace_mark_kernel`) on `stream`: its dispatches delimit a region of a profiler's
 * kernel trace (bench.py brackets its timed steps with two of them; tools/kernel_stats.py reads the region). */
int bf_trace_mark(int tag, void* stream);

/* ---- hot path ----------------------------------------------------------------------------------------- */

/* Steering coefficients, Python layout.
 * Replaces CoeffGenerator._run -> run_coeff_gen (beamformer/beamforming/coeff_generator.py:12-103, 209-250),
 * with the CPU oracle's (c, m, a) mapping (beamformer/unit_test/coeff_generator_cpu.py:120-186).
 *   delay_vals : f32 (C, M, A, 4) = (delay_s, delay_rate, phase_rad, phase_rate); only [0] and [2] are read
 *   out        : f32 (B, P, C, 2A, 2M), block [[cos, sin], [-sin, cos]] per (a, m), replicated over (b, p)
 * The phase is evaluated in float64 in the reference's operation order, so the output is bit-exact to the
 * oracle.  `out` must be 8-byte aligned (a 16-byte aligned table takes the faster 16-byte-store block form). */
int bf_coeff_gen(const float* delay_vals, float* out, int B, int P, int C, int Ctot, int A, int M,
                 int xeng_id, double sample_period, void* stream);

/* Time-dependent compact coefficients (C++ study's steering kernels, BeamformerKernels.cu:7-189, with the
 * Python sign convention):
 *   rot(t, c, m, a) = (phi + phi_rate*dt) - pi*(tau + tau_rate*dt)*(ch - Ctot/2)/(Ctot*Ts),
 *   dt = t0 + t*dt_step for t in [0, n_times)
 *   delay_vals : f32 (Cd, M, A, 4) with Cd = C (per channel) or 1 (one model for every channel)
 *   out        : (n_times, C, A, M) complex: out_fp16 = 0 -> float2 (re, im); 1 -> half2 (b16BitOutput,
 *                BeamformerKernels.cu:111-116) */
int bf_coeff_gen_time(const float* delay_vals, int delay_channels, void* out, int out_fp16, int n_times,
                      int C, int Ctot, int A, int M, int xeng_id, double sample_period, double t0,
                      double dt_step, void* stream);

/* Time-dependent coefficients in the C++ study's OWN convention (replaces
 * calculate_beamweights_grouped_channels_and_timestamps, BeamformerKernels.cu:121-189, formula :155-170):
 *   dt = t*Ts*fft_size, dd = delay_rate*dt,
 *   rot = (delay_rate + dd)*c*pi/(Ts*C) + phase - (delay + dd)*(C/2)*pi/(Ts*C) + phase_rate*dt   (float32),
 * i.e. the delay rate in the channel term and the sign opposite to the Python path -- kept so that a
 * caller of the study's kernel gets its numbers; pinned by the study's own golden (BeamformerCoefficientTest.cu:
 * 294-337, tolerance 1e-4) restated in oracle/.
 *   delay_vals : f32 (A*M, 4), index a*M + m (the study's antenna-major struct delay_vals array)
 *   out        : (n_times, C, A, M) complex: out_fp16 = 0 -> float2 (cos, sin); 1 -> half2 */
int bf_coeff_gen_time_study(const float* delay_vals, void* out, int out_fp16, int n_times, int C, int A, int M,
                            float sample_period, int fft_size, void* stream);

/* The C++ study's fused coefficient + beamform kernel in the study's OWN semantics (replaces
 * calculate_beamweights_and_beamform_single_channel, BeamformerKernels.cu:192-367, as its harness's golden checks it,
 * BeamformerCoefficientTest.cu:356-400): per channel c, time t and beam m
 *   y_re = sum_a cos(rot) x_re,  y_im = sum_a sin(rot) x_im    (NOT a complex product: the study's semantics)
 * with rot bf_coeff_gen_time_study's expression at (t, c, a, m), antennas summed in order in float32.  The kernel's
 * shadowed prefetch (:277-282: every chunk after the first re-uses the first chunk's voltages) is not reproduced.
 *   delay_vals : f32 (M*A, 4), index m*A + a (the combined kernel's beam-major order)
 *   x          : int8 [C][T/16][A][16][2]  (char2 [channels][time/16][station][16]);  T % 16 == 0, A <= 2048
 *   out        : f32  [C][T/16][M][16][2] */
int bf_beamform_study_single_channel(const float* delay_vals, const int8_t* x, float* out, int C, int T, int A, int M,
                                     float sample_period, int fft_size, void* stream);

/* Pre-beamform reorder, bit-exact.
 * Replaces PreBeamformReorder._run / prebeamform_reorder kernel (beamformer/beamforming/prebeamform_reorder.py:
 * 171-186, kernels/prebeamform_reorder_kernel.mako:37-93):
 *   in  : u8 (B, A, C, T, 2, 2)   out : u8 (B, 2, C, T/16, 16, A, 2).   T % 16 == 0. */
int bf_reorder(const uint8_t* in, uint8_t* out, int B, int A, int C, int T, void* stream);

/* Beamform complex multiply (MFMA batched GEMM, f16 hi/lo coefficient split, f32 accumulation).
 * Replaces MatrixMultiply._run -> ComplexMultKernel.complex_mult -> run_complex_mult
 * (beamformer/beamforming/matrix_multiply.py:155-163, complex_mult_kernel.py:11-100, 106-162):
 *   x : 8-bit (B, P, C, NB, 16, A, 2)   w : f32 (B, P, C, 2A, 2M)   y : f32 (B, P, C, NB, 16, 2M)
 *   y[..., col] = sum_k x[..., k] * w[k, col] with x[2a] = re, x[2a+1] = im. */
int bf_beamform(const uint8_t* x, const float* w, float* y, int B, int P, int C, int NB, int A, int M,
                int sample_signed, void* stream);

/* Fused pre-beamform reorder + per-batch coefficient regeneration + beamform (one pass over the voltages).
 * Replaces the OpSequence chain (beamformer/beamforming/beamform_op_sequence.py:117-157: reorder ->
 * coeff gen -> multiply) and the C++ fused study kernel calculate_beamweights_and_beamform_single_channel
 * (beamformer_coefficient_generator/BeamformerKernels.cu:192-367, correct complex multiply):
 *   raw        : 8-bit (B, A, C, T, 2, 2), the reorder's input layout, read directly
 *   delay_vals : f32 (Cd, M, A, 4), Cd = C or 1; batch b uses dt_b = t0 + b*batch_dt (regeneration per
 *                block of T samples, BeamformerParameters.h:17); with zero rates/dt it equals OpSequence
 *   y          : f32 (B, 2, C, T/16, 16, 2M), or int8 = sat127(rne(y * out_scale)) with BF_FUSED_OUT_INT8
 *   flags      : BF_FUSED_SIGNED (int8 samples), BF_FUSED_OUT_INT8, BF_FUSED_EXACT_COEFF (float64 phasors
 *                bit-exact to bf_coeff_gen; default is the ~1-ulp float32 fast phasor).
 * int8 beams have two contracts:
 *   default               : the Q14 integer contract (oracle fused_beamform_int8): W = rne(2^14 * f32 phasor), exact
 *                           int32 sums, q = sat127(rne(f32(y) * out_scale * 2^-14)); integer MFMA, bit-exact;
 *   BF_FUSED_INT8_VIA_F32 : q = sat127(rne(y_f32 * out_scale)) of the float32 beams (the reference's float32
 *                           coefficient arithmetic, requantised in-kernel == bf_requant of the float output).
 * Kernel-path and workgroup-order overrides (BF_FUSED_PATH_*, BF_FUSED_ORDER_*) exist for tests and measurement:
 * every path computes the same contract, a path that does not fit the shape falls through to one that does, and
 * 0 (automatic) picks the fastest path for the shape.  The library never reads the environment. */
#define BF_FUSED_SIGNED 1
#define BF_FUSED_OUT_INT8 2
#define BF_FUSED_EXACT_COEFF 4
#define BF_FUSED_INT8_VIA_F32 8
#define BF_FUSED_PATH_MASK 0x0f00
#define BF_FUSED_PATH_ITEM 0x0100    /* one workgroup per (batch, channel) item (A <= 64, T <= 256), else generic */
#define BF_FUSED_PATH_GENERIC 0x0300 /* any A, any T: groups of 64 antennas */
#define BF_FUSED_PATH_WIDE 0x0400    /* many antennas x beams: multi-wave beam slabs (config 4) */
/* (0x0200 and 0x0600 named two measured-slower kernels of ABI 1.x, and 0x0500 (WIDE16) the 16-beam int8 wide kernel
 * of ABI 2.0, removed from the product in ABI 3.0 (0x0500: the 16-beam float slabs are what WIDE picks for M <= 16; the
 * int8 kernel lives on in the diagnostic build): all three are rejected as unknown.) */
#define BF_FUSED_ORDER_MASK 0x3000
#define BF_FUSED_ORDER_CHANNEL 0x1000 /* plain channel-fastest workgroup order (the persistent config-4 float
                                         kernel walks channel runs and has none: this flag takes the slab kernel) */
#define BF_FUSED_ORDER_XCD 0x2000     /* XCD-range order (XCD x streams channels [x C/8, (x+1) C/8)) */
int bf_beamform_fused(const uint8_t* raw, const float* delay_vals, int delay_channels, void* y, int B, int C,
                      int T, int A, int M, int Ctot, int xeng_id, double sample_period, double t0,
                      double batch_dt, int flags, float out_scale, void* stream);

/* bf_beamform_fused with per-input beam weights folded into the phasors (control-plane hook: the
 * `?beam-weights <beam> w_0 .. w_{A-1}` request, ngkcs/ngkcs/corr3_servlet.py:140-153, forwarded to the
 * B-engines).  gains: f32 (M, A) real weight of antenna a in beam m on the device, or NULL (= all ones, exactly
 * bf_beamform_fused).  Coefficient (a, m) becomes (g*cos, g*sin), one float32 rounding per component.  With
 * BF_FUSED_OUT_INT8 the Q14 integer path needs |g| <= 1.992 (the high limb stays int8) and
 * A*max|x|*(sqrt(2)*max|g|*2^14 + 1) < 2^31 (no int32 overflow; max|x| = 128 signed, 255 unsigned); the Python
 * wrapper, which owns the host copy of the weights, checks both.  Without gains the library checks the unit-gain
 * bound itself (A <= 363 unsigned, A <= 724 signed) and returns BF_ERR_ARG beyond it. */
int bf_beamform_fused_weighted(const uint8_t* raw, const float* delay_vals, int delay_channels, const float* gains,
                               void* y, int B, int C, int T, int A, int M, int Ctot, int xeng_id,
                               double sample_period, double t0, double batch_dt, int flags, float out_scale,
                               void* stream);

/* bf_beamform_fused_weighted with a caller-owned device workspace (the fused call itself never allocates).  With at
 * least bf_fused_workspace_bytes(...) bytes, the int8 beams of many antennas x beams (config 4: the 32-beam integer
 * kernel) take their Q14 coefficients from a table that bf_q14_coeffs' kernel writes into the workspace just before,
 * on `stream` -- the wavefront-parallel phasor generator of the reference's two-kernel structure (coeff_generator.py
 * then matrix_multiply.py; BeamformerKernels.cu:7-189), one float64 complex multiply per coefficient along the
 * channels -- instead of evaluating every phasor inside the contraction kernel.  Same contract, same bits; workspace
 * NULL (or too small) = bf_beamform_fused_weighted.  bf_fused_workspace_bytes gives 0 for shapes and flags that use
 * no workspace.  The workspace must be 16-byte aligned and must not be shared by calls in flight on other streams. */
int bf_fused_workspace_bytes(int B, int C, int T, int A, int M, int flags, size_t* bytes);
int bf_beamform_fused_ws(const uint8_t* raw, const float* delay_vals, int delay_channels, const float* gains, void* y,
                         int B, int C, int T, int A, int M, int Ctot, int xeng_id, double sample_period, double t0,
                         double batch_dt, int flags, float out_scale, void* workspace, size_t workspace_bytes,
                         void* stream);

/* The int8 path's steering coefficients (the Q14 integer contract, oracle quantise_coeffs of fused_tables):
 *   out[b][c][m][a] = (uint16)Wc | (uint32)Ws << 16, Wc = rne(2^14 * RN32(g * RN32(cos rot))), Ws the same for sin,
 *   rot the reference's float64 phase (coeff_generator_cpu.py:145-164) of channel c + C * xeng_id at
 *   dt = t0 + b * batch_dt (SURVEY A3 time extension), g = gains[m][a] (NULL = 1).  delay_vals f32 (Cd, M, A, 4). */
int bf_q14_coeffs(const float* delay_vals, int delay_channels, const float* gains, uint32_t* out, int B, int C, int A,
                  int M, int Ctot, int xeng_id, double sample_period, double t0, double batch_dt, void* stream);

/* 8-bit requantiser (no reference counterpart; SURVEY §7 build step 7): q = clamp(rne(y*scale), -127, 127). */
int bf_requant(const float* y, int8_t* q, size_t n, float scale, void* stream);

/* ---- streaming ingest --------------------------------------------------------
 * Pinned host frames -> H2D stream -> bf_beamform_fused_weighted on a compute stream -> D2H stream, over a ring of
 * `depth` device slots; the phases of successive frames overlap.  Replaces the back-to-back HtoD / kernel / DtoH
 * phases of the reference harness (common/UnitTest.cpp:28-57) and the event-chained PCIe loop
 * (utilities/pcie_bandwidth_tests/cudaPcieRateTest.cpp:63-123).  Frames have the fused operator's shapes: in
 * (B, A, C, T, 2, 2) 8-bit, out (B, 2, C, T/16, 16, 2M) f32 or int8.  Host buffers should be pinned
 * (bf_host_alloc) for the copies to overlap; they must stay untouched until bf_pipeline_wait(ticket, 0) (input)
 * / (ticket, 1) (output).  The pipeline lives on the device current at creation; calls restore the caller's device.
 * Delay-model and weight updates apply to every frame submitted after them (stream-ordered uploads). */
typedef struct bf_pipeline bf_pipeline;
int bf_pipeline_create(bf_pipeline** out, int B, int C, int T, int A, int M, int Ctot, int xeng_id,
                       double sample_period, int flags, float out_scale, int delay_channels, int depth);
int bf_pipeline_destroy(bf_pipeline* p);
int bf_pipeline_frame_bytes(const bf_pipeline* p, size_t* in_bytes, size_t* out_bytes);
int bf_pipeline_set_delays(bf_pipeline* p, const float* host_delay_vals);  /* host f32 (Cd, M, A, 4) */
int bf_pipeline_set_gains(bf_pipeline* p, const float* host_gains);        /* host f32 (M, A); NULL = unit */
int bf_pipeline_submit(bf_pipeline* p, const void* host_in, void* host_out, double t0, double batch_dt,
                       long long* ticket);
int bf_pipeline_wait(bf_pipeline* p, long long ticket, int stage);         /* stage 0 input, 1 output */
int bf_pipeline_query(bf_pipeline* p, long long ticket, int stage, int* done);
int bf_pipeline_flush(bf_pipeline* p);
int bf_pipeline_stage_ms(bf_pipeline* p, long long ticket, float* h2d_ms, float* compute_ms, float* d2h_ms);

/* ---- multi-GPU channel scatter --------------------------------------------------------------
 * One process per GPU, rank r = X-engine r owning channels [C r, C (r+1)) of a C*N-channel band (the reference's
 * absolute-channel convention, beamformer/beamforming/coeff_generator.py:49-53; its only multi-device pattern is a
 * host thread per device, utilities/pcie_bandwidth_tests/main.cpp:193-224, which this replaces).  The hot path
 * needs no collective; the root hands each rank its channel slice of a full-band cube once, device to device over
 * RCCL/xGMI.  RCCL (/opt/rocm librccl.so.1) is loaded at the first bf_comm_* call.
 *   bf_comm_unique_id : rank 0 makes the communicator id (BF_COMM_ID_BYTES); the caller hands it to every rank
 *   bf_comm_create    : collective over all ranks, on the device current at the call
 *   bf_channel_scatter: band (B, A, C*N, T, 2, 2) 8-bit on `root` (ignored elsewhere) -> slice (B, A, C, T, 2, 2) on
 *                       every rank; stream-ordered on `stream`, in pieces of at most 256 MiB (whole (b, a) rows,
 *                       or segments of a longer row), one RCCL group per piece.  Root: each peer's slice 2-D packed
 *                       into a staging buffer of N - 1 slices (grown on demand) and sent with ncclSend, its own slice
 *                       one 2-D copy; at one rank the root's slice is packed and moved by a self ncclSend/ncclRecv
 *                       instead, so one rank runs the point-to-point path of N.  Peers: ncclRecv per piece.
 *   bf_comm_allreduce_max: host value -> max over ranks (blocking; timing brackets and agreement checks)
 *   bf_comm_stats     : bytes this rank has handed to ncclSend / ncclRecv so far (the scatter's RCCL traffic)
 *   bf_comm_load      : BF_OK when RCCL can be loaded (a local precondition each rank checks before the collective
 *                       bf_comm_create, so that no rank waits in it for a rank that already failed) */
#define BF_COMM_ID_BYTES 128
typedef struct bf_comm bf_comm;
int bf_comm_unique_id(void* id, size_t len);
int bf_comm_create(bf_comm** out, const void* id, size_t len, int nranks, int rank);
int bf_comm_destroy(bf_comm* comm);
int bf_comm_allreduce_max(bf_comm* comm, double* value);
int bf_channel_scatter(bf_comm* comm, const uint8_t* band, uint8_t* slice, int B, int A, int C, int T, int root,
                       void* stream);
int bf_comm_stats(const bf_comm* comm, unsigned long long* sent, unsigned long long* received);
int bf_comm_load(void);

/* The scatter's plan for one rank: pure host arithmetic (no device, no RCCL), the exact operation list
 * bf_channel_scatter executes, so the piece / staging-slot / send-receive pairing logic is testable on a CPU for any
 * N and root (tests/test_multi_rank.py replays the N ranks' plans on host buffers).  Ops in execution order:
 *   BF_SCATTER_COPY2D: `height` rows of `width` bytes, (src_space, src_off, src_pitch) -> (dst_space, dst_off,
 *                      dst_pitch); `peer` = the rank whose slice the rows belong to (root only)
 *   BF_SCATTER_SEND  : `width` bytes at (src_space, src_off) to rank `peer` (ncclSend)
 *   BF_SCATTER_RECV  : `width` bytes into (dst_space, dst_off) from rank `peer` (ncclRecv)
 * `group` numbers the pieces: one RCCL group per piece, its COPY2D ops first.  Spaces: the root's band, the root's
 * staging buffer (`*staging_bytes` long), this rank's slice.  chunk = the piece size in bytes (0: the product's
 * 256 MiB).  ops == NULL only counts; a capacity below the count fails with BF_ERR_ARG (`*n_ops` holds the count). */
#define BF_SCATTER_COPY2D 1
#define BF_SCATTER_SEND 2
#define BF_SCATTER_RECV 3
#define BF_SPACE_BAND 1
#define BF_SPACE_STAGING 2
#define BF_SPACE_SLICE 3
typedef struct bf_scatter_op {
  int kind, peer, group, src_space, dst_space, reserved;
  unsigned long long src_off, src_pitch, dst_off, dst_pitch, width, height;
} bf_scatter_op;
int bf_scatter_plan(int nranks, int rank, int root, int B, int A, int C, int T, size_t chunk, bf_scatter_op* ops,
                    size_t capacity, size_t* n_ops, size_t* staging_bytes);

/* Position-weighted 64-bit checksum of a 2-D device region (`rows` runs of `run_bytes`, `pitch_bytes` apart; 4-byte
 * words): sum over packed word index i of splitmix64(splitmix64(i) ^ word_i), mod 2^64 -- equal for a packed slice
 * and the strided band region it came from.  Blocking (synchronises `stream`); verification, not the hot path. */
int bf_checksum(const void* src, size_t run_bytes, size_t pitch_bytes, size_t rows, unsigned long long* out,
                void* stream);

/* Fill `bytes` of device memory with a deterministic pseudo-random byte stream (splitmix64 of seed and position):
 * synthetic voltages made in HBM (bench.py's full-band cube at N GPUs), no host staging. */
int bf_fill_random(void* dst, size_t bytes, unsigned long long seed, void* stream);

/* Algorithmic HBM bytes of one bf_beamform_fused launch (bench / roofline bookkeeping). */
double bf_fused_algorithmic_bytes(int B, int C, int T, int A, int M, int delay_channels, int out_int8);

#ifdef __cplusplus
}
#endif
#endif /* DPDK_DC_SAND_AMD_BF_H */
