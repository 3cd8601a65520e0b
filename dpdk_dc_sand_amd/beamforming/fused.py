"""One-pass beamformer: reorder + per-batch coefficient regeneration + multiply (MI355X-native operator).

The reference's OpSequence (beamform_op_sequence.py:117-157) makes three passes: the reorder reads and
writes the whole voltage cube (prebeamform_reorder_kernel.mako:37-93), the coefficient generator writes a
(B, P, C, 2A, 2M) f32 table replicated over batches and pols (16 B per complex coefficient, as large as the
voltages at 16 beams), and the multiply reads both back.  `FusedBeamformer` reads the raw (B, A, C, T, 2, 2)
cube once, generates each (b, c)'s coefficients in-kernel from the delay model (float64 phase, the same
arithmetic as CoeffGenerator, so with zero rates the output equals OpSequence's), and writes the beams once:
the HBM traffic is the algorithmic minimum.

Beam weights (control-plane hook): the `?beam-weights <beam> w_0 .. w_{A-1}` request the
control servlet forwards to the B-engines (ngkcs/ngkcs/corr3_servlet.py:140-153) sets one real weight per input
for one beam.  With `beam_weights=True` the operator carries an (M, A) weight table (all ones initially) that is
folded into the phasors in-kernel: W(a, m) = g(m, a) * (cos, sin) -- no extra pass, no extra HBM traffic.

Per-block regeneration (BeamformerParameters.h:17 ACCUMULATIONS_BEFORE_NEW_COEFFS, the C++ study's
time-dependent kernels BeamformerKernels.cu:121-189 and the fused study kernel :192-367): batch b is steered
at dt_b = t0 + b * batch_dt using the delay and phase rates (SURVEY A3 convention).
"""
import ctypes

import numpy as np

from .. import _lib, accel


class FusedBeamformerTemplate:
    """Template for the fused beamformer.

    Parameters
    ----------
    context, n_batches, n_channels_per_stream, n_channels (whole band), n_samples_per_channel, n_ants, n_beams,
    xeng_id, sample_period -- as the reference templates.
    delay_channels: 1 (one delay model for every channel, the physical case; 16*A*M bytes) or
        n_channels_per_stream (the reference's per-channel (C, M, A, 4) table).  Default: n_channels_per_stream.
    sample_signed: read voltages as int8 instead of uint8.
    out_int8, out_scale: write int8 beams sat127(rne(y * out_scale)) instead of float32.
    t0, batch_dt: steering time of batch 0 and the step between batches (seconds).
    exact_coeffs: float64 phasors bit-exact to CoeffGenerator (then, with zero rates, the output equals
        OpSequence's bit for bit); default False = float32 phasors within ~1 ulp, several times cheaper.
    beam_weights: carry a per-(beam, input) real weight table (slot beamWeights, set with set_beam_weights).
    int8_contract: with out_int8, "q14" (default: the integer contract, Q14 coefficients and exact int32 sums on the
        integer MFMA path) or "f32" (requantised float32 beams: the reference's float32 coefficient arithmetic).
    kernel_path, workgroup_order: force a kernel path ("auto", "item", "generic", "wide") or
        workgroup order ("auto", "channel", "xcd") -- tests and measurement; every path computes the same contract.
    coeff_table: let the int8 wide path (many antennas x beams, e.g. config 4) take its Q14 coefficients from a
        table generated just before each launch by the wavefront-parallel phasor kernel (bf_beamform_fused_ws: a
        device workspace of `workspace_bytes` the operator allocates once) rather than evaluating every phasor in
        the contraction kernel.  Same contract, same bits; default True.  Other shapes/paths need no workspace.
    """

    # int32 bound of the Q14 contract: |Wc| + |Ws| <= sqrt(2) * 2^14 * |g| + 1 per coefficient
    @staticmethod
    def _int8_sum_bound(n_ants, signed, gain=1.0):
        return n_ants * (128 if signed else 255) * (np.sqrt(2.0) * 16384.0 * gain + 1.0)

    def __init__(self, context, n_batches: int, n_channels_per_stream: int, n_channels: int,
                 n_samples_per_channel: int, n_ants: int, n_beams: int, xeng_id: int = 0,
                 sample_period: float = 1 / 1712e6, delay_channels=None, sample_signed: bool = False,
                 out_int8: bool = False, out_scale: float = 1.0, t0: float = 0.0, batch_dt: float = 0.0,
                 exact_coeffs: bool = False, beam_weights: bool = False, int8_contract: str = "q14",
                 kernel_path: str = "auto", workgroup_order: str = "auto", coeff_table: bool = True) -> None:
        for name, v in dict(n_batches=n_batches, n_channels_per_stream=n_channels_per_stream, n_channels=n_channels,
                            n_samples_per_channel=n_samples_per_channel, n_ants=n_ants, n_beams=n_beams).items():
            if int(v) <= 0:
                raise ValueError(f"{name} must be positive, got {v}")
        if n_samples_per_channel % 16:
            raise ValueError("n_samples_per_channel must be a multiple of 16")
        if delay_channels is None:
            delay_channels = n_channels_per_stream
        if delay_channels not in (1, n_channels_per_stream):
            raise ValueError("delay_channels must be 1 or n_channels_per_stream")
        if not sample_period > 0:
            raise ValueError("sample_period must be > 0")
        if int8_contract not in ("q14", "f32"):
            raise ValueError(f"int8_contract must be 'q14' or 'f32', got {int8_contract!r}")
        if kernel_path not in _lib.FUSED_PATH:
            raise ValueError(f"kernel_path must be one of {sorted(_lib.FUSED_PATH)}, got {kernel_path!r}")
        if workgroup_order not in _lib.FUSED_ORDER:
            raise ValueError(f"workgroup_order must be one of {sorted(_lib.FUSED_ORDER)}, got {workgroup_order!r}")
        if out_int8 and int8_contract == "q14" and self._int8_sum_bound(n_ants, sample_signed) >= 2 ** 31:
            raise ValueError(f"{n_ants} antennas overflow the int8 path's int32 beam sums; use float beams or "
                             "int8_contract='f32'")
        self.context = context
        self.n_batches = n_batches
        self.n_pols = 2
        self.n_channels_per_stream = n_channels_per_stream
        self.n_channels = n_channels
        self.n_samples_per_channel = n_samples_per_channel
        self.n_samples_per_block = 16
        self.n_blocks = n_samples_per_channel // 16
        self.n_ants = n_ants
        self.n_beams = n_beams
        self.xeng_id = xeng_id
        self.sample_period = sample_period
        self.delay_channels = delay_channels
        self.sample_signed = bool(sample_signed)
        self.out_int8 = bool(out_int8)
        self.out_scale = float(out_scale)
        self.t0 = float(t0)
        self.batch_dt = float(batch_dt)
        self.exact_coeffs = bool(exact_coeffs)
        self.beam_weights = bool(beam_weights)
        self.int8_contract = int8_contract
        self.kernel_path = kernel_path
        self.workgroup_order = workgroup_order
        self.flags = ((_lib.FUSED_SIGNED if self.sample_signed else 0) | (_lib.FUSED_OUT_INT8 if self.out_int8 else 0)
                      | (_lib.FUSED_EXACT_COEFF if self.exact_coeffs else 0)
                      | (_lib.FUSED_INT8_VIA_F32 if self.out_int8 and int8_contract == "f32" else 0)
                      | _lib.FUSED_PATH[kernel_path] | _lib.FUSED_ORDER[workgroup_order])
        B, C, T, A, M = n_batches, n_channels_per_stream, n_samples_per_channel, n_ants, n_beams
        self.input_shape = (B, A, C, T, 2, 2)
        self.delay_shape = (delay_channels, M, A, 4)
        self.output_shape = (B, 2, C, T // 16, 16, 2 * M)
        self.weights_shape = (M, A)
        self.coeff_table = bool(coeff_table)
        self.workspace_bytes = 0
        if self.coeff_table:
            n = ctypes.c_size_t(0)
            _lib.call("bf_fused_workspace_bytes", B, C, T, A, M, self.flags, ctypes.byref(n))
            self.workspace_bytes = int(n.value)

    def check_weights(self, weights):
        """Validate an (M, A) weight table for this configuration; returns it as float32.  The int8 output's
        Q14 integer path needs rne(|g| * 2^14) <= 32639, i.e. |g| <= 1.992 (the high limb stays int8), and
        A * max|x| * (sqrt(2) * max|g| * 2^14 + 1) < 2^31 (no int32 overflow); the float path takes any finite
        weights."""
        w = np.asarray(weights, np.float32)
        if w.shape != self.weights_shape:
            raise ValueError(f"beam weights must have shape {self.weights_shape}, got {w.shape}")
        if not np.all(np.isfinite(w)):
            raise ValueError("beam weights must be finite")
        if self.out_int8 and self.int8_contract == "q14":
            g = float(np.max(np.abs(w))) if w.size else 0.0
            if np.rint(g * 16384) > 32639 or self._int8_sum_bound(self.n_ants, self.sample_signed, g) >= 2 ** 31:
                raise ValueError(f"beam weight magnitude {g} out of range for int8 output with {self.n_ants} inputs")
        return w

    def algorithmic_bytes(self):
        """HBM bytes one launch must move: voltages once, beams once, delay model once."""
        return _lib.load().bf_fused_algorithmic_bytes(self.n_batches, self.n_channels_per_stream,
                                                      self.n_samples_per_channel, self.n_ants, self.n_beams,
                                                      self.delay_channels, int(self.out_int8))

    def instantiate(self, command_queue):
        return FusedBeamformer(self, command_queue)


class FusedBeamformer(accel.Operation):
    """.. rubric:: Slots
    inSamples: (n_batches, n_ants, n_channels_per_stream, n_samples_per_channel, 2, 2), uint8 (int8 if signed)
    delay_vals: (delay_channels, n_beams, n_ants, 4), float32
    outData: (n_batches, 2, n_channels_per_stream, n_blocks, 16, 2*n_beams), float32 (int8 if out_int8)
    """

    def __init__(self, template: FusedBeamformerTemplate, command_queue):
        super().__init__(command_queue)
        self.template = t = template
        self.slots["inSamples"] = accel.IOSlot(t.input_shape, np.int8 if t.sample_signed else np.uint8)
        self.slots["delay_vals"] = accel.IOSlot(t.delay_shape, np.float32)
        self.slots["outData"] = accel.IOSlot(t.output_shape, np.int8 if t.out_int8 else np.float32)
        self._weights = None
        self._workspace = None  # the Q14 coefficient table of the int8 wide path (allocated on first use)
        if t.beam_weights:
            self.slots["beamWeights"] = accel.IOSlot(t.weights_shape, np.float32)
            self._weights = np.ones(t.weights_shape, np.float32)
            self._weights_dirty = True

    def set_beam_weights(self, beam, *weights):
        """`?beam-weights <beam> w_0 .. w_{A-1}` (corr3_servlet.py:140-153): set beam `beam`'s per-input weights.
        Same reply condition as the servlet: the count must equal n_ants (ValueError here, FailReply there).
        Takes effect from the next launch (stream-ordered upload)."""
        t = self.template
        if self._weights is None:
            raise ValueError("operator was built without beam_weights=True")
        if len(weights) == 1 and np.ndim(weights[0]) == 1:
            weights = tuple(weights[0])
        if len(weights) != t.n_ants:
            raise ValueError(f"{len(weights)} weights received, expected {t.n_ants}")
        if not 0 <= int(beam) < t.n_beams:
            raise ValueError(f"beam {beam} out of range [0, {t.n_beams})")
        new = self._weights.copy()
        new[int(beam)] = np.asarray(weights, np.float32)
        self._weights = t.check_weights(new)
        self._weights_dirty = True

    def beam_weights(self):
        """The current (M, A) weight table (host copy)."""
        return None if self._weights is None else self._weights.copy()

    def _run(self):
        t = self.template
        gains = None
        if self._weights is not None:
            buf = self.buffer("beamWeights")
            if self._weights_dirty:
                buf.set_async(self.command_queue, self._weights)
                self._weights_dirty = False
            gains = buf.ptr
        if t.workspace_bytes and self._workspace is None:
            self._workspace = accel.DeviceArray(self.command_queue.context, (t.workspace_bytes,), np.uint8)
        ws = self._workspace.ptr if self._workspace is not None else None
        _lib.call("bf_beamform_fused_ws", self.buffer("inSamples").ptr, self.buffer("delay_vals").ptr,
                  t.delay_channels, gains, self.buffer("outData").ptr, t.n_batches, t.n_channels_per_stream,
                  t.n_samples_per_channel, t.n_ants, t.n_beams, t.n_channels, t.xeng_id, float(t.sample_period),
                  t.t0, t.batch_dt, t.flags, t.out_scale, ws, t.workspace_bytes, self.command_queue.handle)
