"""Streaming ingest beamformer: host frames -> GPU -> host beams, overlapped.

The reference moves data host <-> device in separate, back-to-back phases (HtoD, kernel, DtoH: common/UnitTest.cpp:
28-57; the event-chained PCIe rate test, utilities/pcie_bandwidth_tests/cudaPcieRateTest.cpp:63-123).  Here the
native pipeline in libbf (bf_pipeline_*, csrc/bf_pipeline.cpp) keeps `depth` frames in flight on three HIP streams:
the H2D copy of frame n+1, the fused beamform (+ int8 requantisation) of frame n and the D2H copy of frame n-1 run
at once, so the sustained rate is set by the slowest of PCIe-in, compute and PCIe-out rather than their sum.

A frame is one fused-operator batch block: (n_batches, n_ants, n_channels_per_stream, n_samples_per_channel, 2, 2)
8-bit voltages in, (n_batches, 2, n_channels_per_stream, n_blocks, 16, 2 n_beams) beams out.  Consecutive frames
are consecutive in time: frame k is steered from t0 + k * frame_dt (frame_dt = n_batches * batch_dt) unless the
caller passes t0 explicitly.
"""
import ctypes

import numpy as np

from .. import _lib, accel
from .fused import FusedBeamformerTemplate

STAGES = {"input": 0, "output": 1}


class StreamingBeamformerTemplate(FusedBeamformerTemplate):
    """FusedBeamformerTemplate parameters plus `depth` (frames in flight, >= 2 to overlap; default 4)."""

    def __init__(self, context, *args, depth: int = 4, **kwargs):
        super().__init__(context, *args, **kwargs)
        if not 1 <= int(depth) <= 64:
            raise ValueError("depth must be in [1, 64]")
        self.depth = int(depth)
        self.frame_dt = self.n_batches * self.batch_dt

    def instantiate(self):
        return StreamingBeamformer(self)


class StreamingBeamformer:
    """Owns one bf_pipeline (its streams, device ring and pinned staging).  Not thread-safe."""

    def __init__(self, template: StreamingBeamformerTemplate):
        self.template = t = template
        if t.context is not None:
            t.context.activate()
        h = ctypes.c_void_p()
        _lib.call("bf_pipeline_create", ctypes.byref(h), t.n_batches, t.n_channels_per_stream, t.n_samples_per_channel,
                  t.n_ants, t.n_beams, t.n_channels, t.xeng_id, float(t.sample_period), t.flags, t.out_scale,
                  t.delay_channels, t.depth)
        self._h = h.value
        self._inflight = {}  # ticket -> (samples, beams): keep host buffers alive until their copies retire
        self._weights = np.ones(t.weights_shape, np.float32) if t.beam_weights else None
        self.frames_submitted = 0
        self.in_dtype = np.int8 if t.sample_signed else np.uint8
        self.out_dtype = np.int8 if t.out_int8 else np.float32

    # ---- buffers ----
    def host_frames(self, n=None):
        """`n` (default depth) pinned (samples, beams) frame buffer pairs."""
        t = self.template
        return [(accel.HostArray(t.input_shape, self.in_dtype), accel.HostArray(t.output_shape, self.out_dtype))
                for _ in range(t.depth if n is None else n)]

    # ---- control ----
    def set_delays(self, delay_vals):
        """Delay model (delay_channels, n_beams, n_ants, 4) float32; applies to every frame submitted after it."""
        d = np.ascontiguousarray(delay_vals, np.float32)
        if d.shape != self.template.delay_shape:
            raise ValueError(f"delay_vals must have shape {self.template.delay_shape}, got {d.shape}")
        _lib.call("bf_pipeline_set_delays", self._h, d.ctypes.data)

    def set_beam_weights(self, beam, *weights):
        """`?beam-weights <beam> w_0 .. w_{A-1}` (corr3_servlet.py:140-153), from the next submitted frame on."""
        t = self.template
        if self._weights is None:
            raise ValueError("pipeline was built without beam_weights=True")
        if len(weights) == 1 and np.ndim(weights[0]) == 1:
            weights = tuple(weights[0])
        if len(weights) != t.n_ants:
            raise ValueError(f"{len(weights)} weights received, expected {t.n_ants}")
        if not 0 <= int(beam) < t.n_beams:
            raise ValueError(f"beam {beam} out of range [0, {t.n_beams})")
        new = self._weights.copy()
        new[int(beam)] = np.asarray(weights, np.float32)
        self._weights = t.check_weights(new)
        _lib.call("bf_pipeline_set_gains", self._h, self._weights.ctypes.data)

    # ---- data path ----
    def submit(self, samples, beams, t0=None):
        """Queue one frame; returns its ticket.  `samples` / `beams` are host arrays of the frame shapes (pinned
        HostArray for overlap).  Do not touch `samples` before wait(ticket, "input") nor read `beams` before
        wait(ticket, "output")."""
        t = self.template
        for a, shape, dt, what in ((samples, t.input_shape, self.in_dtype, "samples"),
                                   (beams, t.output_shape, self.out_dtype, "beams")):
            if not isinstance(a, np.ndarray) or a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                raise ValueError(f"{what} must be a C-contiguous {np.dtype(dt)} array of shape {shape}")
        if not beams.flags.writeable:
            raise ValueError("beams must be writeable")
        if t0 is None:
            t0 = t.t0 + self.frames_submitted * t.frame_dt
        ticket = ctypes.c_longlong()
        _lib.call("bf_pipeline_submit", self._h, samples.ctypes.data, beams.ctypes.data, float(t0), t.batch_dt,
                  ctypes.byref(ticket))
        self.frames_submitted += 1
        self._inflight[ticket.value] = (samples, beams)
        return ticket.value

    def wait(self, ticket, stage="output"):
        _lib.call("bf_pipeline_wait", self._h, int(ticket), STAGES[stage])
        if stage == "output":
            for k in [k for k in self._inflight if k <= ticket]:
                del self._inflight[k]

    def done(self, ticket, stage="output"):
        flag = ctypes.c_int()
        _lib.call("bf_pipeline_query", self._h, int(ticket), STAGES[stage], ctypes.byref(flag))
        return bool(flag.value)

    def flush(self):
        _lib.call("bf_pipeline_flush", self._h)
        self._inflight.clear()

    def stage_ms(self, ticket):
        """(h2d, compute, d2h) milliseconds of one of the last `depth` frames (waits for it)."""
        v = [ctypes.c_float() for _ in range(3)]
        _lib.call("bf_pipeline_stage_ms", self._h, int(ticket), *[ctypes.byref(x) for x in v])
        return tuple(x.value for x in v)

    def close(self):
        if getattr(self, "_h", None):
            try:
                _lib.load().bf_pipeline_destroy(self._h)  # drains the streams first
            except Exception:  # interpreter shutdown
                pass
            self._h = None
            self._inflight.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()
