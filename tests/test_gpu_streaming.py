"""GPU: the streaming ingest pipeline -- frames through H2D -> fused beamform -> D2H with the
stages overlapped -- reproduces the fused operator's contract frame by frame, including mid-stream delay-model and
beam-weight updates (stream-ordered: they apply from the next submitted frame on)."""
import numpy as np
import pytest

import oracle as O
from dpdk_dc_sand_amd import accel
from dpdk_dc_sand_amd.beamforming import StreamingBeamformerTemplate
from tolerance import assert_beams_allclose

pytestmark = pytest.mark.gpu
TS = O.TS_MEERKAT


def delays(M, A, seed):
    rng = np.random.default_rng(seed)
    d = np.zeros((1, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, (1, M, A))
    d[..., 1] = rng.uniform(-1e-9, 1e-9, (1, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (1, M, A))
    d[..., 3] = rng.uniform(-1, 1, (1, M, A))
    return d


@pytest.mark.parametrize("A,M,C,T,B,depth,signed", [(19, 3, 5, 64, 2, 3, True), (64, 16, 4, 256, 2, 2, False),
                                                    (130, 9, 2, 32, 1, 4, True)])
def test_stream_int8_bit_exact_with_updates(context, A, M, C, T, B, depth, signed):
    Ctot, xeng, bdt = 64 * C, 1, T * 2 * 64 * C * TS
    tmpl = StreamingBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1,
                                       sample_signed=signed, out_int8=True, out_scale=1 / 32, t0=0.25,
                                       batch_dt=bdt, beam_weights=True, depth=depth)
    rng = np.random.default_rng(A + C)
    n_frames = 3 * depth + 1
    frames = [rng.integers(0, 256, tmpl.input_shape, dtype=np.uint8) for _ in range(n_frames)]
    if signed:
        frames = [f.view(np.int8) for f in frames]
    d0, d1 = delays(M, A, 1), delays(M, A, 2)
    g = np.ones((M, A), np.float32)
    expected_models = []
    with tmpl.instantiate() as sb:
        bufs = sb.host_frames()
        sb.set_delays(d0)
        tickets, d_cur = [], d0
        for k, f in enumerate(frames):
            if k == 2:
                w = rng.uniform(-1.5, 1.5, A).astype(np.float32)
                sb.set_beam_weights(M - 1, *w)
                g = g.copy()
                g[M - 1] = w
            if k == depth + 1:
                sb.set_delays(d1)
                d_cur = d1
            samples, beams = bufs[k % depth]
            if k >= depth:
                sb.wait(tickets[k - depth])  # slot's host buffers are free again
                check(tickets[k - depth], bufs, depth, frames, expected_models, tmpl, signed)
            samples[...] = f
            tickets.append(sb.submit(samples, beams))
            expected_models.append((d_cur, g, tmpl.t0 + k * tmpl.frame_dt))
        for tk in tickets[-depth:]:
            sb.wait(tk)
            check(tk, bufs, depth, frames, expected_models, tmpl, signed)
        h2d, comp, d2h = sb.stage_ms(tickets[-1])
        assert h2d > 0 and comp > 0 and d2h > 0
        assert sb.done(tickets[-1]) and sb.done(tickets[-1], "input")


def test_stream_update_before_every_frame(context):
    """A new delay model and new beam weights before every frame (more updates in flight than the pipeline's 4
    staging buffers per table): each frame still uses exactly the model current when it was submitted."""
    A, M, C, T, B, depth = 19, 3, 5, 64, 2, 3
    Ctot, bdt = 64 * C, T * 2 * 64 * C * TS
    tmpl = StreamingBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=0, delay_channels=1, out_int8=True,
                                       out_scale=1 / 32, t0=0.0, batch_dt=bdt, beam_weights=True, depth=depth)
    rng = np.random.default_rng(7)
    n_frames = 4 * depth + 2
    frames = [rng.integers(0, 256, tmpl.input_shape, dtype=np.uint8) for _ in range(n_frames)]
    models = []
    g = np.ones((M, A), np.float32)
    with tmpl.instantiate() as sb:
        bufs = sb.host_frames()
        tickets = []
        for k, f in enumerate(frames):
            d = delays(M, A, 100 + k)
            sb.set_delays(d)
            w = rng.uniform(-1.5, 1.5, A).astype(np.float32)
            sb.set_beam_weights(k % M, *w)
            g = g.copy()
            g[k % M] = w
            samples, beams = bufs[k % depth]
            if k >= depth:
                sb.wait(tickets[k - depth])
                check(tickets[k - depth], bufs, depth, frames, models, tmpl, False)
            samples[...] = f
            tickets.append(sb.submit(samples, beams))
            models.append((d, g, tmpl.t0 + k * tmpl.frame_dt))
        for tk in tickets[-depth:]:
            sb.wait(tk)
            check(tk, bufs, depth, frames, models, tmpl, False)


def test_stream_cfg5_frames_sampled_bit_exact(context):
    """Config 5 at its real frame size: 2 * depth + 1 frames of (1, 64, 4096, 256, 2, 2) int8 voltages (256 MiB each,
    int8 beams out) streamed through the pipeline with a new delay model from frame `depth` on; in EVERY frame,
    sampled channel items (first, last and random) are bit-exact to the integer contract evaluated on that channel
    slice at the frame's steering time (as tests/test_gpu_fullsize.py samples a full-size launch)."""
    B, A, C, T, M, depth = 1, 64, 4096, 256, 16, 4
    Ctot, xeng = C, 0
    bdt = T * 2 * Ctot * TS
    tmpl = StreamingBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1,
                                       sample_signed=True, out_int8=True, out_scale=1 / 64, t0=1e-3, batch_dt=bdt,
                                       depth=depth)
    rng = np.random.default_rng(55)
    n_frames = 2 * depth + 1
    frames = [np.frombuffer(rng.bytes(int(np.prod(tmpl.input_shape))), np.int8).reshape(tmpl.input_shape)
              for _ in range(n_frames)]
    d0, d1 = delays(M, A, 21), delays(M, A, 22)
    models, tickets, checked = [], [], []

    def check_sampled(tk, beams):
        d, t0 = models[tk]
        items = {0, C - 1} | {int(c) for c in np.random.default_rng(tk).integers(0, C, 6)}
        for c in sorted(items):
            sl = np.ascontiguousarray(frames[tk][:, :, c:c + 1])
            ref = O.fused_beamform_int8(sl, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, scale=1 / 64, signed=True,
                                        ch0=C * xeng + c)
            np.testing.assert_array_equal(beams[:, :, c:c + 1], ref, err_msg=f"frame {tk} channel {c}")
        checked.append(tk)

    with tmpl.instantiate() as sb:
        bufs = sb.host_frames()
        sb.set_delays(d0)
        d_cur = d0
        for k, f in enumerate(frames):
            if k == depth:
                sb.set_delays(d1)
                d_cur = d1
            samples, beams = bufs[k % depth]
            if k >= depth:
                sb.wait(tickets[k - depth])
                check_sampled(tickets[k - depth], beams)
            samples[...] = f
            tickets.append(sb.submit(samples, beams))
            models.append((d_cur, tmpl.t0 + k * tmpl.frame_dt))
        for tk in tickets[-depth:]:
            sb.wait(tk)
            check_sampled(tk, bufs[tk % depth][1])
    assert checked == list(range(n_frames))
    assert np.abs(bufs[0][1].astype(int)).max() >= 8  # a live requantised range, not all zeros


def check(ticket, bufs, depth, frames, models, tmpl, signed):
    d, g, t0 = models[ticket]
    ref = O.fused_beamform_int8(frames[ticket], d, tmpl.n_channels, xeng_id=tmpl.xeng_id, t0=t0,
                                batch_dt=tmpl.batch_dt, scale=tmpl.out_scale, signed=signed, gains=g)
    np.testing.assert_array_equal(bufs[ticket % depth][1], ref, err_msg=f"frame {ticket}")


def test_stream_float_and_pageable_buffers(context):
    """float32 beams, plain (pageable) numpy frames: still correct, just without DMA overlap guarantees."""
    B, A, C, T, M, depth = 2, 32, 3, 128, 8, 2
    Ctot, bdt = 96, 128 * 2 * 96 * TS
    tmpl = StreamingBeamformerTemplate(context, B, C, Ctot, T, A, M, delay_channels=1, batch_dt=bdt, depth=depth)
    rng = np.random.default_rng(4)
    d = delays(M, A, 3)
    frames = [rng.integers(0, 256, tmpl.input_shape, dtype=np.uint8) for _ in range(5)]
    outs = [np.empty(tmpl.output_shape, np.float32) for _ in range(5)]
    with tmpl.instantiate() as sb:
        sb.set_delays(d)
        tickets = [sb.submit(f, o) for f, o in zip(frames, outs)]
        sb.flush()
        assert sb.done(tickets[-1])
    for k, (f, o) in enumerate(zip(frames, outs)):
        t0 = k * tmpl.frame_dt
        ref = O.fused_beamform(f, d, Ctot, t0=t0, batch_dt=bdt)
        w = O.fused_tables(d, B, C, Ctot, A, t0=t0, batch_dt=bdt)
        assert_beams_allclose(o, ref, O.reorder(f), w)


def test_stream_gain_bound_checked_by_the_library(context):
    """bf_pipeline_set_gains refuses weights that would overflow the Q14 path's int32 sums (or push the high limb past
    int8) itself -- a C caller need not rely on the Python wrapper's check; unit weights and the float
    contract's pipelines take them."""
    from dpdk_dc_sand_amd import _lib
    A, M = 300, 2  # uint8: 300 * 255 * (sqrt2 * 2^14 * g + 1) < 2^31 holds at g = 1, fails at g = 1.5
    tmpl = StreamingBeamformerTemplate(context, 1, 2, 4, 16, A, M, delay_channels=1, out_int8=True, depth=2)
    with tmpl.instantiate() as sb:
        ok = np.ones((M, A), np.float32)
        _lib.call("bf_pipeline_set_gains", sb._h, ok.ctypes.data)
        for bad in (np.full((M, A), 1.5, np.float32), np.full((M, A), 2.5, np.float32)):
            with pytest.raises(_lib.BeamformerError, match="out of range"):
                _lib.call("bf_pipeline_set_gains", sb._h, bad.ctypes.data)
        nan = ok.copy()
        nan[1, 7] = np.nan
        with pytest.raises(_lib.BeamformerError, match="not finite"):
            _lib.call("bf_pipeline_set_gains", sb._h, nan.ctypes.data)
    f32 = StreamingBeamformerTemplate(context, 1, 2, 4, 16, A, M, delay_channels=1, out_int8=True, int8_contract="f32",
                                      depth=2)
    with f32.instantiate() as sb:
        _lib.call("bf_pipeline_set_gains", sb._h, np.full((M, A), 2.5, np.float32).ctypes.data)


def test_stream_errors(context):
    tmpl = StreamingBeamformerTemplate(context, 1, 2, 4, 16, 4, 1, delay_channels=1, depth=2)
    with tmpl.instantiate() as sb:
        s, b = sb.host_frames(1)[0]
        with pytest.raises(Exception, match="no delay model"):
            sb.submit(s, b)
        with pytest.raises(ValueError):
            sb.submit(np.zeros((1, 4, 2, 16, 2, 3), np.uint8), b)
        with pytest.raises(Exception, match="never submitted"):
            sb.wait(5)
        assert isinstance(s, accel.HostArray) and s.ptr
