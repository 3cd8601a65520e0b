"""GPU parity: the HIP operators (through the C ABI) against the goldens and the CPU oracle.

Mirrors the reference's four GPU unit tests (beamformer/unit_test/*_test.py) -- same parameter grid
(test_parameters.py), same input generators, same tolerances -- and adds what they mask:
non-uniform per-(c, m, a) delays, xeng_id > 0, per-beam-varying coefficients, signed samples, odd shapes.
"""
import ctypes

import numpy as np
import pytest

import oracle as O
from dpdk_dc_sand_amd import _lib, accel
from dpdk_dc_sand_amd.beamforming import (CoeffGeneratorTemplate, FusedBeamformerTemplate, MatrixMultiplyTemplate,
                                          OpSequenceTemplate, PreBeamformReorderTemplate, RequantTemplate)
from golden_io import cases, get, voltages
from tolerance import assert_beams_allclose, assert_reference_bar

pytestmark = pytest.mark.gpu

TS = O.TS_MEERKAT
# beamformer/unit_test/test_parameters.py:5-36
N_BATCHES = [3]
N_ANTS = [4, 8, 16, 32, 64, 79, 80, 84, 130, 192, 256, 5, 23, 61, 19]
N_SAMPLES = [256]
N_CHANNELS = [1024, 4096, 32768]
N_BEAMS = [2]
XENG_ID = [0]
SAMPLES_DELAY = [5]
PHASE = [np.pi / 2]


def uniform_delays(C, M, A, samples_delay=5, phase=np.pi / 2):
    """beamform_coeff_test.py:86-112."""
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = np.single(samples_delay * TS)
    d[..., 2] = np.single(phase)
    return d


def random_delays(C, M, A, seed, rates=True):
    rng = np.random.default_rng(seed)
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, (C, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (C, M, A))
    if rates:
        d[..., 1] = rng.uniform(-1e-9, 1e-9, (C, M, A))
        d[..., 3] = rng.uniform(-1.0, 1.0, (C, M, A))
    return d


def i8_path(name):
    """FusedBeamformerTemplate kernel options of an int8 test path: the kernel path, plus "wide-inkernel" = the
    32-beam int8 kernel evaluating its phasors itself (no generated coefficient table)."""
    if name == "wide-inkernel":
        return dict(kernel_path="wide", coeff_table=False)
    return dict(kernel_path=name)


def run(op, queue, inputs, outputs):
    op.ensure_all_bound()
    for name, host in inputs.items():
        op.buffer(name).set(queue, host)
    op()
    return [op.buffer(name).get(queue) for name in outputs]


def assert_beams_close(y, x_real, w):
    """Error bound for the f16 hi/lo MFMA path against an exact (float64) product: each coefficient carries
    <= 2^-22 relative (+ 2^-25 absolute) error and each f32 rounding of the running sum adds <= 2^-24 of it,
    so |err| <= (3e-7 + 1.2e-7 * roundings) * sum_k |x_k w_k| + 1e-6.
    x_real: (..., T, 2A) float; w: (..., 2A, 2M)."""
    exact = np.matmul(x_real.astype(np.float64), w.astype(np.float64))
    mag = np.matmul(np.abs(x_real).astype(np.float64), np.abs(w).astype(np.float64))
    err = np.abs(y.reshape(exact.shape).astype(np.float64) - exact)
    nsteps = 2 * ((w.shape[-2] + 31) // 32)  # f32 roundings of the running sum (hi and lo per k-step)
    bound = (3e-7 + 1.2e-7 * nsteps) * mag + 1e-6
    worst = float((err / bound).max()) if err.size else 0.0
    assert worst <= 1.0, f"beam error exceeds the f32-class bound by {worst:.2f}x"


# ---- pre-beamform reorder (prebeamform_reorder_test.py:33-122) -------------------------------------------
@pytest.mark.parametrize("case", cases("reorder_"))
def test_reorder_golden(context, command_queue, case):
    B, A, C, T = (int(v) for v in get(case, "dims"))
    x = voltages(case, (B, A, C, T, 2, 2))
    op = PreBeamformReorderTemplate(context, A, C, T, B).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inSamples": x}, ["outReordered"])
    np.testing.assert_array_equal(y, O.reorder(x))


@pytest.mark.parametrize("n_batches", N_BATCHES)
@pytest.mark.parametrize("n_ants", N_ANTS)
@pytest.mark.parametrize("n_channels", N_CHANNELS)
@pytest.mark.parametrize("n_samples_per_channel", N_SAMPLES)
def test_prebeamform_reorder_parametrised(context, command_queue, n_batches, n_ants, n_channels,
                                          n_samples_per_channel):
    C = n_channels // n_ants // 4
    op = PreBeamformReorderTemplate(context, n_ants=n_ants, n_channels_per_stream=C,
                                    n_samples_per_channel=n_samples_per_channel,
                                    n_batches=n_batches).instantiate(command_queue)
    x = O.u8_voltages((n_batches, n_ants, C, n_samples_per_channel, 2, 2))
    (y,) = run(op, command_queue, {"inSamples": x}, ["outReordered"])
    np.testing.assert_array_equal(O.reorder(x), y)


@pytest.mark.parametrize("A,C,T", [(1, 1, 16), (3, 7, 48), (257, 2, 64), (64, 3, 1024), (8, 1, 4096)])
def test_reorder_edge_shapes(context, command_queue, A, C, T):
    op = PreBeamformReorderTemplate(context, A, C, T, 2).instantiate(command_queue)
    x = O.u8_voltages((2, A, C, T, 2, 2), seed=A * 1000 + T)
    (y,) = run(op, command_queue, {"inSamples": x}, ["outReordered"])
    np.testing.assert_array_equal(O.reorder(x), y)


# ---- coefficient generator (beamform_coeff_test.py:29-172: bit-exact) ------------------------------------
@pytest.mark.parametrize("case", cases("coeff_"))
def test_coeffs_golden(context, command_queue, case):
    B, P, C, Ctot, A, M, xeng_id = (int(v) for v in get(case, "dims"))
    op = CoeffGeneratorTemplate(context, B, P, C, Ctot, 16, 16, A, M, xeng_id, TS).instantiate(command_queue)
    (w,) = run(op, command_queue, {"delay_vals": get(case, "delays")}, ["outCoeffs"])
    for b in range(B):
        for p in range(P):
            np.testing.assert_array_equal(w[b, p], get(case, "coeffs00"))


@pytest.mark.parametrize("n_batches", N_BATCHES)
@pytest.mark.parametrize("n_ants", N_ANTS)
@pytest.mark.parametrize("n_channels", N_CHANNELS)
@pytest.mark.parametrize("n_beams", N_BEAMS)
@pytest.mark.parametrize("xeng_id", [0, 5])
@pytest.mark.parametrize("kind", ["uniform", "random"])
def test_beamform_coeffs(context, command_queue, n_batches, n_ants, n_channels, n_beams, xeng_id, kind):
    C = n_channels // n_ants // 4
    d = uniform_delays(C, n_beams, n_ants) if kind == "uniform" else random_delays(C, n_beams, n_ants, n_ants)
    op = CoeffGeneratorTemplate(context, n_batches, 2, C, n_channels, 16, 16, n_ants, n_beams, xeng_id,
                                TS).instantiate(command_queue)
    (w,) = run(op, command_queue, {"delay_vals": d}, ["outCoeffs"])
    np.testing.assert_array_equal(O.coeffs(d, n_batches, 2, C, n_channels, n_ants, n_beams, xeng_id), w)


@pytest.mark.parametrize("A,M,C", [(256, 64, 3), (40, 33, 2), (32, 32, 2), (100, 47, 1), (33, 70, 2)])
def test_coeff_gen_tiled_matches_oracle(context, command_queue, A, M, C):
    """The tiled coefficient generator (A >= 32 and M >= 32: 32 x 32 tiles, coalesced model reads through LDS),
    ragged tiles included: bit-exact to the coefficient contract, random per-(c, m, a) delays."""
    d = random_delays(C, M, A, A * M)
    op = CoeffGeneratorTemplate(context, 2, 2, C, 8192, 16, 16, A, M, 3, TS).instantiate(command_queue)
    (w,) = run(op, command_queue, {"delay_vals": d}, ["outCoeffs"])
    np.testing.assert_array_equal(O.coeffs(d, 2, 2, C, 8192, A, M, 3), w)


@pytest.mark.parametrize("A,M", [(5, 3), (64, 16)])
def test_coeff_gen_8_byte_aligned_output(context, command_queue, A, M):
    """bf_coeff_gen requires an 8-byte aligned table: at an address that is 8 but not 16-byte aligned (a C-ABI
    caller's offset pointer) it must not take the 16-byte-store block form, and the table is the contract's."""
    B, P, C, Ctot = 2, 2, 3, 4096
    d = random_delays(C, M, A, 5 * A + M)
    dv = accel.DeviceArray(context, d.shape, np.float32)
    dv.set(command_queue, d)
    n = B * P * C * 2 * A * 2 * M
    buf = accel.DeviceArray(context, (n + 4,), np.float32)
    buf.set(command_queue, np.full(n + 4, 7.0, np.float32))
    _lib.call("bf_coeff_gen", dv.ptr, buf.ptr + 8, B, P, C, Ctot, A, M, 1, TS, command_queue.handle)
    got = buf.get(command_queue)
    np.testing.assert_array_equal(got[2:2 + n].reshape(B, P, C, 2 * A, 2 * M), O.coeffs(d, B, P, C, Ctot, A, M, 1))
    np.testing.assert_array_equal(got[:2], [7.0, 7.0])
    np.testing.assert_array_equal(got[2 + n:], [7.0, 7.0])


def test_coeff_gen_time_matches_oracle(context, command_queue):
    from dpdk_dc_sand_amd import accel
    C, A, M, Ctot, nt = 6, 5, 3, 4096, 4
    d = random_delays(C, M, A, 7)
    dv = accel.DeviceArray(context, d.shape, np.float32)
    dv.set(command_queue, d)
    out = accel.DeviceArray(context, (nt, C, A, M, 2), np.float32)
    out16 = accel.DeviceArray(context, (nt, C, A, M, 2), np.float16)
    t0, step = 1e-3, 8192 * TS
    _lib.call("bf_coeff_gen_time", dv.ptr, C, out.ptr, 0, nt, C, Ctot, A, M, 2, TS, t0, step, command_queue.handle)
    _lib.call("bf_coeff_gen_time", dv.ptr, C, out16.ptr, 1, nt, C, Ctot, A, M, 2, TS, t0, step, command_queue.handle)
    got, got16 = out.get(command_queue), out16.get(command_queue)
    for t in range(nt):
        cos, sin = O.coeffs_at(d, C, Ctot, A, M, 2, TS, t0 + t * step)
        np.testing.assert_array_equal(got[t, ..., 0], cos.transpose(0, 2, 1))
        np.testing.assert_array_equal(got[t, ..., 1], sin.transpose(0, 2, 1))
        np.testing.assert_array_equal(got16[t, ..., 0], cos.transpose(0, 2, 1).astype(np.float16))
        np.testing.assert_array_equal(got16[t, ..., 1], sin.transpose(0, 2, 1).astype(np.float16))


@pytest.mark.parametrize("case", cases("rates_"))
def test_coeff_gen_time_reference_golden(context, command_queue, case):
    """dt != 0 pinned by the reference itself (G5, tests/golden/make_golden.py): delay models WITH rates whose
    advanced delay and phase are exact float32 numbers at every batch time, so the reference's cpu_coeffs on the
    advanced model is the time extension evaluated exactly.  The time generator's phasors equal it bit for bit."""
    A, M, C, Ctot, xeng_id, nb = (int(v) for v in get(case, "dims"))
    t0, bdt = (float(v) for v in get(case, "times"))
    d = get(case, "delays")
    w = get(case, "coeffs")  # (nb, C, 2A, 2M): W[2a][2m] = cos, W[2a][2m+1] = sin
    dv = accel.DeviceArray(context, d.shape, np.float32)
    dv.set(command_queue, d)
    out = accel.DeviceArray(context, (nb, C, A, M, 2), np.float32)
    _lib.call("bf_coeff_gen_time", dv.ptr, 1, out.ptr, 0, nb, C, Ctot, A, M, xeng_id, TS, t0, bdt,
              command_queue.handle)
    got = out.get(command_queue)
    np.testing.assert_array_equal(got[..., 0], w[:, :, 0::2, 0::2])
    np.testing.assert_array_equal(got[..., 1], w[:, :, 0::2, 1::2])


@pytest.mark.parametrize("case", cases("rates_"))
def test_fused_time_extension_reference_golden(context, command_queue, fused_path, case):
    """The fused operator at dt != 0 (exact coefficients, per-batch regeneration from a model with rates) is the
    reference's multiply applied to the reference's own per-batch tables (G5): identical bits to MatrixMultiply fed
    the golden tables, on every fused kernel path."""
    A, M, C, Ctot, xeng_id, B = (int(v) for v in get(case, "dims"))
    t0, bdt = (float(v) for v in get(case, "times"))
    T = 256
    d = get(case, "delays")
    w = np.ascontiguousarray(np.broadcast_to(get(case, "coeffs")[:, None], (B, 2, C, 2 * A, 2 * M)))
    raw = O.u8_voltages((B, A, C, T, 2, 2), seed=A + M)
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng_id, sample_period=TS, delay_channels=1,
                                 t0=t0, batch_dt=bdt, exact_coeffs=True,
                                 kernel_path=fused_path).instantiate(command_queue)
    (y_fu,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    mm = MatrixMultiplyTemplate(context, A, C, T, M, B).instantiate(command_queue)
    (y_mm,) = run(mm, command_queue, {"inData": O.reorder(raw), "inCoeffs": w}, ["outData"])
    np.testing.assert_array_equal(y_fu, y_mm)
    assert_beams_allclose(y_fu, O.complex_mult(O.reorder(raw), w), O.reorder(raw), w)


@pytest.mark.parametrize("case", cases("rates_"))
@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("i8_kernel", ["auto", "item", "generic", "wide", "wide-inkernel"])
def test_fused_int8_time_extension_reference_golden(context, command_queue, i8_kernel, signed, case):
    """The int8 (requantised) beams at dt != 0 from the reference's own per-batch tables (G5): W = rne(2^14 w) of the
    golden float32 coefficients, exact integer products, one rounding to int8 -- bit for bit on every int8 kernel
    path, the in-kernel phasor path included."""
    A, M, C, Ctot, xeng_id, B = (int(v) for v in get(case, "dims"))
    t0, bdt = (float(v) for v in get(case, "times"))
    T, scale = 256, 1.0 / 64
    d = get(case, "delays")
    W = O.quantise_coeffs(np.broadcast_to(get(case, "coeffs")[:, None], (B, 2, C, 2 * A, 2 * M)))
    rng = np.random.default_rng(A * 5 + M)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    op = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng_id, sample_period=TS, delay_channels=1,
                                 sample_signed=signed, out_int8=True, out_scale=scale, t0=t0, batch_dt=bdt,
                                 **i8_path(i8_kernel)).instantiate(command_queue)
    (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    xr = O.reorder(raw)
    X = (xr.view(np.int8) if signed else xr).astype(np.int64).reshape(B, 2, C, T, 2 * A)
    s = np.float32(np.float32(scale) * np.float32(2.0 ** -14))
    ref = np.clip(np.rint(np.matmul(X, W).astype(np.float32) * s), -127, 127).astype(np.int8)
    np.testing.assert_array_equal(q, ref.reshape(q.shape))


@pytest.mark.parametrize("shape", [(256, 64, 64, 16), (3, 6, 5, 3), (4, 7, 5, 3)])
def test_coeff_gen_time_study_matches_study_golden(context, command_queue, shape):
    """The C++ study's own time-dependent convention (bf_coeff_gen_time_study, BeamformerKernels.cu:155-170) against
    its harness's golden (BeamformerCoefficientTest.cu:294-337, restated in oracle.study_coeffs_time) on the
    harness's delay ramp (simulate_input, :185-196) with nonzero delay and phase rates, at the study's default shape
    (256 times x 64 channels x 64 antennas x 16 beams) and a ragged one.  Bar: the harness's own 1e-4 absolute
    tolerance on every float (runBeamformerTests.cpp:30, verify_output :348-357); the half2 output (which the
    harness does not check, :281-287) within half a float16 ulp of 1 plus the float bar."""
    from dpdk_dc_sand_amd import accel
    NT, C, A, M = shape
    d = O.study_delay_ramp(A, M)
    dv = accel.DeviceArray(context, d.shape, np.float32)
    dv.set(command_queue, d)
    out = accel.DeviceArray(context, (NT, C, A, M, 2), np.float32)
    out16 = accel.DeviceArray(context, (NT, C, A, M, 2), np.float16)
    _lib.call("bf_coeff_gen_time_study", dv.ptr, out.ptr, 0, NT, C, A, M, ctypes.c_float(1e-7), 8192,
              command_queue.handle)
    _lib.call("bf_coeff_gen_time_study", dv.ptr, out16.ptr, 1, NT, C, A, M, ctypes.c_float(1e-7), 8192,
              command_queue.handle)
    w = O.study_coeffs_time(d, NT, C, A, M)
    ref = np.stack([w.real, w.imag], axis=-1)
    got, got16 = out.get(command_queue), out16.get(command_queue).astype(np.float32)
    assert np.abs(got - ref).max() <= 1e-4
    assert np.abs(got16 - ref).max() <= 2 ** -11 + 1e-4
    # the rates matter at the study's shape: its last time's phasors are far from its first's
    if NT >= 256:
        assert np.abs(ref[-1] - ref[0]).max() > 0.5


@pytest.mark.parametrize("shape,inputs", [((64, 256, 64, 16), "harness"), ((5, 48, 37, 20), "random")])
def test_study_single_channel_beamformer_matches_study_golden(context, command_queue, shape, inputs):
    """The C++ study's fused kernel in its own semantics (bf_beamform_study_single_channel; replaces
    calculate_beamweights_and_beamform_single_channel, BeamformerKernels.cu:192-367) against its harness's golden
    (BeamformerCoefficientTest.cu:356-400, restated in oracle.study_beams_single_channel): y_re = sum_a cos x_re,
    y_im = sum_a sin x_im per (channel, time, beam), the study's time-dependent phasor per sample.  At the study's
    default shape on the harness's own inputs (simulate_input: delay ramp, x[i] = (int8) i), and at a ragged shape
    (odd channel count, more beams than a workgroup's 16 beam slots, random int8 samples and delay model with rates).
    Bars: the harness's own, 1e-1 absolute on every beam (runBeamformerTests.cpp:14); and a float32 one, 2e-5 of
    sum_a |x| -- the phasors' argument carries the study's float32 rounding (|rot| up to ~60 rad: ulp 4e-6) and the
    kernel's dt = t Ts fft against the golden's truncated nanoseconds."""
    C, T, A, M = shape
    if inputs == "harness":
        d = O.study_delay_ramp(A, M)
        x = np.arange(C * T * A * 2, dtype=np.int64).astype(np.int8).reshape(C, T // 16, A, 16, 2)
    else:
        rng = np.random.default_rng(C * T + A)
        d = np.zeros((M * A, 4), np.float32)
        d[:, 0] = rng.uniform(0, 1e-7 / 3, M * A)
        d[:, 1] = rng.uniform(-3e-6, 3e-6, M * A)
        d[:, 2] = rng.uniform(-np.pi, np.pi, M * A)
        d[:, 3] = rng.uniform(-1e-5, 1e-5, M * A)
        x = rng.integers(-128, 128, (C, T // 16, A, 16, 2), dtype=np.int64).astype(np.int8)
    dv = accel.DeviceArray(context, d.shape, np.float32)
    dv.set(command_queue, d)
    xv = accel.DeviceArray(context, x.shape, np.int8)
    xv.set(command_queue, x)
    out = accel.DeviceArray(context, (C, T // 16, M, 16, 2), np.float32)
    _lib.call("bf_beamform_study_single_channel", dv.ptr, xv.ptr, out.ptr, C, T, A, M, ctypes.c_float(1e-7), 8192,
              command_queue.handle)
    y = out.get(command_queue)
    ref = O.study_beams_single_channel(d, x, C, T, A, M)
    err = np.abs(y.astype(np.float64) - ref)
    assert err.max() <= 1e-1  # the harness's tolerance for this kernel (runBeamformerTests.cpp:14)
    mag = np.abs(x.astype(np.float64)).sum(axis=2).transpose(0, 1, 2, 3)[:, :, None]  # (C, T/16, 1, 16, 2)
    assert (err <= 2e-5 * mag + 1e-6).all(), float((err / (2e-5 * mag + 1e-6)).max())
    assert np.abs(ref).max() > 100  # the beams are far from zero


# ---- beamform multiply (beamform_mult_kernel_test.py:119-269: rtol = atol = 1e-4) -------------------------
@pytest.mark.parametrize("case", cases("mult_"))
def test_matrix_multiply_golden(context, command_queue, case):
    B, A, M, Ctot, T, C = (int(v) for v in get(case, "dims"))
    w = O.coeffs(get(case, "delays"), B, 2, C, Ctot, A, M, 0)
    x = voltages(case, (B, 2, C, T // 16, 16, A, 2))
    op = MatrixMultiplyTemplate(context, A, C, T, M, B).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    # the reference's own bar on the reference's own (uniform-delay) inputs and outputs: beamform_mult_kernel_test.py:
    # 267-269 -- every element, no exceptions
    np.testing.assert_allclose(y, get(case, "output"), rtol=1e-4, atol=1e-4)
    assert_beams_allclose(y, get(case, "output"), x, w)


@pytest.mark.combinations(
    "n_batches, n_ants, n_channels, n_samples_per_channel, n_beams, xeng_id, samples_delay, phase",
    N_BATCHES, N_ANTS, N_CHANNELS, N_SAMPLES, N_BEAMS, XENG_ID, SAMPLES_DELAY, PHASE)
def test_beamform(context, command_queue, n_batches, n_ants, n_channels, n_samples_per_channel, n_beams, xeng_id,
                  samples_delay, phase):
    """beamform_mult_kernel_test.py:119-269: coeff generator + multiply, reference tolerance."""
    C = n_channels // n_ants // 4
    d = uniform_delays(C, n_beams, n_ants, samples_delay, phase)
    cg = CoeffGeneratorTemplate(context, n_batches, 2, C, n_channels, 16, 16, n_ants, n_beams, xeng_id,
                                TS).instantiate(command_queue)
    (w,) = run(cg, command_queue, {"delay_vals": d}, ["outCoeffs"])
    x = O.u8_voltages((n_batches, 2, C, n_samples_per_channel // 16, 16, n_ants, 2))
    mm = MatrixMultiplyTemplate(context, n_ants, C, n_samples_per_channel, n_beams, n_batches).instantiate(
        command_queue)
    (y,) = run(mm, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    w_ref = O.coeffs(d, n_batches, 2, C, n_channels, n_ants, n_beams, xeng_id)
    expected = O.complex_mult(x, w_ref)
    n_miss = assert_reference_bar(y, expected, x, w_ref)  # beamform_mult_kernel_test.py:267-269, see tolerance.py
    if n_miss:
        print(f"{n_miss}/{y.size} beams miss rtol=atol=1e-4 vs the f32 oracle; each is within the bar of the exact "
              "product or closer to it than the f32 oracle")
    assert_beams_allclose(y, expected, x, w_ref)


@pytest.mark.parametrize("A,M,C,T,signed", [
    (64, 16, 4, 256, False), (64, 16, 4, 256, True), (19, 3, 5, 64, False), (5, 1, 3, 32, True),
    (130, 9, 2, 48, False), (256, 64, 1, 32, False), (61, 8, 3, 16, True), (2, 40, 2, 16, False),
    (64, 4, 2, 16, True), (96, 16, 2, 48, False)])
def test_matrix_multiply_random_tables(context, command_queue, A, M, C, T, signed):
    """Per-beam-varying coefficients (which the reference CPU oracle gets wrong) and int8 samples."""
    B = 2
    rng = np.random.default_rng(A * 7 + M)
    x = rng.integers(0, 256, (B, 2, C, T // 16, 16, A, 2), dtype=np.uint8)
    if signed:
        x = x.view(np.int8)
    d = random_delays(C, M, A, A + M)
    w = O.coeffs(d, B, 2, C, 8192, A, M, 1)
    w[1] *= rng.uniform(0.25, 2.0, w[1].shape).astype(np.float32)  # arbitrary table, not just phasors
    op = MatrixMultiplyTemplate(context, A, C, T, M, B, sample_signed=signed).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    assert_beams_close(y, x.astype(np.float32).reshape(B, 2, C, T, 2 * A), w)
    assert_beams_allclose(y, O.complex_mult(x, w, signed=signed), x, w, signed=signed)


@pytest.mark.parametrize("T,signed", [(32, True), (128, False)])
def test_matrix_multiply_persistent_equals_ring(context, command_queue, T, signed):
    """256 antennas in two-workgroup slabs with >= 8 (b, p, c) items take the persistent table kernel (the next
    slab loaded under the current item, the ring's last turn prefetching the next item's rows; 640 slab items here,
    more than one per workgroup, xcd padding items skipped).  Its per-item MFMA sequence is the ring kernel's, which
    one-channel calls (4 items) still take: the results must be identical bits, and within tolerance of the oracle.
    T = 32 leaves two of the four waves without row groups; T = 128 gives each wave one row-group pair (T = 256
    takes the output-stationary kernel, tested below)."""
    B, A, M, C = 2, 256, 64, 40
    rng = np.random.default_rng(T + 5)
    x = rng.integers(0, 256, (B, 2, C, T // 16, 16, A, 2), dtype=np.uint8)
    if signed:
        x = x.view(np.int8)
    w = rng.uniform(-1.0, 1.0, (B, 2, C, 2 * A, 2 * M)).astype(np.float32)
    op = MatrixMultiplyTemplate(context, A, C, T, M, B, sample_signed=signed).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    one = MatrixMultiplyTemplate(context, A, 1, T, M, B, sample_signed=signed).instantiate(command_queue)
    for c in (0, 1, 17, C - 1):
        (yc,) = run(one, command_queue, {"inData": np.ascontiguousarray(x[:, :, c:c + 1]),
                                          "inCoeffs": np.ascontiguousarray(w[:, :, c:c + 1])}, ["outData"])
        np.testing.assert_array_equal(y[:, :, c:c + 1], yc)
    sel = [0, 9, 23, C - 1]
    xs, ws = np.ascontiguousarray(x[:, :, sel]), np.ascontiguousarray(w[:, :, sel])
    assert_beams_allclose(y[:, :, sel], O.complex_mult(xs, ws, signed=signed), xs, ws, signed=signed)


@pytest.mark.parametrize("B,C,M", [(1, 5, 16), (1, 7, 9), (3, 3, 12)])
def test_matrix_multiply_persistent_single_slab_any_item_count(context, command_queue, B, C, M):
    """256 antennas with 9..16 beams (one slab, no XCD item order) and a (b, p, c) item count that is not a multiple
    of 8 (10, 14, 18 items): the persistent table kernel's grid needs no multiple of 8 there (such calls
    were refused with BF_ERR_ARG)."""
    A, T = 256, 64
    rng = np.random.default_rng(B * 100 + C)
    x = rng.integers(0, 256, (B, 2, C, T // 16, 16, A, 2), dtype=np.uint8)
    w = rng.uniform(-1.0, 1.0, (B, 2, C, 2 * A, 2 * M)).astype(np.float32)
    op = MatrixMultiplyTemplate(context, A, C, T, M, B).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    assert_beams_allclose(y, O.complex_mult(x, w), x, w)


@pytest.mark.parametrize("A,C,signed", [(256, 6, False), (256, 3, True), (128, 4, False), (64, 5, True)])
def test_matrix_multiply_output_stationary_equals_slab_kernels(context, command_queue, A, C, signed):
    """Config 4's item shape (2M = 128 columns, T = 256, A % 64 == 0) takes the output-stationary table kernel
    (whole items per workgroup, K streamed through LDS).  A table pointer that is only 4-byte aligned keeps the
    same call on the slab kernels (ring / persistent): per output both run the same MFMA sequence, so the bits
    must be equal -- and within tolerance of the oracle."""
    B, M, T = 2, 64, 256
    rng = np.random.default_rng(A + C)
    x = rng.integers(0, 256, (B, 2, C, T // 16, 16, A, 2), dtype=np.uint8)
    if signed:
        x = x.view(np.int8)
    w = rng.uniform(-1.0, 1.0, (B, 2, C, 2 * A, 2 * M)).astype(np.float32)
    op = MatrixMultiplyTemplate(context, A, C, T, M, B, sample_signed=signed).instantiate(command_queue)
    (y,) = run(op, command_queue, {"inData": x, "inCoeffs": w}, ["outData"])
    xd = accel.DeviceArray(context, x.shape, x.dtype)
    xd.set(command_queue, x)
    wd = accel.DeviceArray(context, (w.size + 4,), np.float32)
    wd.set(command_queue, np.concatenate([np.zeros(1, np.float32), w.reshape(-1), np.zeros(3, np.float32)]))
    yd = accel.DeviceArray(context, y.shape, np.float32)
    _lib.call("bf_beamform", xd.ptr, wd.ptr + 4, yd.ptr, B, 2, C, T // 16, A, M, int(signed), command_queue.handle)
    np.testing.assert_array_equal(y, yd.get(command_queue))
    sel = [0, C - 1]
    xs, ws = np.ascontiguousarray(x[:, :, sel]), np.ascontiguousarray(w[:, :, sel])
    assert_beams_allclose(y[:, :, sel], O.complex_mult(xs, ws, signed=signed), xs, ws, signed=signed)


# ---- full sequence (beamform_op_sequence_test.py:37-200) ---------------------------------------------------
def test_op_sequence_golden(context, command_queue):
    B, A, M, Ctot, T, C = (int(v) for v in get("opseq_cfg1", "dims"))
    raw = voltages("opseq_cfg1", (B, A, C, T, 2, 2))
    tmpl = OpSequenceTemplate(context, B, 2, C, Ctot, T // 16, 16, A, M, 0, TS, T)
    op = tmpl.instantiate(command_queue)
    op.ensure_all_bound()
    op.beamform_coeff.buffer("delay_vals").set(command_queue, get("opseq_cfg1", "delays"))
    op.prebeamform_reorder.buffer("inSamples").set(command_queue, raw)
    op()
    y = op.beamform_mult.buffer("outData").get(command_queue)
    d = get("opseq_cfg1", "delays")
    np.testing.assert_allclose(y, get("opseq_cfg1", "output"), rtol=1e-4, atol=1e-4)  # beamform_op_sequence_test.py:198-199
    assert_beams_allclose(y, get("opseq_cfg1", "output"), O.reorder(raw), O.coeffs(d, B, 2, C, Ctot, A, M, 0))


@pytest.mark.parametrize("n_batches", N_BATCHES)
@pytest.mark.parametrize("n_ants", N_ANTS)
@pytest.mark.parametrize("n_channels", N_CHANNELS)
@pytest.mark.parametrize("n_beams", N_BEAMS)
def test_beamform_op_sequence(context, command_queue, n_batches, n_ants, n_channels, n_beams):
    C = n_channels // n_ants // 4
    T = 256
    d = uniform_delays(C, n_beams, n_ants)
    op = OpSequenceTemplate(context, n_batches, 2, C, n_channels, T // 16, 16, n_ants, n_beams, 0, TS,
                            T).instantiate(command_queue)
    op.ensure_all_bound()
    raw = O.u8_voltages((n_batches, n_ants, C, T, 2, 2))
    op.beamform_coeff.buffer("delay_vals").set(command_queue, d)
    op.prebeamform_reorder.buffer("inSamples").set(command_queue, raw)
    op()
    y = op.beamform_mult.buffer("outData").get(command_queue)
    w = O.coeffs(d, n_batches, 2, C, n_channels, n_ants, n_beams, 0)
    expected = O.op_sequence(raw, d, C, n_channels, n_ants, n_beams)
    assert_reference_bar(y, expected, O.reorder(raw), w)  # beamform_op_sequence_test.py:198-199
    assert_beams_allclose(y, expected, O.reorder(raw), w)


# ---- fused one-pass operator --------------------------------------------------------------------------------
def test_fused_equals_op_sequence_bitwise(context, command_queue, fused_path):
    """Same coefficients (float64 phase), same fragment order, same accumulation: identical bits."""
    B, A, M, C, Ctot, T = 2, 64, 16, 8, 4096, 256
    d = random_delays(C, M, A, 11, rates=False)
    raw = O.u8_voltages((B, A, C, T, 2, 2), seed=3)
    seq = OpSequenceTemplate(context, B, 2, C, Ctot, T // 16, 16, A, M, 2, TS, T).instantiate(command_queue)
    seq.ensure_all_bound()
    seq.beamform_coeff.buffer("delay_vals").set(command_queue, d)
    seq.prebeamform_reorder.buffer("inSamples").set(command_queue, raw)
    seq()
    y_seq = seq.beamform_mult.buffer("outData").get(command_queue)
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=2, sample_period=TS,
                                 exact_coeffs=True, kernel_path=fused_path).instantiate(command_queue)
    (y_fu,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(y_fu, y_seq)
    assert_beams_allclose(y_fu, O.op_sequence(raw, d, C, Ctot, A, M, xeng_id=2), O.reorder(raw),
                          O.coeffs(d, B, 2, C, Ctot, A, M, 2))


@pytest.fixture(params=["auto", "item", "generic", "wide"])
def fused_path(request):
    """Run a fused test through each kernel (FusedBeamformerTemplate kernel_path = BF_FUSED_PATH_* flags): the
    automatic choice, the single-item kernel (A <= 64, T <= 256), the generic kernel, and the wide kernel (many antennas x beams) with 32- and 16-beam slabs.  A path that does not fit a shape
    falls through to one that does."""
    return request.param


@pytest.mark.parametrize("A,M,C,T,B,dch,signed", [
    (64, 16, 4, 256, 3, 1, True), (64, 1, 4, 256, 2, 4, False), (4, 1, 64, 1024, 1, 64, False),
    (19, 2, 13, 256, 3, 1, False), (5, 3, 7, 48, 2, 7, True), (130, 9, 2, 64, 2, 1, False),
    (256, 64, 1, 32, 1, 1, True), (80, 2, 3, 16, 3, 3, False), (64, 16, 700, 256, 2, 1, False),
    (32, 24, 9, 128, 5, 9, True),
    # the wide kernel's 32-beam slabs with a pulled-back last k-step (A % 16 != 0), a partial last slab, a partial
    # sample chunk and per-channel models: the phasor pairs' uniform/lane addressing at every edge it has
    (200, 40, 3, 96, 2, 3, True), (72, 33, 2, 64, 1, 1, False)])
@pytest.mark.parametrize("exact", [False, True])
def test_fused_matches_oracle(context, command_queue, fused_path, exact, A, M, C, T, B, dch, signed):
    Ctot, xeng = 8192, 3
    d = random_delays(dch, M, A, A * 31 + M)
    rng = np.random.default_rng(A + M + C)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    t0, bdt = 2.5e-3, 256 * 8192 * TS
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, sample_period=TS, delay_channels=dch,
                                 sample_signed=signed, t0=t0, batch_dt=bdt, exact_coeffs=exact,
                                 kernel_path=fused_path).instantiate(command_queue)
    (y,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    ref = O.fused_beamform(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, signed=signed)
    w = O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, t0=t0, batch_dt=bdt)
    assert_beams_allclose(y, ref, O.reorder(raw), w, signed=signed)


@pytest.mark.parametrize("A,M,C,T,B,dch,signed", [
    (64, 16, 4, 256, 2, 1, True), (64, 16, 3, 256, 2, 3, False), (64, 1, 5, 256, 2, 1, True),
    (19, 3, 7, 48, 2, 7, False), (130, 9, 2, 64, 2, 1, True), (256, 64, 1, 32, 1, 1, False),
    (4, 1, 16, 1024, 1, 16, True), (80, 24, 3, 16, 3, 1, True), (32, 8, 4, 64, 2, 1, False),
    (48, 12, 2, 128, 2, 1, False), (33, 5, 3, 80, 2, 3, True), (16, 8, 3, 48, 2, 1, True),
    (64, 16, 2, 112, 1, 1, False), (40, 32, 2, 64, 1, 2, True), (600, 5, 1, 32, 1, 1, True)])
@pytest.mark.parametrize("i8_kernel", ["auto", "item", "generic", "wide", "wide-inkernel"])
def test_fused_int8_bit_exact(context, command_queue, i8_kernel, A, M, C, T, B, dch, signed):
    """int8 (requantised) beams: the integer MFMA path reproduces the oracle's integer contract bit for bit, on the
    item kernel (A <= 64, T <= 256; others fall through to generic) and the generic kernel (any A, T)."""
    Ctot, xeng, t0, bdt = 4096, 1, 1e-3, 256 * 8192 * TS
    d = random_delays(dch, M, A, A * 7 + M)
    rng = np.random.default_rng(A * 3 + C)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    for scale in (1.0 / 64, 1.0 / 16):
        op = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=dch, sample_signed=signed,
                                     out_int8=True, out_scale=scale, t0=t0, batch_dt=bdt,
                                     **i8_path(i8_kernel)).instantiate(command_queue)
        (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
        ref = O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, scale=scale, signed=signed)
        assert q.dtype == np.int8
        np.testing.assert_array_equal(q, ref)
        assert np.abs(ref.astype(int)).max() >= 4  # not a trivially zero case


@pytest.mark.parametrize("A,M,C,T", [(64, 16, 4, 256), (256, 64, 8, 256), (19, 3, 5, 48)])
@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("i8_kernel", ["auto", "item", "generic", "wide", "wide-inkernel", "f32"])
def test_fused_int8_requant_double_rounding(context, command_queue, i8_kernel, A, M, C, T, signed):
    """The requantisation's two roundings, RN(float32(y) * s) and then rne, at a scale that is not a power of two.
    Zero delays and phases make every Q14 coefficient (16384, 0), and only antenna 0 carries voltages, so
    y = 16384 x and the requantiser sees x * scale: at scale = float32(1/6) that product rounds onto a half-integer
    for 22 of the 256 byte values x, where one fused multiply-add (a single rounding) would give the other integer.
    Every int8 path must give the contract's value (oracle.fused_beamform_int8; oracle.requantise of the float beams
    for the float path)."""
    Ctot, scale = 4096, float(np.float32(1 / 6))
    rng = np.random.default_rng(A + T)
    raw = np.zeros((1, A, C, T, 2, 2), np.uint8)
    raw[:, 0] = rng.integers(0, 256, (1, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    d = np.zeros((1, M, A, 4), np.float32)
    ref = O.fused_beamform_int8(raw, d, Ctot, scale=scale, signed=signed)
    # the test has teeth: a single-rounding requantiser differs from the contract on this input
    y = 16384.0 * (raw[0, 0].view(np.int8) if signed else raw[0, 0]).astype(np.float64)
    s = np.float32(np.float32(scale) * np.float32(2.0 ** -14))
    once = np.clip(np.rint(y.astype(np.float32).astype(np.float64) * np.float64(s)), -127, 127)
    twice = np.clip(np.rint(y.astype(np.float32) * s), -127, 127)
    assert np.count_nonzero(once != twice) > 0
    kw = dict(int8_contract="f32") if i8_kernel == "f32" else i8_path(i8_kernel)
    op = FusedBeamformerTemplate(context, 1, C, Ctot, T, A, M, delay_channels=1, sample_signed=signed, out_int8=True,
                                 out_scale=scale, **kw).instantiate(command_queue)
    (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(q, ref)


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("A,T", [(64, 256), (61, 256), (64, 144), (19, 64)])
def test_fused_int8_one_two_beams(context, command_queue, A, T, M, signed):
    """Config-2-like shapes (one or two beams): the item kernels' packed row stores -- int8 bit-exact, f32 within the
    tolerance."""
    B, C, Ctot, xeng, bdt = 2, 3, 4096, 2, 256 * 8192 * TS
    d = random_delays(1, M, A, 11 * A + M)
    rng = np.random.default_rng(5 * A + T + M)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    op = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=signed,
                                 out_int8=True, out_scale=1 / 32, batch_dt=bdt).instantiate(command_queue)
    (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(q, O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, batch_dt=bdt, scale=1 / 32,
                                                           signed=signed))
    assert np.abs(q.astype(int)).max() >= 4
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=signed,
                                 batch_dt=bdt).instantiate(command_queue)
    (y,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    assert_beams_allclose(y, O.fused_beamform(raw, d, Ctot, xeng_id=xeng, batch_dt=bdt, signed=signed),
                          O.reorder(raw), O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, batch_dt=bdt), signed=signed)


@pytest.mark.parametrize("order", ["xcd", "channel"])
@pytest.mark.parametrize("B,C,M", [(2, 16, 16), (3, 24, 8), (1, 8, 16), (2, 40, 12)])
def test_item_kernels_workgroup_order(context, command_queue, order, B, C, M):
    """The item kernels' XCD-range workgroup order (C % 8 == 0, >= 8 beams; item_coords) covers every (batch,
    channel) exactly once: int8 bit-exact and f32 within the tolerance, in both orders."""
    A, T, Ctot, xeng, bdt = 64, 256, 8 * C, 1, 256 * 8192 * TS
    d = random_delays(1, M, A, B * C + M)
    rng = np.random.default_rng(C * 3 + M)
    raw = rng.integers(-128, 128, (B, A, C, T, 2, 2), dtype=np.int8)
    q8 = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=True,
                                 out_int8=True, out_scale=1 / 64, batch_dt=bdt,
                                 workgroup_order=order).instantiate(command_queue)
    (q,) = run(q8, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(q, O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, batch_dt=bdt, scale=1 / 64,
                                                           signed=True))
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=True,
                                 batch_dt=bdt, workgroup_order=order).instantiate(command_queue)
    (y,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    assert_beams_allclose(y, O.fused_beamform(raw, d, Ctot, xeng_id=xeng, batch_dt=bdt, signed=True), O.reorder(raw),
                          O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, batch_dt=bdt), signed=True)


@pytest.mark.parametrize("A,M,T", [(64, 16, 256), (64, 8, 256), (40, 32, 64), (64, 16, 48), (33, 24, 128),
                                   (64, 1, 256)])
def test_fused_int8_float_path_is_requantised_f32(context, command_queue, A, M, T):
    """int8_contract='f32' (BF_FUSED_INT8_VIA_F32): float beams requantised in-kernel == bf_requant(float beams).
    Shapes: whole-row slabs (1 KiB store blocks), multi-slab rows, partial waves (T < 256), partial tiles, 1 beam."""
    B, C, Ctot = 2, 4, 4096
    d = random_delays(1, M, A, 9)
    raw = O.u8_voltages((B, A, C, T, 2, 2), seed=9).view(np.int8)
    scale = 1.0 / 64
    f32 = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, delay_channels=1, sample_signed=True).instantiate(
        command_queue)
    (y,) = run(f32, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    i8 = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, delay_channels=1, sample_signed=True, out_int8=True,
                                 out_scale=scale, int8_contract="f32").instantiate(command_queue)
    (q,) = run(i8, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(q, O.requantise(y, scale))
    rq = RequantTemplate(context, y.shape, scale).instantiate(command_queue)
    (q2,) = run(rq, command_queue, {"inData": y}, ["outData"])
    np.testing.assert_array_equal(q2, q)


# ---- errors --------------------------------------------------------------------------------------------------
def test_errors_raise(context, command_queue):
    with pytest.raises(ValueError):
        PreBeamformReorderTemplate(context, 4, 4, 100, 1)
    from dpdk_dc_sand_amd import accel
    a = accel.DeviceArray(context, (64,), np.uint8)
    with pytest.raises(_lib.BeamformerError, match="multiple of 16"):
        _lib.call("bf_reorder", a.ptr, a.ptr, 1, 1, 1, 17, command_queue.handle)
    op = MatrixMultiplyTemplate(context, 4, 2, 32, 1, 1).instantiate(command_queue)
    with pytest.raises(ValueError):
        op.bind(inData=accel.DeviceArray(context, (3,), np.uint8))


@pytest.mark.parametrize("A,M,C,T,B,dch,signed", [
    (64, 16, 3, 256, 2, 1, True), (19, 3, 4, 48, 2, 4, False), (130, 9, 2, 64, 1, 1, True), (33, 8, 2, 64, 2, 2, False),
    # the wide kernel's 32-beam slabs with weights: config 4's item shape, and a pulled-back step + partial slab
    (256, 64, 1, 32, 1, 1, False), (200, 40, 2, 96, 1, 2, True)])
@pytest.mark.parametrize("exact", [False, True])
def test_fused_beam_weights(context, command_queue, fused_path, exact, A, M, C, T, B, dch, signed):
    """?beam-weights (corr3_servlet.py:140-153): per-(beam, input) weights folded into the phasors, set through the
    request-shaped API, against the oracle's weighted tables (float path: f32-class tolerance)."""
    Ctot, xeng, t0, bdt = 4096, 1, 1e-3, 256 * 8192 * TS
    d = random_delays(dch, M, A, A + 7 * M)
    rng = np.random.default_rng(A * 5 + M)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=dch, sample_signed=signed,
                                 t0=t0, batch_dt=bdt, exact_coeffs=exact, beam_weights=True,
                                 kernel_path=fused_path).instantiate(command_queue)
    g = rng.uniform(-1.5, 1.5, (M, A)).astype(np.float32)
    g[0, : A // 2] = 0.0  # switched-off inputs
    for m in range(M):
        fu.set_beam_weights(m, *g[m])
    (y,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    ref = O.fused_beamform(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, signed=signed, gains=g)
    w = O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, t0=t0, batch_dt=bdt, gains=g)
    assert_beams_allclose(y, ref, O.reorder(raw), w, signed=signed)
    fu.set_beam_weights(M - 1, *np.ones(A))  # a later request takes effect on the next launch
    g[M - 1] = 1.0
    fu()
    y2 = fu.buffer("outData").get(command_queue)
    ref2 = O.fused_beamform(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, signed=signed, gains=g)
    w2 = O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, t0=t0, batch_dt=bdt, gains=g)
    assert_beams_allclose(y2, ref2, O.reorder(raw), w2, signed=signed)


@pytest.mark.parametrize("A,M,C,T,B,dch,signed", [
    (64, 16, 3, 256, 2, 1, True), (64, 16, 2, 256, 2, 1, False), (19, 3, 4, 48, 2, 4, False),
    (130, 9, 2, 64, 1, 1, True),
    # the 32-beam int8 kernels (Q14 table generator with gains / in-kernel phasors) at 256 antennas x 64 beams, and a
    # pulled-back antenna step with a partial slab and per-channel models
    (256, 64, 2, 64, 1, 1, True), (200, 40, 2, 96, 1, 2, True)])
@pytest.mark.parametrize("i8_kernel", ["auto", "item", "generic", "wide", "wide-inkernel"])
def test_fused_int8_beam_weights_bit_exact(context, command_queue, i8_kernel, A, M, C, T, B, dch, signed):
    """Weighted int8 beams: Q14 limbs of the weighted float32 coefficients, bit-exact to the integer contract."""
    Ctot, xeng, t0, bdt = 4096, 2, 1e-3, 256 * 8192 * TS
    d = random_delays(dch, M, A, A * 3 + M)
    rng = np.random.default_rng(A * 11 + C)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    g = rng.uniform(-1.9, 1.9, (M, A)).astype(np.float32)
    op = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=dch, sample_signed=signed,
                                 out_int8=True, out_scale=1 / 64, t0=t0, batch_dt=bdt,
                                 beam_weights=True, **i8_path(i8_kernel)).instantiate(command_queue)
    for m in range(M):
        op.set_beam_weights(m, g[m])
    (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    ref = O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, scale=1 / 64, signed=signed, gains=g)
    np.testing.assert_array_equal(q, ref)
    assert np.abs(ref.astype(int)).max() >= 4


def boundary_delays(M, A, seed):
    """Zero delays (rot = phase exactly) with phases whose cos or sin lands within ~1e-7 of a Q14 rounding
    boundary (k + 1/2) / 2^14: the fast float32 phasor cannot decide those, so nearly every coefficient takes
    the exact fallback (several per lane), and some with a gain too."""
    rng = np.random.default_rng(seed)
    k = rng.integers(-16000, 16000, (M, A))
    target = (k + 0.5) / 16384.0
    phi = np.arccos(target)
    use_sin = rng.random((M, A)) < 0.5
    phi = np.where(use_sin, np.pi / 2 - phi, phi)  # sin(pi/2 - x) = cos(x)
    phi = np.where(rng.random((M, A)) < 0.5, -phi, phi)
    d = np.zeros((1, M, A, 4), np.float32)
    d[0, ..., 2] = phi.astype(np.float32)
    return d


@pytest.mark.parametrize("A,M,C,T,B,signed", [(64, 16, 3, 256, 2, True), (64, 16, 2, 256, 2, False),
                                              (19, 3, 3, 48, 2, False), (256, 64, 1, 32, 1, True)])
@pytest.mark.parametrize("i8_kernel", ["auto", "item", "generic", "wide", "wide-inkernel"])
@pytest.mark.parametrize("weighted", [False, True])
def test_fused_int8_rounding_boundaries(context, command_queue, i8_kernel, weighted, A, M, C, T, B,
                                        signed):
    """Q14 coefficients whose exact value sits at a rounding boundary: the fast-phasor + exact-fixup path
    (bf_phase.hpp q14_coeffs) must still reproduce the integer contract bit for bit."""
    Ctot, xeng, t0, bdt = 4096, 0, 1e-3, 256 * 8192 * TS
    d = boundary_delays(M, A, A + M)
    rng = np.random.default_rng(A * 5 + M)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    g = rng.choice(np.float32([1.0, 0.5, -1.0, 0.75]), (M, A)).astype(np.float32) if weighted else None
    op = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=signed,
                                 out_int8=True, out_scale=1 / 64, t0=t0, batch_dt=bdt,
                                 beam_weights=weighted, **i8_path(i8_kernel)).instantiate(command_queue)
    if weighted:
        for m in range(M):
            op.set_beam_weights(m, g[m])
    (q,) = run(op, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    ref = O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, scale=1 / 64, signed=signed,
                                gains=g)
    np.testing.assert_array_equal(q, ref)


@pytest.mark.parametrize("A,M,C,T,B", [(1, 1, 1, 16, 1), (2, 1, 3, 16, 2), (16, 24, 2, 16, 1), (32, 33, 1, 32, 1),
                                       (257, 3, 1, 16, 1)])
@pytest.mark.parametrize("kernel", ["auto", "item", "generic", "wide"])
def test_fused_edge_shapes(context, command_queue, kernel, A, M, C, T, B):
    """Smallest and ragged shapes on every fused path (paths that do not fit a shape fall through to one that does):
    one antenna / beam / channel / batch, T = 16, M not a multiple of 8, A just past a k-step -- f32 within the
    tolerance and int8 bit-exact."""
    Ctot = 8 * C
    d = random_delays(1, M, A, A + M)
    rng = np.random.default_rng(A * M + T)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    fu = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=1, delay_channels=1,
                                 batch_dt=1e-4, kernel_path=kernel).instantiate(command_queue)
    (y,) = run(fu, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    assert_beams_allclose(y, O.fused_beamform(raw, d, Ctot, xeng_id=1, batch_dt=1e-4), O.reorder(raw),
                          O.fused_tables(d, B, C, Ctot, A, xeng_id=1, batch_dt=1e-4))
    q8 = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=1, delay_channels=1, batch_dt=1e-4,
                                 out_int8=True, out_scale=1 / 8, kernel_path=kernel).instantiate(command_queue)
    (q,) = run(q8, command_queue, {"inSamples": raw, "delay_vals": d}, ["outData"])
    np.testing.assert_array_equal(q, O.fused_beamform_int8(raw, d, Ctot, xeng_id=1, batch_dt=1e-4, scale=1 / 8))


@pytest.mark.parametrize("A,M,C,T,B", [(1, 1, 1, 16, 1), (3, 2, 2, 16, 1), (257, 5, 1, 32, 1)])
def test_drop_in_edge_shapes(context, command_queue, A, M, C, T, B):
    """The reference-structure chain (reorder -> coefficients -> table multiply) on the smallest and ragged shapes."""
    Ctot = 4 * C
    d = random_delays(C, M, A, 3 * A + M, rates=False)
    raw = O.u8_voltages((B, A, C, T, 2, 2), seed=A + T)
    seq = OpSequenceTemplate(context, B, 2, C, Ctot, T // 16, 16, A, M, 0, TS, T).instantiate(command_queue)
    seq.ensure_all_bound()
    seq.beamform_coeff.buffer("delay_vals").set(command_queue, d)
    seq.prebeamform_reorder.buffer("inSamples").set(command_queue, raw)
    seq()
    np.testing.assert_array_equal(seq.prebeamform_reorder.buffer("outReordered").get(command_queue), O.reorder(raw))
    np.testing.assert_array_equal(seq.beamform_coeff.buffer("outCoeffs").get(command_queue),
                                  O.coeffs(d, B, 2, C, Ctot, A, M, 0))
    y = seq.beamform_mult.buffer("outData").get(command_queue)
    assert_beams_allclose(y, O.op_sequence(raw, d, C, Ctot, A, M), O.reorder(raw), O.coeffs(d, B, 2, C, Ctot, A, M, 0))
