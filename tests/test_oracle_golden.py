"""The CPU oracle (oracle/) against golden vectors produced by the reference's own CPU oracles.

Pins: coefficients bit-exact (coeff_generator_cpu.py:78-187), reorder bit-exact (reorder.py:40-42), multiply and
the full OpSequence chain within the reference tests' rtol = atol = 1e-4 (beamform_mult_kernel_test.py:267-269,
beamform_op_sequence_test.py:198-200).
"""
import numpy as np
import pytest

import oracle as O
from golden_io import cases, get, sha256, voltages


@pytest.mark.parametrize("case", cases("reorder_"))
def test_reorder_golden(case):
    B, A, C, T = (int(v) for v in get(case, "dims"))
    x = voltages(case, (B, A, C, T, 2, 2))
    y = O.reorder(x)
    assert y.shape == tuple(get(case, "output_shape"))
    assert sha256(y) == str(get(case, "output_sha256"))


@pytest.mark.parametrize("case", cases("coeff_"))
def test_coeffs_golden(case):
    B, P, C, Ctot, A, M, xeng_id = (int(v) for v in get(case, "dims"))
    w = O.coeffs(get(case, "delays"), B, P, C, Ctot, A, M, xeng_id)
    np.testing.assert_array_equal(w[0, 0], get(case, "coeffs00"))
    assert sha256(w) == str(get(case, "coeffs_sha256"))


@pytest.mark.parametrize("case", cases("mult_"))
def test_complex_mult_golden(case):
    B, A, M, Ctot, T, C = (int(v) for v in get(case, "dims"))
    w = O.coeffs(get(case, "delays"), B, 2, C, Ctot, A, M, 0)
    assert sha256(w) == str(get(case, "coeffs_sha256"))
    x = voltages(case, (B, 2, C, T // 16, 16, A, 2))
    np.testing.assert_allclose(O.complex_mult(x, w), get(case, "output"), rtol=1e-4, atol=1e-4)


def test_op_sequence_golden():
    B, A, M, Ctot, T, C = (int(v) for v in get("opseq_cfg1", "dims"))
    raw = voltages("opseq_cfg1", (B, A, C, T, 2, 2))
    y = O.op_sequence(raw, get("opseq_cfg1", "delays"), C, Ctot, A, M)
    np.testing.assert_allclose(y, get("opseq_cfg1", "output"), rtol=1e-4, atol=1e-4)


def test_fused_contract_reduces_to_op_sequence():
    """With zero rates/dt the fused contract equals reorder -> coeffs -> multiply exactly."""
    B, A, M, Ctot, T, C = (int(v) for v in get("opseq_cfg1", "dims"))
    raw = voltages("opseq_cfg1", (B, A, C, T, 2, 2))
    d = get("opseq_cfg1", "delays")
    np.testing.assert_array_equal(O.fused_beamform(raw, d, Ctot), O.op_sequence(raw, d, C, Ctot, A, M))


def test_time_extension_at_zero_is_reference_phase():
    rng = np.random.default_rng(5)
    d = rng.uniform(-1, 1, (3, 2, 5, 4)).astype(np.float32)
    d[..., 0] *= 1e-8
    r0 = O.coeff_rotation(d, 3, 1024, 2, O.TS_MEERKAT)
    r1 = O.coeff_rotation(d, 3, 1024, 2, O.TS_MEERKAT, dt=0.0)
    np.testing.assert_array_equal(r0, r1)
    r2 = O.coeff_rotation(d, 3, 1024, 2, O.TS_MEERKAT, dt=1e-3)
    assert not np.array_equal(r0, r2)


@pytest.mark.parametrize("case", cases("rates_"))
def test_time_extension_golden(case):
    """dt != 0 pinned by the reference (G5): the fused tables at dt_b = t0 + b*batch_dt, built from delay models WITH
    rates, equal the reference's cpu_coeffs on the float32-exact advanced models (tau_b, 0, phi_b, 0) bit for bit."""
    A, M, C, Ctot, xeng_id, nb = (int(v) for v in get(case, "dims"))
    t0, batch_dt = (float(v) for v in get(case, "times"))
    d = get(case, "delays")
    assert d.shape == (1, M, A, 4) and (d[..., 1] != 0).all() and (d[..., 3] != 0).all()
    w = O.fused_tables(d, nb, C, Ctot, A, xeng_id, O.TS_MEERKAT, t0, batch_dt)
    for p in range(2):
        np.testing.assert_array_equal(w[:, p], get(case, "coeffs"))
    # and the rates matter: with them zeroed every batch's table is the dt = 0 table
    d0 = d.copy()
    d0[..., 1] = d0[..., 3] = 0
    assert not np.array_equal(O.fused_tables(d0, nb, C, Ctot, A, xeng_id, O.TS_MEERKAT, t0, batch_dt)[:, 0],
                              get(case, "coeffs"))


@pytest.mark.parametrize("case", cases("rates_"))
def test_int8_time_extension_golden(case):
    """The int8 contract at dt != 0 (oracle.fused_beamform_int8 on a model with rates) from the reference's own
    per-batch tables (G5): Q14 of the golden coefficients, exact integer products, one rounding."""
    A, M, C, Ctot, xeng_id, B = (int(v) for v in get(case, "dims"))
    t0, bdt = (float(v) for v in get(case, "times"))
    T, scale = 32, 1.0 / 16
    raw = np.random.default_rng(A).integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8).view(np.int8)
    q = O.fused_beamform_int8(raw, get(case, "delays"), Ctot, xeng_id=xeng_id, t0=t0, batch_dt=bdt, scale=scale,
                              signed=True)
    W = O.quantise_coeffs(np.broadcast_to(get(case, "coeffs")[:, None], (B, 2, C, 2 * A, 2 * M)))
    X = O.reorder(raw).view(np.int8).astype(np.int64).reshape(B, 2, C, T, 2 * A)
    s = np.float32(np.float32(scale) * np.float32(2.0 ** -14))
    ref = np.clip(np.rint(np.matmul(X, W).astype(np.float32) * s), -127, 127).astype(np.int8)
    np.testing.assert_array_equal(q, ref.reshape(q.shape))


def test_q14_time_extension_golden_at_config4_shape():
    """G5 at config 4's shape: the int8 contract's Q14 coefficients of the oracle (quantise_coeffs of fused_tables,
    a model with rates at dt_b = t0 + b batch_dt) equal rne(2^14 w) of the reference's coefficients."""
    A, M, C, Ctot, xeng, B = (int(v) for v in get("q14rates_a256_m64", "dims"))
    t0, bdt = (float(v) for v in get("q14rates_a256_m64", "times"))
    w = O.quantise_coeffs(O.fused_tables(get("q14rates_a256_m64", "delays"), B, C, Ctot, A, xeng, O.TS_MEERKAT, t0,
                                         bdt))
    q = get("q14rates_a256_m64", "q14")
    np.testing.assert_array_equal(w[:, 0, :, 0::2, 0::2].transpose(0, 1, 3, 2), q[..., 0])
    np.testing.assert_array_equal(w[:, 0, :, 0::2, 1::2].transpose(0, 1, 3, 2), q[..., 1])


def test_requantise_contract():
    y = np.array([0.5, 1.5, 2.5, -0.5, -1.5, 126.6, 1e9, -1e9, np.float32(127.49)], np.float32)
    np.testing.assert_array_equal(O.requantise(y, 1.0), [0, 2, 2, 0, -2, 127, 127, -127, 127])


def test_reference_tolerance_is_not_fp32_attainable():
    """Why the beam tolerance carries an fp32 dot-product term (tests/tolerance.py): the reference's own fp32
    arithmetic (np.dot / np.matmul in float32, complex_mult_cpu.py:98) misses rtol = atol = 1e-4 against the
    exact product once delays are non-uniform, and stays inside the stated tolerance."""
    from tolerance import assert_beams_allclose
    C, M, A, B = 16, 16, 64, 1
    rng = np.random.default_rng(0)
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * O.TS_MEERKAT, (C, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (C, M, A))
    w = O.coeffs(d, B, 2, C, 4096, A, M, 0)
    x = O.u8_voltages((B, 2, C, 16, 16, A, 2))
    y32 = O.complex_mult(x, w)
    exact = np.matmul(x.reshape(B, 2, C, 256, 2 * A).astype(np.float64), w.astype(np.float64)).reshape(y32.shape)
    assert (np.abs(y32 - exact) > 1e-4 + 1e-4 * np.abs(exact)).sum() > 0
    assert_beams_allclose(y32, exact, x, w)


def test_int8_contract_is_close_to_float_beams():
    """The integer int8 contract (Q14 coefficients, exact integer sums) stays within one LSB of requantising the
    float32 beams except at rounding ties."""
    B, A, M, C, T, Ctot = 1, 19, 3, 5, 32, 1024
    rng = np.random.default_rng(2)
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * O.TS_MEERKAT, (C, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (C, M, A))
    raw = O.u8_voltages((B, A, C, T, 2, 2), seed=4)
    q = O.fused_beamform_int8(raw, d, Ctot, scale=1 / 16).astype(int)
    qf = O.requantise(O.fused_beamform(raw, d, Ctot), 1 / 16).astype(int)
    assert np.abs(q - qf).max() <= 1
    assert (q == qf).mean() > 0.99


def test_beam_weights_oracle_properties():
    """Weights of one are the identity; power-of-two weights scale beams exactly (linearity); weights are per
    (beam, input): zeroing input a of beam m removes exactly antenna a's contribution to beam m."""
    rng = np.random.default_rng(5)
    raw = O.u8_voltages((2, 6, 3, 32, 2, 2), seed=9)
    d = np.zeros((1, 4, 6, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * O.TS_MEERKAT, (1, 4, 6))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (1, 4, 6))
    base = O.fused_beamform(raw, d, 64)
    np.testing.assert_array_equal(O.fused_beamform(raw, d, 64, gains=np.ones((4, 6), np.float32)), base)
    np.testing.assert_array_equal(O.fused_beamform(raw, d, 64, gains=np.full((4, 6), 0.25, np.float32)), base * 0.25)
    g = np.ones((4, 6), np.float32)
    g[2, 3] = 0.0
    only = raw.copy()
    only[:, [a for a in range(6) if a != 3]] = 0  # antenna 3 alone
    diff = base - O.fused_beamform(raw, d, 64, gains=g)
    contrib = O.fused_beamform(only, d, 64)
    np.testing.assert_allclose(diff[..., 4:6], contrib[..., 4:6], rtol=1e-5, atol=1e-3)  # beam 2 = cols 4, 5
    np.testing.assert_array_equal(diff[..., :4], 0)
    q1 = O.fused_beamform_int8(raw, d, 64, scale=1 / 16)
    np.testing.assert_array_equal(O.fused_beamform_int8(raw, d, 64, scale=1 / 16, gains=np.ones((4, 6), np.float32)), q1)


def test_reference_bar_arbitration_path():
    """assert_reference_bar's fallback for elements that miss rtol=atol=1e-4 (taken on the GPU only when a beam
    cancels to near zero): a miss that is exact against the float64 product passes, one that is not fails."""
    import pytest
    from tolerance import assert_reference_bar
    rng = np.random.default_rng(3)
    B, P, C, NB, A, M = 1, 2, 3, 2, 5, 2
    x = rng.integers(0, 256, (B, P, C, NB, 16, A, 2), dtype=np.uint8)
    w = rng.uniform(-1, 1, (B, P, C, 2 * A, 2 * M)).astype(np.float32)
    exact = O.complex_mult(x, w).astype(np.float64)
    ref = exact.copy()
    ref.reshape(-1)[7] += 1.0  # the "reference f32" result is off at one element; the GPU result is exact there
    assert assert_reference_bar(exact, ref, x, w) == 1
    bad = exact.copy()
    bad.reshape(-1)[7] += 2.0  # farther from the exact product than the reference, outside the bar and the fp32 bound
    with pytest.raises(AssertionError):
        assert_reference_bar(bad, ref, x, w)


def test_study_time_golden_restatement():
    """oracle.study_coeffs_time (the C++ study's CPU golden, BeamformerCoefficientTest.cu:294-337, vectorised) equals
    a scalar restatement of that loop, element by element in the golden's own float / double order, on the study's
    delay ramp (simulate_input, :185-196) at a spread of (t, c, a, m) -- the study's dt != 0 convention."""
    import math

    f32, f64 = np.float32, np.float64
    A, M, C, NT = 64, 16, 64, 256  # the study's defaults (BeamformerParameters.h:7-11)
    d = O.study_delay_ramp(A, M)
    assert d.dtype == np.float32 and d.shape == (A * M, 4)
    # simulate_input's ramp, scalar: ((float)i / (float)n) * SAMPLING_PERIOD / 3.0
    for i in (0, 1, 517, A * M - 1):
        assert d[i, 0] == f32(f64(f32(f32(i) / f32(A * M)) * f32(1e-7)) / 3.0)
        assert d[i, 2] == f32(f64(f32(f32(1) - f32(i) / f32(A * M)) * f32(1e-7)) / 3.0)
    w = O.study_coeffs_time(d, NT, C, A, M)
    assert w.shape == (NT, C, A, M) and w.dtype == np.complex64
    ts, pi = f32(1e-7), f32(math.pi)
    for t, c, a, m in ((0, 0, 0, 0), (1, 3, 5, 7), (17, 63, 0, 15), (128, 31, 40, 2), (255, 63, 63, 15)):
        step = int(f32(f32(f32(t) * ts) * f32(1e9)) * f32(8192))  # long timeStep = t*SAMPLING_PERIOD*1e9f*FFT_SIZE
        dt = f32(f32(step) / f32(1e9))  # ts_diff: (float) nanosec_difference / 1e9f
        delay, rate, phase, prate = (f32(v) for v in d[a * M + m])
        dd = f32(rate * dt)
        delay_n = f32(f32(f32(f32(rate + dd) * f32(c)) * pi) / f32(ts * f32(C)))
        delay_n2 = f32(f64(f32(delay + dd)) * (C / 2.0) * f64(pi) / f64(f32(ts * f32(C))))
        rot = f32(delay_n + f32(f32(phase - delay_n2) + f32(prate * dt)))
        assert w[t, c, a, m].real == f32(math.cos(rot)) and w[t, c, a, m].imag == f32(math.sin(rot)), (t, c, a, m)
    # the convention differs from the Python path's (delay rate in the channel term, opposite sign): at t = 0 and
    # c = 0 the study's phase is phase - delay * (C/2) * pi / (Ts C), the Python path's phase + pi * delay / (2 Ts)
    assert np.allclose(np.angle(w[0, 0, :, :]).ravel(),
                       np.angle(np.exp(1j * (d[:, 2].astype(np.float64) - d[:, 0] * (C / 2) * np.pi / (1e-7 * C)))),
                       atol=1e-6)


def test_study_single_channel_beams_restatement():
    """oracle.study_beams_single_channel (the study harness's golden for its fused kernel, BeamformerCoefficientTest.cu:
    356-400, vectorised over channels, chunks and beams) equals the golden's own loop nest restated literally -- per
    (c, t_ex, b, t_in) a float32 sum over the antennas in order of cos(rot) x_re and sin(rot) x_im (the study's
    non-complex product) with the coefficient of delay entry b*A + a -- on the harness's inputs
    (simulate_input, :185-204: the delay ramp and x[i] = (int8) i)."""
    f32 = np.float32
    C, T, A, M = 6, 32, 5, 3
    d = O.study_delay_ramp(A, M)
    x = np.arange(C * T * A * 2, dtype=np.int64).astype(np.int8).reshape(C, T // 16, A, 16, 2)
    y = O.study_beams_single_channel(d, x, C, T, A, M)
    assert y.shape == (C, T // 16, M, 16, 2) and y.dtype == np.float32
    w = O.study_coeffs_time(d.reshape(M, A, 4).transpose(1, 0, 2).reshape(A * M, 4), T, C, A, M)  # index a*M + b
    for c, tex, b, tin in ((0, 0, 0, 0), (5, 1, 2, 15), (3, 0, 1, 7), (1, 1, 0, 9)):
        re = im = f32(0)
        for a in range(A):
            co = w[16 * tex + tin, c, a, b]
            re = f32(re + f32(co.real * f32(x[c, tex, a, tin, 0])))
            im = f32(im + f32(co.imag * f32(x[c, tex, a, tin, 1])))
        assert y[c, tex, b, tin, 0] == re and y[c, tex, b, tin, 1] == im, (c, tex, b, tin)
    # not a complex product: the real beam ignores x_im entirely
    x2 = x.copy()
    x2[..., 1] = 0
    np.testing.assert_array_equal(O.study_beams_single_channel(d, x2, C, T, A, M)[..., 0], y[..., 0])
