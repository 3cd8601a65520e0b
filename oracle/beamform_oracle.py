"""NumPy restatement of the reference beamformer algorithms (TEST INFRASTRUCTURE ONLY; see __init__).

Every function cites the reference file:line it restates.  Conventions:
B = batches, P = pols (2), C = channels on this engine, Ctot = channels in the band, A = antennas,
M = beams, T = samples per channel, NB = T // 16.
"""
import math

import numpy as np

TS_MEERKAT = 1 / 1712e6  # ADC sample period used by every reference test (e.g. beamform_op_sequence_test.py:90)
SAMPLES_PER_BLOCK = 16  # matrix_multiply.py:76 (128 // 8)


def u8_voltages(shape, seed=2021):
    """The reference tests' voltage generator (beamform_op_sequence_test.py:143-149)."""
    rng = np.random.default_rng(seed=seed)
    return rng.uniform(np.iinfo(np.uint8).min, np.iinfo(np.uint8).max, shape).astype(np.uint8)


def coeff_rotation(delay_vals, C, Ctot, xeng_id, Ts, dt=0.0, ch0=None):
    """Steering phase in float64, in the reference's exact left-to-right operation order.

    coeff_generator_cpu.py:125-164 (and coeff_generator.py:46-65):
        initial = delay_s * ichannel * (-pi) / (Ctot * Ts) + phase_rad
        centre  = delay_s * (Ctot / 2) * (-pi) / (Ctot * Ts)
        rot     = initial - centre
    Under numpy 1.x every step promotes to float64 (np.float32 * int -> float64).

    Time extension (used by the fused per-block regeneration): the delay and phase are
    first advanced by their rates, tau' = tau + tau_rate*dt and phi' = phi + phi_rate*dt, then the same
    expression is evaluated; at dt == 0 this is bit-identical to the reference.
    ch0: absolute channel of row 0 when the rows are a slice of an engine's channels (default C * xeng_id, the
    reference's `ichannel = c + C * xeng_id`, coeff_generator.py:53); lets tests check sampled channels of a
    full-size launch.
    Returns float64 (C, M, A).
    """
    d = np.asarray(delay_vals, dtype=np.float32)
    assert d.shape[0] == C and d.shape[-1] == 4
    tau = d[..., 0].astype(np.float64)
    phi = d[..., 2].astype(np.float64)
    if dt != 0.0:
        tau = tau + d[..., 1].astype(np.float64) * dt
        phi = phi + d[..., 3].astype(np.float64) * dt
    first = C * xeng_id if ch0 is None else int(ch0)
    ch = (np.arange(C, dtype=np.int64) + first).astype(np.float64)[:, None, None]
    denom = float(Ctot) * Ts
    initial = tau * ch * (-math.pi) / denom + phi
    centre = tau * (Ctot / 2) * (-math.pi) / denom
    return initial - centre


def _cos_sin_f32(rot):
    # math.cos/sin (libm, as the reference's Python calls) then round to float32 on store.
    flat = rot.ravel()
    c = np.fromiter((math.cos(v) for v in flat), dtype=np.float64, count=flat.size)
    s = np.fromiter((math.sin(v) for v in flat), dtype=np.float64, count=flat.size)
    return c.astype(np.float32).reshape(rot.shape), s.astype(np.float32).reshape(rot.shape)


def _pack_blocks(cos, sin, B, P):
    """[[R, I], [-I, R]] 2x2 real blocks: W[2a][2m]=R, W[2a][2m+1]=I, W[2a+1][2m]=-I, W[2a+1][2m+1]=R
    (coeff_generator_cpu.py:170-186), replicated over (batch, pol)."""
    C, M, A = cos.shape
    w = np.empty((C, A, 2, M, 2), np.float32)
    cT = cos.transpose(0, 2, 1)
    sT = sin.transpose(0, 2, 1)
    w[:, :, 0, :, 0] = cT
    w[:, :, 0, :, 1] = sT
    w[:, :, 1, :, 0] = -sT
    w[:, :, 1, :, 1] = cT
    w = w.reshape(C, 2 * A, 2 * M)
    return np.broadcast_to(w, (B, P, C, 2 * A, 2 * M)).copy()


def coeffs(delay_vals, B, P, C, Ctot, A, M, xeng_id, Ts=TS_MEERKAT):
    """CoeffGenerator.cpu_coeffs (coeff_generator_cpu.py:78-187): f32 (B, P, C, 2A, 2M).

    delay_vals[c][m][a] feeds antenna a, beam m (the CPU oracle's mapping; the numba kernel's transposed
    read, SURVEY A1, is not reproduced)."""
    d = np.asarray(delay_vals, np.float32)
    assert d.shape == (C, M, A, 4), d.shape
    cos, sin = _cos_sin_f32(coeff_rotation(d, C, Ctot, xeng_id, Ts))
    return _pack_blocks(cos, sin, B, P)


def coeffs_at(delay_vals, C, Ctot, A, M, xeng_id, Ts, dt, ch0=None):
    """Compact complex coefficients at time offset dt: (cos, sin) f32, each (C, M, A)."""
    d = np.asarray(delay_vals, np.float32)
    return _cos_sin_f32(coeff_rotation(d, C, Ctot, xeng_id, Ts, dt, ch0))


def reorder(x):
    """reorder.run_reorder (beamforming/reorder.py:40-42): (B,A,C,T,2,2) -> (B,2,C,T/16,16,A,2)."""
    B, A, C, T, P, Z = x.shape
    return np.ascontiguousarray(
        x.reshape(B, A, C, T // SAMPLES_PER_BLOCK, SAMPLES_PER_BLOCK, P, Z).transpose(0, 5, 2, 3, 4, 1, 6))


def _as_real(x, signed):
    if signed:
        return np.asarray(x).view(np.int8).astype(np.float32)
    return np.asarray(x).astype(np.float32)


def complex_mult(x, w, signed=False):
    """complex_mult_cpu.complex_mult (unit_test/complex_mult_cpu.py:82-147), vectorised.

    x: u8 (B,P,C,NB,16,A,2); w: f32 (B,P,C,2A,2M) -> f32 (B,P,C,NB,16,2M):
        out[..., col] = sum_k X[..., k] * W[k, col],  X[2a] = re, X[2a+1] = im   (complex_mult_kernel.py:89-100)
    Per-beam correct (the reference CPU loop reads beam-0 coefficients for every beam; the two agree
    whenever coefficients are beam-uniform, which is what the reference tests use)."""
    B, P, C, NB, S, A, Z = x.shape
    X = _as_real(x, signed).reshape(B, P, C, NB * S, 2 * A)
    Y = np.matmul(X, np.asarray(w, np.float32))
    return Y.reshape(B, P, C, NB, S, -1)


def op_sequence(raw, delay_vals, C, Ctot, A, M, xeng_id=0, Ts=TS_MEERKAT):
    """OpSequence (beamform_op_sequence.py:117-157): reorder -> coeffs -> complex mult."""
    B = raw.shape[0]
    return complex_mult(reorder(raw), coeffs(delay_vals, B, 2, C, Ctot, A, M, xeng_id, Ts))


def fused_beamform(raw, delay_vals, Ctot, xeng_id=0, Ts=TS_MEERKAT, t0=0.0, batch_dt=0.0, signed=False, gains=None,
                   ch0=None):
    """The fused MI355X operator's contract: reorder + per-batch coefficient regeneration + complex mult.

    raw: (B, A, C, T, 2, 2) 8-bit; delay_vals: (C, M, A, 4) or compact (1, M, A, 4) (same model for every
    channel).  Batch b uses coefficients at dt_b = t0 + b * batch_dt (the per-block regeneration of
    BeamformerParameters.h:17 ACCUMULATIONS_BEFORE_NEW_COEFFS).  gains: optional (M, A) real beam weights
    (see fused_tables).  ch0: see coeff_rotation.  Output f32 (B, 2, C, T/16, 16, 2M)."""
    B, A, C, T, P, Z = raw.shape
    w = fused_tables(delay_vals, B, C, Ctot, A, xeng_id, Ts, t0, batch_dt, gains, ch0)
    return complex_mult(reorder(raw), w, signed=signed)


def fused_tables(delay_vals, B, C, Ctot, A, xeng_id=0, Ts=TS_MEERKAT, t0=0.0, batch_dt=0.0, gains=None, ch0=None):
    """The (B, 2, C, 2A, 2M) coefficient tables the fused operator applies (batch b at dt = t0 + b*batch_dt).

    gains: optional (M, A) float32 per-input beam weights (the `?beam-weights <beam> w_0..w_{A-1}` control request,
    ngkcs/ngkcs/corr3_servlet.py:140-153): the float32 phasor of (a, m) is scaled by g[m, a] in float32, one
    rounding per component, before the [[R, I], [-I, R]] packing."""
    d = np.asarray(delay_vals, np.float32)
    if d.shape[0] == 1 and C > 1:
        d = np.broadcast_to(d, (C,) + d.shape[1:])
    M = d.shape[1]
    w = np.empty((B, 2, C, 2 * A, 2 * M), np.float32)
    for b in range(B):
        cos, sin = coeffs_at(d, C, Ctot, A, M, xeng_id, Ts, t0 + b * batch_dt, ch0)
        if gains is not None:
            g = np.asarray(gains, np.float32)
            assert g.shape == (M, A), g.shape
            cos, sin = cos * g, sin * g  # float32 x float32 -> float32
        w[b] = _pack_blocks(cos, sin, 1, 2)[0]
    return w


def dot_magnitude(x, w, signed=False):
    """sum_k |x_k| |w_k| per output (float64): the scale of fp32 rounding in each beam's dot product."""
    B, P, C, NB, S, A, Z = x.shape
    X = np.abs(_as_real(x, signed).reshape(B, P, C, NB * S, 2 * A)).astype(np.float64)
    return np.matmul(X, np.abs(np.asarray(w, np.float64))).reshape(B, P, C, NB, S, -1)


def requantise(y, scale):
    """8-bit requantiser contract (the reference has none; SURVEY hard part 5): round-half-to-even of
    y * scale, saturated to [-127, 127] (symmetric, so conjugation never overflows).  int8 output."""
    v = np.rint(np.asarray(y, np.float32) * np.float32(scale))
    return np.clip(v, -127, 127).astype(np.int8)


Q14 = 14  # fractional bits of the integer beamformer's coefficients


def quantise_coeffs(w):
    """Q14 steering coefficients: W = rne(w * 2^14) of the float32 coefficient (exact product), int64."""
    return np.rint(np.asarray(w, np.float32).astype(np.float64) * (1 << Q14)).astype(np.int64)


def fused_beamform_int8(raw, delay_vals, Ctot, xeng_id=0, Ts=TS_MEERKAT, t0=0.0, batch_dt=0.0, scale=1.0,
                        signed=False, gains=None, ch0=None):
    """Contract of the fused operator's int8 (requantised) output -- bit-exact:
        W = rne(w * 2^14)  (w: the exact float32 coefficients of fused_tables, i.e. CoeffGenerator's at dt = 0)
        y = sum_k x_k W_k  (exact integers)
        q = clamp(rne(float32(y) * float32(float32(scale) * 2^-14)), -127, 127)
    raw: (B, A, C, T, 2, 2) 8-bit -> int8 (B, 2, C, T/16, 16, 2M)."""
    B, A, C, T, P, Z = raw.shape
    W = quantise_coeffs(fused_tables(delay_vals, B, C, Ctot, A, xeng_id, Ts, t0, batch_dt, gains, ch0))
    xr = reorder(raw)
    X = (xr.view(np.int8) if signed else xr).astype(np.int64).reshape(B, 2, C, T, 2 * A)
    Y = np.matmul(X, W)
    s = np.float32(np.float32(scale) * np.float32(2.0 ** -Q14))
    q = np.rint(Y.astype(np.float32) * s)
    return np.clip(q, -127, 127).astype(np.int8).reshape(B, 2, C, T // 16, 16, -1)


# ---- the C++ study's time-dependent steering coefficients (beamformer_coefficient_generator/) -----------------
STUDY_TS = np.float32(1e-7)  # SAMPLING_PERIOD 1e-7f (BeamformerParameters.h:14)
STUDY_FFT = 8192  # FFT_SIZE (BeamformerParameters.h:15)


def study_delay_ramp(A, M, Ts=STUDY_TS):
    """The study harness's delay model (BeamformerCoeffTest::simulate_input, BeamformerCoefficientTest.cu:185-196):
    entry i of the A*M antenna-major array = (i/(A M) * Ts/3, 2e-6, (1 - i/(A M)) * Ts/3, 3e-6), float32."""
    n = A * M
    i = np.arange(n, dtype=np.float32)
    d = np.empty((n, 4), np.float32)
    # ((float)i / (float)n) * SAMPLING_PERIOD is float arithmetic; "/ 3.0" is double; the struct field is float
    ts = np.float32(Ts)
    d[:, 0] = ((i / np.float32(n)) * ts).astype(np.float64) / 3.0
    d[:, 1] = np.float32(2e-6)
    d[:, 2] = ((np.float32(1) - i / np.float32(n)) * ts).astype(np.float64) / 3.0
    d[:, 3] = np.float32(3e-6)
    return d


def study_coeffs_time(delay_vals, n_times, C, A, M, Ts=STUDY_TS, fft_size=STUDY_FFT):
    """The study's CPU golden for its time-dependent kernels (BeamformerCoeffTest::verify_output,
    BeamformerCoefficientTest.cu:294-337), operation for operation:
        timeStep_ns = long(float32(t * Ts * 1e9f * FFT));  dt = float32(timeStep_ns) / 1e9f       (:299, ts_diff :12-18)
        dd = rate * dt;  delayN = (rate + dd) * c * pi / (Ts * C)                                   (float32, :321-322)
        delayN2 = float32((delay + dd) * (C / 2.0) * pi / (Ts * C))   -- C / 2.0 is a double: double arithmetic (:323)
        rot = delayN + (phase - delayN2 + phase_rate * dt);  (cos rot, sin rot)                     (:324-328)
    delay_vals: (A*M, 4) float32, index a*M + m.  Returns complex64 (n_times, C, A, M)."""
    f32 = np.float32
    d = np.asarray(delay_vals, np.float32).reshape(A, M, 4)
    delay, rate, phase, prate = (d[..., k][None, None] for k in range(4))
    t = np.arange(n_times, dtype=np.float32)
    step_ns = np.trunc(t * f32(Ts) * f32(1e9) * f32(fft_size)).astype(np.int64)
    dt = (step_ns.astype(np.float32) / f32(1e9)).astype(np.float32)[:, None, None, None]
    c = np.arange(C, dtype=np.float32)[None, :, None, None]
    pi = f32(math.pi)
    tsc = f32(f32(Ts) * f32(C))
    dd = (rate * dt).astype(np.float32)
    delay_n = ((((rate + dd) * c) * pi) / tsc).astype(np.float32)
    delay_n2 = ((((delay + dd).astype(np.float64) * (C / 2.0)) * np.float64(pi)) / np.float64(tsc)).astype(np.float32)
    dphase = (prate * dt).astype(np.float32)
    phase0 = ((phase - delay_n2) + dphase).astype(np.float32)
    rot = (delay_n + phase0).astype(np.float32).astype(np.float64)
    return (np.cos(rot).astype(np.float32) + 1j * np.sin(rot).astype(np.float32)).astype(np.complex64)


def study_beams_single_channel(delay_vals, x, C, T, A, M, Ts=STUDY_TS, fft_size=STUDY_FFT):
    """The study harness's golden for its fused kernel (BeamformerCoeffTest::verify_output, the
    COMBINED_COEFF_GEN_AND_BEAMFORMER_SINGLE_CHANNEL case, BeamformerCoefficientTest.cu:356-400):
        y_re[c][t_ex][b][t_in] = sum_a cos(rot) * x_re,   y_im = sum_a sin(rot) * x_im        (:385-394)
    -- the study's own semantics, not a complex product -- with the coefficients of study_coeffs_time at
    time t = 16 t_ex + t_in and the delay model of (a, b) at index b*A + a (the combined kernel's ordering, :307-316).
    Each product and each partial sum is one float32 rounding, antennas in order, as the golden's loop.
    delay_vals: (M*A, 4) float32; x: int8 (C, T/16, A, 16, 2).  Returns float32 (C, T/16, M, 16, 2)."""
    d = np.asarray(delay_vals, np.float32).reshape(M, A, 4).transpose(1, 0, 2).reshape(A * M, 4)
    w = study_coeffs_time(d, T, C, A, M, Ts, fft_size)  # (T, C, A, M)
    w = w.reshape(T // 16, 16, C, A, M).transpose(2, 0, 3, 4, 1)  # (C, T/16, A, M, 16)
    cs, sn = np.ascontiguousarray(w.real), np.ascontiguousarray(w.imag)
    xv = np.asarray(x, np.int8).reshape(C, T // 16, A, 16, 2).astype(np.float32)
    re = np.zeros((C, T // 16, M, 16), np.float32)
    im = np.zeros((C, T // 16, M, 16), np.float32)
    for a in range(A):
        re += cs[:, :, a] * xv[:, :, a, None, :, 0]
        im += sn[:, :, a] * xv[:, :, a, None, :, 1]
    return np.stack([re, im], axis=-1)

