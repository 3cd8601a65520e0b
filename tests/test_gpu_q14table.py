"""GPU: the int8 path's wavefront-parallel Q14 coefficient generator (bf_q14_coeffs, csrc/bf_q14table.hip) and the
table-driven 32-beam int8 kernel it feeds (bf_beamform_fused_ws).

The generator walks each (antenna, beam) along the channels with a float64 complex recurrence and decides every
Q14 value against the guard band of bf_phase.hpp; undecided values are re-evaluated exactly.  Its output must equal
the contract's coefficients bit for bit: oracle quantise_coeffs of fused_tables (the float64 phase in the reference's
operation order, coeff_generator_cpu.py:145-164, rounded to float32, times the gain, times 2^14, ties to even)."""
import ctypes

import numpy as np
import pytest

import oracle as O
from dpdk_dc_sand_amd import _lib, accel
from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate
from golden_io import get

pytestmark = pytest.mark.gpu
TS = O.TS_MEERKAT


def delays(C, M, A, seed, tau_max=10 * TS, rates=True):
    rng = np.random.default_rng(seed)
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, tau_max, (C, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (C, M, A))
    if rates:
        d[..., 1] = rng.uniform(-1e-9, 1e-9, (C, M, A))
        d[..., 3] = rng.uniform(-1.0, 1.0, (C, M, A))
    return d


def expected_words(d, B, C, Ctot, A, M, xeng, t0, bdt, gains=None):
    w = O.quantise_coeffs(O.fused_tables(d, B, C, Ctot, A, xeng_id=xeng, t0=t0, batch_dt=bdt, gains=gains))
    wc = w[:, 0, :, 0::2, 0::2]  # (B, C, A, M): W[2a][2m] = cos
    ws = w[:, 0, :, 0::2, 1::2]  # W[2a][2m+1] = sin
    word = (wc.astype(np.int64) & 0xffff) | ((ws.astype(np.int64) & 0xffff) << 16)
    return np.ascontiguousarray(word.transpose(0, 1, 3, 2)).astype(np.uint32)  # (B, C, M, A)


def generate(context, queue, d, B, C, Ctot, A, M, xeng, t0, bdt, gains=None):
    dd = accel.DeviceArray(context, d.shape, np.float32)
    dd.set(queue, d)
    out = accel.DeviceArray(context, (B, C, M, A), np.uint32)
    g = None
    if gains is not None:
        g = accel.DeviceArray(context, gains.shape, np.float32)
        g.set(queue, gains)
    _lib.call("bf_q14_coeffs", dd.ptr, d.shape[0], _lib.ptr(g), out.ptr, B, C, A, M, Ctot, xeng, TS, t0, bdt,
              queue.handle)
    return out.get(queue)


@pytest.mark.parametrize("B,C,A,M,Ctot,xeng,dch", [
    (1, 1, 4, 1, 64, 0, 1), (2, 64, 19, 3, 1024, 3, 1), (1, 200, 64, 16, 4096, 1, 1), (3, 70, 5, 2, 8192, 5, 1),
    (1, 130, 256, 8, 32768, 7, 1), (2, 9, 33, 5, 4096, 2, 9), (1, 65, 64, 4, 65536, 15, 1)])
@pytest.mark.parametrize("weighted", [False, True])
def test_q14_coeffs_match_the_contract(context, command_queue, B, C, A, M, Ctot, xeng, dch, weighted):
    """Bit-exact over channel runs of 64 (and a ragged last run), batches (per-batch steering time with rates),
    X-engines (absolute channels), per-channel delay models, and beam weights."""
    t0, bdt = 2.5e-3, 256 * 2 * Ctot * TS
    d = delays(dch, M, A, seed=B * 1000 + C + A)
    g = np.random.default_rng(A + M).uniform(-1.9, 1.9, (M, A)).astype(np.float32) if weighted else None
    got = generate(context, command_queue, d, B, C, Ctot, A, M, xeng, t0, bdt, g)
    np.testing.assert_array_equal(got, expected_words(d, B, C, Ctot, A, M, xeng, t0, bdt, g))


def test_q14_coeffs_rounding_boundaries(context, command_queue):
    """Zero delays with phases whose cos or sin sits within ~1e-7 of a Q14 rounding boundary: no rotation along the
    channels, and nearly every value needs the exact evaluation."""
    M, A, C, Ctot = 4, 64, 80, 4096
    rng = np.random.default_rng(3)
    k = rng.integers(-16000, 16000, (M, A))
    phi = np.arccos((k + 0.5) / 16384.0)
    phi = np.where(rng.random((M, A)) < 0.5, np.pi / 2 - phi, phi)
    d = np.zeros((1, M, A, 4), np.float32)
    d[0, ..., 2] = phi.astype(np.float32)
    got = generate(context, command_queue, d, 1, C, Ctot, A, M, 0, 0.0, 0.0)
    np.testing.assert_array_equal(got, expected_words(d, 1, C, Ctot, A, M, 0, 0.0, 0.0))


@pytest.mark.parametrize("tau_samples", [1e3, 1e5, 4e5])
def test_q14_coeffs_large_delays(context, command_queue, tau_samples):
    """Delays up to and past the guard's validated phase range (bf_phase.hpp kQ14MaxMag): large rotations per
    channel; beyond the range every value is evaluated exactly."""
    M, A, C, Ctot = 3, 16, 96, 32768
    d = delays(1, M, A, seed=int(tau_samples), tau_max=tau_samples * TS)
    got = generate(context, command_queue, d, 1, C, Ctot, A, M, 6, 1e-3, 0.0)
    np.testing.assert_array_equal(got, expected_words(d, 1, C, Ctot, A, M, 6, 1e-3, 0.0))


@pytest.mark.parametrize("A,M,C,T,B,signed,weighted", [
    (256, 64, 24, 64, 1, True, False), (256, 64, 17, 32, 1, False, True), (200, 40, 9, 48, 2, False, False),
    (128, 32, 12, 256, 1, True, True), (96, 24, 5, 16, 3, False, False),
    # 8 k-steps x 2 passes (the straight-line 2-buffer form) with ragged sample chunks, a partial second slab and a
    # ragged last channel group
    (256, 40, 5, 208, 1, False, True), (256, 64, 6, 144, 2, True, False),
    # config 4's item shape, signed (64 beams, T = 256: the straight-line 8-step x 2-pass form at A = 256), and 3
    # k-steps (A = 96) with 64 beams
    (256, 64, 12, 256, 1, True, False), (256, 64, 9, 256, 2, True, True), (96, 64, 7, 256, 1, True, False),
    # the LDS-DMA ring kernel (w32r: signed, 224 < A <= 256, T = 256, M % 32 == 0) with padded antennas in its last
    # k-step (zero table entries, pulled-back loads), one and three 32-beam slabs, ragged channel runs
    (240, 32, 11, 256, 2, True, False), (232, 96, 13, 256, 1, True, True), (248, 64, 21, 256, 1, True, False)])
def test_fused_int8_table_path_equals_in_kernel_and_oracle(context, command_queue, A, M, C, T, B, signed, weighted):
    """The int8 wide path with the generated table (default) and with in-kernel phasors (coeff_table=False): the
    same bits, and the integer contract's."""
    Ctot, xeng, t0, bdt = 32768, 5, 1e-3, 256 * 2 * 32768 * TS
    d = delays(1, M, A, seed=A + M + C)
    rng = np.random.default_rng(A * 7 + C)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    if signed:
        raw = raw.view(np.int8)
    g = rng.uniform(-1.2, 1.2, (M, A)).astype(np.float32) if weighted else None
    outs = {}
    for table in (True, False):
        tmpl = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1,
                                       sample_signed=signed, out_int8=True, out_scale=1 / 64, t0=t0, batch_dt=bdt,
                                       beam_weights=weighted, coeff_table=table)
        assert (tmpl.workspace_bytes > 0) == table
        op = tmpl.instantiate(command_queue)
        if weighted:
            for m in range(M):
                op.set_beam_weights(m, g[m])
        op.ensure_all_bound()
        op.buffer("inSamples").set(command_queue, raw)
        op.buffer("delay_vals").set(command_queue, d)
        op()
        outs[table] = op.buffer("outData").get(command_queue)
    np.testing.assert_array_equal(outs[True], outs[False])
    ref = O.fused_beamform_int8(raw, d, Ctot, xeng_id=xeng, t0=t0, batch_dt=bdt, scale=1 / 64, signed=signed, gains=g)
    np.testing.assert_array_equal(outs[True], ref)
    assert np.abs(ref.astype(int)).max() >= 8


def golden_q14_words(case="q14rates_a256_m64"):
    """The reference-pinned Q14 image of golden G5 at config 4's shape: (B, C, M, A) words Wc | Ws << 16."""
    q = get(case, "q14").astype(np.int64)
    return ((q[..., 0] & 0xffff) | ((q[..., 1] & 0xffff) << 16)).astype(np.uint32)


def test_q14_coeffs_reference_golden_at_config4_shape(context, command_queue):
    """dt != 0 at config 4's shape (A = 256, M = 64, Ctot = 32768, X-engine 5, three batches) pinned by the reference
    (G5, tests/golden/make_golden.py): a delay model with rates whose advanced delay and phase are exact float32
    numbers at each batch time, so the reference's cpu_coeffs on the advanced model is the time extension evaluated
    exactly.  The generator's words equal rne(2^14 w) of those coefficients."""
    A, M, C, Ctot, xeng, B = (int(v) for v in get("q14rates_a256_m64", "dims"))
    t0, bdt = (float(v) for v in get("q14rates_a256_m64", "times"))
    got = generate(context, command_queue, get("q14rates_a256_m64", "delays"), B, C, Ctot, A, M, xeng, t0, bdt)
    np.testing.assert_array_equal(got, golden_q14_words())


@pytest.mark.parametrize("table", [True, False])
def test_fused_int8_config4_shape_reference_golden(context, command_queue, table):
    """The cfg4 int8 beams at dt != 0 -- the Q14 generator + LDS-DMA ring contraction (table) and the in-kernel
    phasor kernel -- from the reference's own coefficients (G5): exact integer products of Q14(golden), one rounding."""
    A, M, C, Ctot, xeng, B = (int(v) for v in get("q14rates_a256_m64", "dims"))
    t0, bdt = (float(v) for v in get("q14rates_a256_m64", "times"))
    T, scale = 256, 1.0 / 64
    raw = np.random.default_rng(11).integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8).view(np.int8)
    tmpl = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=True,
                                   out_int8=True, out_scale=scale, t0=t0, batch_dt=bdt, coeff_table=table)
    assert (tmpl.workspace_bytes > 0) == table
    op = tmpl.instantiate(command_queue)
    op.ensure_all_bound()
    op.buffer("inSamples").set(command_queue, raw)
    op.buffer("delay_vals").set(command_queue, get("q14rates_a256_m64", "delays"))
    op()
    q = op.buffer("outData").get(command_queue)
    g = get("q14rates_a256_m64", "q14").astype(np.int64)  # (B, C, M, A, [Wc, Ws])
    W = np.empty((B, C, 2 * A, 2 * M), np.int64)  # [[Wc, Ws], [-Ws, Wc]] blocks (coeff_generator_cpu.py:170-186)
    wc, ws = g[..., 0].transpose(0, 1, 3, 2), g[..., 1].transpose(0, 1, 3, 2)
    W[:, :, 0::2, 0::2], W[:, :, 0::2, 1::2], W[:, :, 1::2, 0::2], W[:, :, 1::2, 1::2] = wc, ws, -ws, wc
    X = O.reorder(raw).view(np.int8).astype(np.int64).reshape(B, 2, C, T, 2 * A)
    s = np.float32(np.float32(scale) * np.float32(2.0 ** -14))
    ref = np.clip(np.rint(np.matmul(X, W[:, None]).astype(np.float32) * s), -127, 127).astype(np.int8)
    np.testing.assert_array_equal(q, ref.reshape(q.shape))
    assert np.abs(ref.astype(int)).max() >= 8


def run_int8_wide(context, queue, raw, d, B, C, T, A, M, signed, table, g=None):
    Ctot, xeng, t0, bdt = 32768, 3, 2e-3, 256 * 2 * 32768 * TS
    tmpl = FusedBeamformerTemplate(context, B, C, Ctot, T, A, M, xeng_id=xeng, delay_channels=1, sample_signed=signed,
                                   out_int8=True, out_scale=1 / 64, t0=t0, batch_dt=bdt, beam_weights=g is not None,
                                   coeff_table=table)
    op = tmpl.instantiate(queue)
    if g is not None:
        for m in range(M):
            op.set_beam_weights(m, g[m])
    op.ensure_all_bound()
    op.buffer("inSamples").set(queue, raw)
    op.buffer("delay_vals").set(queue, d)
    op()
    return op.buffer("outData").get(queue)


@pytest.mark.parametrize("A,C,B,weighted", [(64, 600, 1, False), (128, 150, 2, True), (32, 270, 1, True),
                                            (32, 257, 1, False), (256, 300, 1, False)])
def test_int8_table_path_channel_groups(context, command_queue, A, C, B, weighted):
    """The table-driven slab kernel at 64 beams and T = 256 over many channels: ragged last channel groups (4 per
    workgroup, C % 4 = 1, 2; 8 at A = 256, C % 8 = 4), two batches, 1, 2, 4 and 8 k-steps (A = 32 ... 256), more
    workgroups than CUs.  Bitwise equal to
    the in-kernel-phasor slab kernel (itself pinned to the oracle above and in test_gpu_fullsize.py).  (These shapes
    also pinned the output-stationary LDS-DMA kernel measured in round 3, bf_wide_i8os.hip, diagnostic build.)"""
    M, T = 64, 256
    d = delays(1, M, A, seed=A + C)
    rng = np.random.default_rng(A * 3 + C)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8).view(np.int8)
    g = rng.uniform(-1.2, 1.2, (M, A)).astype(np.float32) if weighted else None
    got = run_int8_wide(context, command_queue, raw, d, B, C, T, A, M, True, True, g)
    ref = run_int8_wide(context, command_queue, raw, d, B, C, T, A, M, True, False, g)
    np.testing.assert_array_equal(got, ref)
    assert np.abs(ref.astype(int)).max() >= 8


def test_workspace_sizes_and_errors(context, command_queue):
    n = ctypes.c_size_t()
    _lib.call("bf_fused_workspace_bytes", 1, 4096, 256, 256, 64, _lib.FUSED_OUT_INT8 | _lib.FUSED_SIGNED,
              ctypes.byref(n))
    assert n.value == 4096 * 2 * 8 * 1024 * 4  # (c, 32-beam slab): 1024 Sp words, Sp = 8 k-steps
    for flags in (0, _lib.FUSED_OUT_INT8 | _lib.FUSED_INT8_VIA_F32, _lib.FUSED_OUT_INT8 | _lib.FUSED_PATH["generic"]):
        _lib.call("bf_fused_workspace_bytes", 1, 4096, 256, 256, 64, flags, ctypes.byref(n))
        assert n.value == 0, flags
    _lib.call("bf_fused_workspace_bytes", 8, 4096, 256, 64, 16, _lib.FUSED_OUT_INT8, ctypes.byref(n))
    assert n.value == 0  # config 3: the item kernel evaluates its phasors in-kernel
    _lib.call("bf_fused_workspace_bytes", 1, 8, 16, 300, 8, _lib.FUSED_OUT_INT8, ctypes.byref(n))
    assert n.value == 0  # more than 256 antennas: the 32-beam kernel keeps its in-kernel phasors
    with pytest.raises(_lib.BeamformerError, match="delay_channels"):
        _lib.call("bf_q14_coeffs", 1 << 20, 3, None, 1 << 20, 1, 4, 4, 1, 64, 0, TS, 0.0, 0.0, None)
