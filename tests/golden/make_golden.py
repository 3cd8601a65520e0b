"""Generate golden vectors from the reference's own CPU oracles (run HERE only, never on the GPU box).

Run with the numpy-1.x interpreter so the reference's scalar arithmetic keeps its original float64
promotion:

    PYTHONDONTWRITEBYTECODE=1 /opt/conda/bin/python3.9 -W ignore tests/golden/make_golden.py

The reference modules used (read-only, imported from /root/reference/beamformer):
  * unit_test/coeff_generator_cpu.py:78-187   CoeffGenerator.cpu_coeffs   (coefficient contract)
  * unit_test/complex_mult_cpu.py:11-147      complex_mult                (beamform contract)
  * beamforming/reorder.py:6-84               reorder                     (reorder contract)
`numba.njit` is replaced by the identity decorator (numba is not importable here), so the oracles run as
plain Python with the same dtypes.  Inputs follow the reference tests' generators:
  * voltages:  np.random.default_rng(seed=2021).uniform(0, 255, shape).astype(np.uint8)
               (beamform_op_sequence_test.py:143-149, prebeamform_reorder_test.py:100-106)
  * delays:    (samples_delay*Ts, 0, phase, 0) for every (c, m, a) (beamform_coeff_test.py:86-90), plus
               non-uniform random delays (this file) to pin the per-(c, m, a) index mapping, plus (G5) delay models
               with rates advanced to each batch's time exactly in float32 (the dt != 0 pin).

Output: tests/golden/golden.npz (data only: inputs and the reference's outputs).
"""
import hashlib
import os
import sys
import types

numba = types.ModuleType("numba")
numba.njit = lambda f: f
sys.modules["numba"] = numba
sys.path.insert(0, "/root/reference/beamformer")

import numpy as np  # noqa: E402
from beamforming import reorder as ref_reorder  # noqa: E402
from unit_test import complex_mult_cpu  # noqa: E402
from unit_test.coeff_generator_cpu import CoeffGenerator  # noqa: E402

assert np.__version__.startswith("1."), "goldens must come from numpy 1.x (float64 scalar promotion)"

TS = 1 / 1712e6
OUT = {}


def uniform_delays(C, M, A, samples_delay=5, phase=np.pi / 2):
    vals = []
    for _ in range(C * M * A):
        vals += [np.single(samples_delay * TS), np.single(0.0), np.single(phase), np.single(0.0)]
    return np.array(vals).reshape(C, M, A, 4)


def random_delays(C, M, A, seed):
    rng = np.random.default_rng(seed)
    d = np.empty((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, (C, M, A))
    d[..., 1] = rng.uniform(-1e-9, 1e-9, (C, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (C, M, A))
    d[..., 3] = rng.uniform(-1.0, 1.0, (C, M, A))
    return d


def u8_voltages(shape):
    rng = np.random.default_rng(seed=2021)
    return rng.uniform(np.iinfo(np.uint8).min, np.iinfo(np.uint8).max, shape).astype(np.uint8)


def ref_coeffs(delays, B, P, C, Ctot, A, M, xeng_id):
    NB, S = 16, 16
    return CoeffGenerator(delays, B, P, C, Ctot, NB, S, A, M, xeng_id, TS).cpu_coeffs()


def sha(a):
    return np.array(hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest())


def put(name, **arrays):
    for k, v in arrays.items():
        OUT[f"{name}/{k}"] = np.asarray(v)


# Voltages come from default_rng(2021).uniform(...) (bit-identical under numpy 1.26 and 2.x, checked), so
# only their shape + sha256 are stored; tests regenerate them and check the digest.  Bit-exact outputs
# (reorder) are stored as sha256 digests; float outputs are stored whole.  Coefficients are replicated
# over (batch, pol) by the reference (coeff_generator_cpu.py:120-122); only the [0, 0] slice is stored
# after asserting the replication.


# ---- G1: pre-beamform reorder (prebeamform_reorder_test.py:33-122) -------------------------------
for name, (B, A, C, T) in {
    "reorder_cfg1": (1, 4, 64, 1024),      # BASELINE config 1
    "reorder_a5": (3, 5, 1024 // 5 // 4, 256),
    "reorder_a256": (3, 256, 1024 // 256 // 4, 256),   # C = 1
}.items():
    x = u8_voltages((B, A, C, T, 2, 2))
    out_shape = (B, 2, C, T // 16, 16, A, 2)
    y = ref_reorder.reorder(x, x.shape, out_shape)
    put(name, dims=np.array([B, A, C, T]), input_sha256=sha(x), output_sha256=sha(y), output_shape=np.array(y.shape))
    print(name, x.shape, "->", y.shape)

# ---- G2: coefficients (beamform_coeff_test.py:29-172, bit-exact contract) ------------------------
case = 0
for A in (4, 19, 64):
    for Ctot in (1024, 4096):
        for xeng_id in (0, 3):
            for kind in ("uniform", "random"):
                M, B, P = 2, 3, 2
                if A == 19 and Ctot == 1024 and kind == "random":
                    M = 1
                C = Ctot // A // 4
                d = uniform_delays(C, M, A) if kind == "uniform" else random_delays(C, M, A, 100 + case)
                w = ref_coeffs(d, B, P, C, Ctot, A, M, xeng_id)
                assert all((w[b, p] == w[0, 0]).all() for b in range(B) for p in range(P))
                put(f"coeff_{case:02d}", dims=np.array([B, P, C, Ctot, A, M, xeng_id]), delays=d, coeffs00=w[0, 0],
                    coeffs_sha256=sha(w), kind=np.array(kind))
                print(f"coeff_{case:02d}", kind, (A, Ctot, xeng_id, M), w.shape)
                case += 1

# ---- G3: beamform multiply, uniform delays (beamform_mult_kernel_test.py:119-269) ----------------
# complex_mult_cpu uses beam-0 coefficients for every beam; with the reference's
# uniform delays every beam is identical, which is the regime the reference pins.
for name, (B, A, M, Ctot, T) in {
    "mult_cfg1": (1, 4, 1, 1024, 1024),    # BASELINE config 1
    "mult_a4_m2": (2, 4, 2, 256, 256),
    "mult_a19_m1": (2, 19, 1, 1024, 256),
    "mult_a61_m2": (2, 61, 2, 1024, 256),
    "mult_a80_m1": (2, 80, 1, 1024, 256),
}.items():
    C = Ctot // A // 4
    d = uniform_delays(C, M, A)
    w = ref_coeffs(d, B, 2, C, Ctot, A, M, 0)
    x = u8_voltages((B, 2, C, T // 16, 16, A, 2))
    y = complex_mult_cpu.complex_mult(x, w, (B, 2, C, T // 16, 16, 2 * M))
    put(name, dims=np.array([B, A, M, Ctot, T, C]), delays=d, coeffs_sha256=sha(w), input_sha256=sha(x), output=y)
    print(name, x.shape, "->", y.shape)

# ---- G4: full OpSequence chain, config 1 (beamform_op_sequence_test.py:37-200) ------------------
B, A, M, Ctot, T = 1, 4, 1, 1024, 1024
C = Ctot // A // 4
d = uniform_delays(C, M, A)
raw = u8_voltages((B, A, C, T, 2, 2))
w = ref_coeffs(d, B, 2, C, Ctot, A, M, 0)
xr = ref_reorder.reorder(raw, raw.shape, (B, 2, C, T // 16, 16, A, 2))
y = complex_mult_cpu.complex_mult(xr, w, (B, 2, C, T // 16, 16, 2 * M))
put("opseq_cfg1", dims=np.array([B, A, M, Ctot, T, C]), delays=d, input_sha256=sha(raw), output=y)
print("opseq_cfg1", raw.shape, "->", y.shape)

# ---- G5: the time extension (dt != 0) against the reference's own formula -----------------------------------
# The Python reference reads only delay and phase (coeff_generator_cpu.py:125-164); a delay model with rates steers
# batch b at dt_b = t0 + b * batch_dt as tau_b = tau + tau_rate * dt_b, phi_b = phi + phi_rate * dt_b.
# The models here are built so that tau_b and phi_b are EXACT float32 numbers (tau on the 2^-51 grid inside
# [2^-28, 2^-27), tau_rate * dt_b a multiple of 2^-51; phi on the 2^-23 grid inside [1, 2) or (-2, -1], phi_rate *
# dt_b a multiple of 2^-23; t0 and batch_dt powers of two): the reference's cpu_coeffs on the advanced float32 model
# (tau_b, 0, phi_b, 0) is then the time extension evaluated exactly, so the fused operator's coefficients at dt != 0
# are pinned bit for bit by the reference's code, not by this framework's restatement.  Rates: up to ~2 sample
# periods of delay drift and ~0.5 rad of phase drift over the batches (the convention -- which term each rate enters,
# and its sign -- moves every coefficient).
def exact_rate_model(M, A, seed, t0, batch_dt, nb):
    rng = np.random.default_rng(seed)
    d = np.empty((1, M, A, 4), np.float32)
    tau_k = rng.integers(int(1.2 * 2 ** 23), int(1.8 * 2 ** 23), (M, A))          # tau = k 2^-51 in [2^-28, 2^-27)
    tau_m = rng.integers(-2 ** 17, 2 ** 17, (M, A)) * 2                              # rate = m 2^-44
    phi_k = rng.integers(int(1.1 * 2 ** 23), int(1.9 * 2 ** 23), (M, A)) * rng.choice([-1, 1], (M, A))
    phi_n = rng.integers(-2 ** 15, 2 ** 15, (M, A))                                   # phase rate = n 2^-16
    d[0, :, :, 0] = tau_k * 2.0 ** -51
    d[0, :, :, 1] = tau_m * 2.0 ** -44
    d[0, :, :, 2] = phi_k * 2.0 ** -23
    d[0, :, :, 3] = phi_n * 2.0 ** -16
    advanced = []
    for b in range(nb):
        dt = t0 + b * batch_dt
        tau_b = d[0, :, :, 0].astype(np.float64) + d[0, :, :, 1].astype(np.float64) * dt
        phi_b = d[0, :, :, 2].astype(np.float64) + d[0, :, :, 3].astype(np.float64) * dt
        assert (tau_b.astype(np.float32) == tau_b).all() and (phi_b.astype(np.float32) == phi_b).all()
        assert (np.abs(tau_b) >= 2.0 ** -28).all() and (np.abs(tau_b) < 2.0 ** -27).all()
        assert (np.abs(phi_b) >= 1.0).all() and (np.abs(phi_b) < 2.0).all()
        adv = np.zeros((M, A, 4), np.float32)
        adv[..., 0] = tau_b
        adv[..., 2] = phi_b
        advanced.append(adv)
    return d, advanced


for name, (A, M, C, Ctot, xeng_id, nb) in {
    "rates_a19_m2": (19, 2, 8, 1024, 3, 3),
    "rates_a64_m16": (64, 16, 4, 4096, 5, 3),
}.items():
    t0, batch_dt = 2.0 ** -7, 2.0 ** -6
    d, advanced = exact_rate_model(M, A, 500 + A, t0, batch_dt, nb)
    w = np.empty((nb, C, 2 * A, 2 * M), np.float32)
    for b, adv in enumerate(advanced):
        wb = ref_coeffs(np.broadcast_to(adv, (C, M, A, 4)).copy(), 1, 2, C, Ctot, A, M, xeng_id)
        w[b] = wb[0, 0]
    drift = float(np.abs(w[-1] - w[0]).max())
    assert drift > 0.1, drift  # the rates move the coefficients
    put(name, dims=np.array([A, M, C, Ctot, xeng_id, nb]), times=np.array([t0, batch_dt]), delays=d, coeffs=w)
    print(name, d.shape, "->", w.shape, "max drift over the batches", round(drift, 3))

# G5 at config 4's shape (A = 256, M = 64: the int8 path's Q14 generator and LDS-DMA contraction).  The float table
# would be 1.5 MB per channel pair; the int8 contract only needs its Q14 image, W = rne(2^14 w) of the reference's
# float32 coefficient (oracle.quantise_coeffs), stored as int16 (Wc, Ws) per (batch, channel, beam, antenna).
for name, (A, M, C, Ctot, xeng_id, nb) in {"q14rates_a256_m64": (256, 64, 2, 32768, 5, 3)}.items():
    t0, batch_dt = 2.0 ** -7, 2.0 ** -6
    d, advanced = exact_rate_model(M, A, 700 + A, t0, batch_dt, nb)
    q = np.empty((nb, C, M, A, 2), np.int16)
    for b, adv in enumerate(advanced):
        wb = ref_coeffs(np.broadcast_to(adv, (C, M, A, 4)).copy(), 1, 2, C, Ctot, A, M, xeng_id)[0, 0]
        qb = np.rint(wb.astype(np.float64) * 16384.0).astype(np.int64)  # (C, 2A, 2M)
        q[b, ..., 0] = qb[:, 0::2, 0::2].transpose(0, 2, 1)  # Wc: W[2a][2m]
        q[b, ..., 1] = qb[:, 0::2, 1::2].transpose(0, 2, 1)  # Ws: W[2a][2m + 1]
    put(name, dims=np.array([A, M, C, Ctot, xeng_id, nb]), times=np.array([t0, batch_dt]), delays=d, q14=q)
    print(name, d.shape, "->", q.shape)

path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz")
np.savez_compressed(path, **OUT)
print("wrote", path, os.path.getsize(path), "bytes; sha256",
      hashlib.sha256(open(path, "rb").read()).hexdigest()[:16])
