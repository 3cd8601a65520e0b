"""Write tests/golden/c_smoke.bin: the input and expected outputs tests/c/bf_smoke.c checks the C ABI against.

Generated from the oracle (oracle/, itself pinned to the reference's CPU oracles by golden.npz), so the C caller is
held to the same contracts as the Python tests:
  * reorder: bit-exact (reorder.py:40-42);
  * coefficients: bit-exact (coeff_generator_cpu.py:120-186);
  * fused int8 beams: bit-exact to the Q14 integer contract (oracle.fused_beamform_int8);
  * fused f32 beams: within the stated fp32 tolerance (tests/tolerance.py), per element.
Layout (little-endian): int32[8] B, A, C, T, M, Ctot, xeng_id, signed; float64[3] Ts, t0, batch_dt;
float32 out_scale; then raw u8 (B,A,C,T,2,2); delays f32 (C,M,A,4); reorder u8 (B,2,C,T/16,16,A,2);
coeffs f32 (1,1,C,2A,2M); beams_i8 (B,2,C,T/16,16,2M); beams_f32 and tol_f32 f32 (B,2,C,T/16,16,2M).
The delay model has zero rates and is the same for every channel, so it serves both the per-channel coefficient
generator and the fused operator's compact form, and every streamed frame has the same expected beams.

    python tests/golden/make_c_fixture.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))
import oracle as O  # noqa: E402
from tolerance import fp32_tolerance  # noqa: E402

B, A, C, T, M, Ctot, XENG = 2, 19, 5, 32, 3, 40, 2
TS, T0, BDT, SCALE = O.TS_MEERKAT, 0.0, 0.0, 1.0 / 32


def main():
    rng = np.random.default_rng(20211)
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)
    d1 = np.zeros((1, M, A, 4), np.float32)
    d1[..., 0] = rng.uniform(0, 10 * TS, (M, A))
    d1[..., 2] = rng.uniform(-np.pi, np.pi, (M, A))
    dC = np.ascontiguousarray(np.broadcast_to(d1, (C, M, A, 4)))
    reordered = O.reorder(raw)
    coeffs = O.coeffs(dC, 1, 1, C, Ctot, A, M, XENG)
    q = O.fused_beamform_int8(raw, d1, Ctot, xeng_id=XENG, t0=T0, batch_dt=BDT, scale=SCALE)
    y = O.fused_beamform(raw, d1, Ctot, xeng_id=XENG, t0=T0, batch_dt=BDT)
    w = O.fused_tables(d1, B, C, Ctot, A, xeng_id=XENG, t0=T0, batch_dt=BDT)
    tol = fp32_tolerance(y, reordered, w).astype(np.float32)
    with open(os.path.join(HERE, "c_smoke.bin"), "wb") as f:
        f.write(np.array([B, A, C, T, M, Ctot, XENG, 0], "<i4").tobytes())
        f.write(np.array([TS, T0, BDT], "<f8").tobytes())
        f.write(np.array([SCALE], "<f4").tobytes())
        for a in (raw, dC, reordered, coeffs, q, y, tol):
            f.write(np.ascontiguousarray(a).tobytes())
    print("wrote c_smoke.bin", os.path.getsize(os.path.join(HERE, "c_smoke.bin")), "bytes")


if __name__ == "__main__":
    main()
