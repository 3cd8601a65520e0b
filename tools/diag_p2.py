"""GPU box: where the persistent float wide kernel (beamform_fused_wide_p2_kernel) differs from the generic kernel
at config 4's item shape -- counts of wrong beams by pol / channel / sample (wave, lane, i) / beam, for int8 and
uint8 samples.  usage: python tools/diag_p2.py [C] [M]"""
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dpdk_dc_sand_amd import accel  # noqa: E402
from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate  # noqa: E402

TS = 1 / 1712e6
C = int(sys.argv[1]) if len(sys.argv) > 1 else 8
M = int(sys.argv[2]) if len(sys.argv) > 2 else 64
A, T, B, Ctot = 256, 256, 1, 32768
ctx = accel.create_some_context()
q = ctx.create_command_queue()
rng = np.random.default_rng(C)
d = np.zeros((1, M, A, 4), np.float32)
d[..., 0] = rng.uniform(0, 10 * TS, (M, A))
d[..., 1] = rng.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = rng.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = rng.uniform(-1, 1, (M, A))


def run(raw, signed, path):
    op = FusedBeamformerTemplate(ctx, B, C, Ctot, T, A, M, sample_period=TS, delay_channels=1, sample_signed=signed,
                                 t0=2e-3, batch_dt=T * 2 * Ctot * TS, kernel_path=path).instantiate(q)
    op.ensure_all_bound()
    op.buffer("inSamples").set(q, raw)
    op.buffer("delay_vals").set(q, d)
    op()
    return op.buffer("outData").get(q).astype(np.float64)


for signed in (True, False):
    for pattern in ("random", "const"):
        if pattern == "random":
            raw = np.frombuffer(rng.bytes(B * A * C * T * 4), np.int8 if signed else np.uint8).reshape(B, A, C, T, 2, 2)
        else:
            raw = np.full((B, A, C, T, 2, 2), 3, np.int8 if signed else np.uint8)
        y = run(raw, signed, "auto")
        g = run(raw, signed, "generic")
        err = np.abs(y - g)
        bad = np.argwhere(err > 1e-2 * (1 + np.abs(g)))
        print(f"signed={signed} {pattern}: max |dy| {err.max():.3e} (max |y| {np.abs(g).max():.3e}); "
              f"{len(bad)} of {err.size} beams off", flush=True)
        if len(bad):
            b_, p_, c_, tb, t16, col = bad.T
            t = tb * 16 + t16
            for nm, v in {"pol": p_, "c": c_, "wave (t // 32)": t // 32, "tl ((t % 32) // 2)": (t % 32) // 2,
                          "i (t % 2)": t % 2, "slab": col // 64, "tile ((col % 64) // 32)": (col % 64) // 32,
                          "col % 32": col % 32}.items():
                cnt = collections.Counter(v.tolist())
                print(f"     {nm:22s} {len(cnt):5d} distinct; top {cnt.most_common(8)}", flush=True)
