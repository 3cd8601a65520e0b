"""GPU box, diagnostic build: same-process timing of the config-4 int8 contraction (w32r, bf_diag_w32_table mode
2000 + Mode bits) against its variants, interleaved over rounds (median of the per-round averages), plus a bitwise
check of every variant that must produce the product's beams.

    python tools/diag_w32r_ab.py [rounds] [mode ...]

Modes: 2000 (or 10000) + w32r's Mode bits, 3000 + w32r3's (the three-slot ring), 4000 + w32s's (loader waves).  Mode bits (bf_wide_i8.hip): 4 no stores, 8 no voltage DMA, 16 no table, 128 DMA through a zero-record descriptor (the
instructions issue, no bytes move), 256 the stores likewise, 512 one M0 per step's four DMA pieces, 1024 every channel's voltages from the workgroup's first
channel (L2 hits), 2048 every store into one of 256 8 KiB blocks (L2-resident writes)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
_lib._lib = lib
I, V, D = ctypes.c_int, ctypes.c_void_p, ctypes.c_double
lib.bf_diag_w32_table.argtypes = [I, V, V, V, V, I, I, I, I, I, I, D, V]
B, C, T, A, M, Ctot = 1, 4096, 256, 256, 64, 32768
ctx = accel.create_some_context(device=0)
q = ctx.create_command_queue()
nin, nout = B * A * C * T * 4, B * 2 * C * T * 2 * M
xs = [accel.DeviceArray(ctx, (nin,), np.uint8) for _ in range(2)]
for i, x in enumerate(xs):
    x.set(q, np.random.default_rng(1 + i).integers(0, 256, nin, dtype=np.uint8))
ys = [accel.DeviceArray(ctx, (nout,), np.uint8) for _ in range(2)]
d = np.zeros((M, A, 4), np.float32)
r = np.random.default_rng(0)
d[..., 0] = r.uniform(0, 10 / 1712e6, (M, A))
d[..., 1] = r.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = r.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = r.uniform(-1, 1, (M, A))
dv = accel.DeviceArray(ctx, (M * A * 4,), np.float32)
dv.set(q, d.reshape(-1))
tb = accel.DeviceArray(ctx, (B * C * (M // 32) * 1024 * 8 + 4096,), np.uint32)

EXACT = {2000, 2512, 3000, 4000}  # modes that must give the product's beams bitwise (w32r, M0-once w32r, w32r3)


def launch(mode, i):
    assert lib.bf_diag_w32_table(mode, xs[i % 2].ptr, dv.ptr, ys[i % 2].ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                                 q.handle) == 0


def timeit(mode, n=20):
    for i in range(3):
        launch(mode, i)
    e0, e1 = accel.Event(), accel.Event()
    q.finish()
    e0.record(q)
    for i in range(n):
        launch(mode, i)
    e1.record(q)
    q.finish()
    return e1.time_since(e0) / n * 1e6


launch(-1, 0)  # the table (kLayoutW32), once
q.finish()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
modes = [int(m) for m in sys.argv[2:]] or [2000, 2128, 2256, 2384, 2512, 2008, 2004, 2012]
ref = None
for mode in modes:
    if mode in EXACT:
        launch(mode, 0)
        q.finish()
        out = ys[0].get(q)
        if ref is None:
            ref = out
        print(f"mode {mode}: {'bitwise equal' if np.array_equal(out, ref) else 'DIFFERS'} to mode {modes[0]}",
              flush=True)
times = {m: [] for m in modes}
for k in range(rounds):
    for mode in modes:
        times[mode].append(timeit(mode))
    print(f"round {k}: " + "  ".join(f"{m}:{times[m][-1]:.1f}" for m in modes), flush=True)
for mode in modes:
    t = np.array(times[mode])
    print(f"mode {mode}: median {np.median(t):.1f} us  (min {t.min():.1f}, max {t.max():.1f})")
