"""GPU box: where the LDS-DMA ring contraction (w32r, diag mode 2000) differs from the table kernel (w32t, mode 900)
on the same kLayoutW32 table and input.  Prints the mismatch count per index component of the output
(B, P, C, T/16, 16, 2M) int8.  Usage: python tools/diag_w32r.py [runs] [modes...]"""
import collections
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
x = accel.DeviceArray(ctx, (nin,), np.uint8)
x.set(q, np.random.default_rng(1).integers(0, 256, nin, dtype=np.uint8))
y = accel.DeviceArray(ctx, (nout,), np.uint8)
d = np.zeros((M, A, 4), np.float32)
r = np.random.default_rng(0)
d[..., 0] = r.uniform(0, 10 / 1712e6, (M, A))
d[..., 1] = r.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = r.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = r.uniform(-1, 1, (M, A))
dv = accel.DeviceArray(ctx, (M * A * 4,), np.float32)
dv.set(q, d.reshape(-1))
tb = accel.DeviceArray(ctx, (B * C * (M // 32) * 1024 * 8 + 4096,), np.uint32)


def run(mode):
    _lib.call("bf_memset", y.ptr, 0, nout, q.handle)
    assert lib.bf_diag_w32_table(mode, x.ptr, dv.ptr, y.ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle) == 0
    q.finish()
    return y.get(q).view(np.int8).reshape(B, 2, C, T, 2 * M)


run(-1)
ref = run(900)
runs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
modes = [int(m) for m in sys.argv[2:]] or [2000]
for mode in modes:
    for k in range(runs):
        out = run(mode)
        bad = np.argwhere(out != ref)
        print(f"mode {mode} run {k}: {len(bad)} of {out.size} bytes differ", flush=True)
        if len(bad) == 0:
            continue
        b_, p, c, t, col = bad.T
        pair = t // 2
        comp = {"pol": p, "kc (c % 8)": c % 8, "c": c, "wave": (pair // 16) % 4, "pass": pair // 64, "tl": pair % 16,
                "i": t % 2, "slab": col // 64, "tile": (col % 64) // 32, "h": (col % 32) // 8, "r": (col % 8) // 2,
                "re/im": col % 2, "grp (c // 8)": c // 8}
        for name, v in comp.items():
            cnt = collections.Counter(v.tolist())
            top = cnt.most_common(12)
            print(f"   {name:12s} {len(cnt):5d} distinct; top {top}")
        print("   first:", bad[:5].tolist(), "got", out[tuple(bad[:5].T)].tolist(), "want", ref[tuple(bad[:5].T)].tolist())
