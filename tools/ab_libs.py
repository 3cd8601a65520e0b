"""GPU box: same-process A/B of one fused launch across several builds of libbf.so (e.g. an earlier round's tree
built under build/ab_<tag>/): the same device buffers, interleaved rounds, median per library; the int8 outputs of
every library are compared with the first one's (bitwise).
(AB_DELAYS=ops: the ops benchmark's delay model.  AB_WS=1: through bf_beamform_fused_ws with a workspace, as the
operator runs it -- config 4's int8 path is then the Q14 generator + the table-driven contraction.)
usage: python tools/ab_libs.py <workload cfg3|cfg4> <flags> <scale> <tag=path/to/libbf.so> ..."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

SHAPES = {"cfg2": (8, 4096, 256, 64, 1, 4096), "cfg3": (8, 4096, 256, 64, 16, 4096), "cfg4": (1, 4096, 256, 256, 64, 32768)}
wl, flags, scale = sys.argv[1], int(sys.argv[2], 0), float(sys.argv[3])
libs = []
for spec in sys.argv[4:]:
    tag, path = spec.split("=", 1)
    lib = ctypes.CDLL(os.path.abspath(path))
    f = lib.bf_beamform_fused
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 7 + \
                 [ctypes.c_double] * 3 + [ctypes.c_int, ctypes.c_float, ctypes.c_void_p]
    g = lib.bf_beamform_fused_ws
    g.restype = ctypes.c_int
    g.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p] + \
                 [ctypes.c_int] * 7 + [ctypes.c_double] * 3 + [ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
                                                               ctypes.c_size_t, ctypes.c_void_p]
    lib.bf_fused_workspace_bytes.argtypes = [ctypes.c_int] * 6 + [ctypes.POINTER(ctypes.c_size_t)]
    lib.bf_last_error.restype = ctypes.c_char_p
    libs.append((tag, lib))
B, C, T, A, M, Ctot = SHAPES[wl]
ts = 1 / 1712e6
ctx = accel.create_some_context(device=0)
q = ctx.create_command_queue()
nin = B * A * C * T * 4
outb = B * 2 * C * T * 2 * M * (1 if flags & 2 else 4)
rng = np.random.default_rng(1)
xs = [accel.DeviceArray(ctx, (nin,), np.uint8) for _ in range(2)]
for x in xs:
    x.set(q, rng.integers(0, 256, nin, dtype=np.uint8))
ys = [accel.DeviceArray(ctx, (outb,), np.uint8) for _ in range(2)]
d = np.zeros((M, A, 4), np.float32)
r = np.random.default_rng(0)
d[..., 0] = r.uniform(0, 10 * ts, (M, A))
d[..., 1] = r.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = r.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = r.uniform(-1, 1, (M, A))
T0 = 1e-3
if os.environ.get("AB_DELAYS") == "ops":  # tools/bench_ops.py's model: no rates, t0 = 0
    d[..., 1] = d[..., 3] = 0.0
    T0 = 0.0
dv = accel.DeviceArray(ctx, (M * A * 4,), np.float32)
dv.set(q, d.reshape(-1))
bdt = T * 2 * Ctot * ts


USE_WS = os.environ.get("AB_WS") == "1"
wsb = ctypes.c_size_t(0)
if USE_WS:
    libs[0][1].bf_fused_workspace_bytes(B, C, T, A, M, flags, ctypes.byref(wsb))
ws = accel.DeviceArray(ctx, (max(wsb.value, 16),), np.uint8)


def launch(lib, i):
    if USE_WS:
        st = lib.bf_beamform_fused_ws(xs[i % 2].ptr, dv.ptr, 1, None, ys[i % 2].ptr, B, C, T, A, M, Ctot, 0, ts, T0,
                                      bdt, flags, scale, ws.ptr, wsb.value, q.handle)
    else:
        st = lib.bf_beamform_fused(xs[i % 2].ptr, dv.ptr, 1, ys[i % 2].ptr, B, C, T, A, M, Ctot, 0, ts, T0, bdt,
                                   flags, scale, q.handle)
    if st != 0:
        raise RuntimeError(lib.bf_last_error().decode())


ref = None
for tag, lib in libs:
    launch(lib, 0)
    q.finish()
    out = ys[0].get(q)
    if ref is None:
        ref = out
    print(f"{tag}: output {'bitwise equal to' if np.array_equal(out, ref) else 'DIFFERS from'} {libs[0][0]}'s",
          flush=True)
res = {tag: [] for tag, _ in libs}
for rnd in range(int(os.environ.get("AB_ROUNDS", "7"))):
    for tag, lib in libs:
        for i in range(3):
            launch(lib, i)
        e0, e1 = accel.Event(), accel.Event()
        q.finish()
        e0.record(q)
        n = 20
        for i in range(n):
            launch(lib, i)
        e1.record(q)
        q.finish()
        res[tag].append(e1.time_since(e0) / n * 1e6)
for tag, v in res.items():
    v = sorted(v)
    print(f"{wl} flags {flags:#x} scale {scale}: {tag:10s} median {v[len(v) // 2]:7.1f} us  (min {v[0]:.1f}, "
          f"max {v[-1]:.1f}, {len(v)} rounds)", flush=True)
