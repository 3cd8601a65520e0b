"""A/B of the config-4 Q14 table generator (q14_table_kernel, kLayoutW32) -- or, with GEN_AB_WHAT=launch, of the whole
int8 wide launch (generator + contraction, bf_diag_w32_launch) -- under the diagnostic build's measurement env knobs,
same process, interleaved rounds, and a bitwise check of the tables (or int8 beams) they write.
Usage: GEN_AB="name=ENV:value,..." python tools/diag_gen_ab.py [B C T A M]
e.g.   GEN_AB="two-sided=BF_Q14_UNIT:0,margin=BF_Q14_UNIT:1"
       GEN_AB_WHAT=launch GEN_AB="serial=BF_W32_OVERLAP:1,2 chunks=BF_W32_OVERLAP:2" (generator chunks on a second
       stream beside the contraction chunks)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
V, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
lib.bf_diag_w32_table.argtypes = [I, V, V, V, V, I, I, I, I, I, I, D, V]
lib.bf_diag_w32_launch.argtypes = [V, V, V, V, I, I, I, I, I, I, D, V]
WHAT = os.environ.get("GEN_AB_WHAT", "gen")
B, C, T, A, M = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (1, 4096, 256, 256, 64))]
Ctot = int(os.environ.get("DIAG_CTOT", "32768"))
forms = [f.split("=") for f in os.environ.get("GEN_AB", "margin=BF_Q14_UNIT:1,two-sided=BF_Q14_UNIT:0").split(",")]
ctx = accel.create_some_context()
q = ctx.create_command_queue()
rng = np.random.default_rng(1)
d = np.zeros((M, A, 4), np.float32)
d[..., 0] = rng.uniform(0, 10 / 1712e6, (M, A))
d[..., 1] = rng.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = rng.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = rng.uniform(-1, 1, (M, A))
dv = accel.DeviceArray(ctx, d.shape, np.float32)
dv.set(q, d)
nin, nout = (B * A * C * T * 4, B * 2 * C * T * 2 * M) if WHAT == "launch" else (16, 16)
x = accel.DeviceArray(ctx, (nin,), np.uint8)
x.set(q, rng.integers(0, 256, nin, dtype=np.uint8))
y = accel.DeviceArray(ctx, (nout,), np.int8)
words = B * C * ((M + 31) // 32) * (1024 * 8 + 256)
tb = accel.DeviceArray(ctx, (words + 4096,), np.uint32)


def setenv(form):
    k, v = form[1].split(":")
    os.environ[k] = v


def gen():
    if WHAT == "launch":
        e = lib.bf_diag_w32_launch(x.ptr, dv.ptr, y.ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)
    else:
        e = lib.bf_diag_w32_table(-1, x.ptr, dv.ptr, y.ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)
    assert e == 0, lib.bf_last_error()


tables = {}
for f in forms:
    setenv(f)
    _lib.call("bf_memset", tb.ptr, 0, tb.nbytes, q.handle)
    _lib.call("bf_memset", y.ptr, 0, y.nbytes, q.handle)
    gen()
    q.finish()
    tables[f[0]] = (y if WHAT == "launch" else tb).get(q).copy()
ref = forms[0][0]
for f in forms[1:]:
    same = np.array_equal(tables[ref], tables[f[0]])
    print(f"  {'int8 beams' if WHAT == 'launch' else 'table'} {f[0]} vs {ref}: {'bitwise equal' if same else 'DIFFERENT'}", flush=True)
res = {f[0]: [] for f in forms}
for r in range(int(os.environ.get("DIAG_ROUNDS", "7"))):
    for f in forms:
        setenv(f)
        for _ in range(3):
            gen()
        e0, e1 = accel.Event(), accel.Event()
        q.finish()
        e0.record(q)
        for _ in range(20):
            gen()
        e1.record(q)
        q.finish()
        res[f[0]].append(e1.time_since(e0) / 20)
for name, ts in res.items():
    ts = sorted(ts)
    print(f"  {WHAT} {name:24s}: median {ts[len(ts) // 2] * 1e6:7.1f} us  (all {', '.join(f'{t * 1e6:.1f}' for t in ts)})",
          flush=True)
