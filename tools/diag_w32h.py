"""A/B of the config-4 int8 launch (generator + contraction, bf_diag_w32_launch in build/libbf_diag.so): the
halved-image kernel (beamform_fused_i8_w32h_kernel) against the table kernel
(q14_table_kernel + beamform_fused_i8_w32t_kernel, the product form; BF_W32H=1 selects the halved-image launch in the
diagnostic build), the parts alone and the 64-beam-wave forms (w64h), same process, interleaved, random voltages.
The int8 beams of the two must be bitwise equal.  Usage: python tools/diag_w32h.py [B C T A M] (default cfg4)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
V, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
lib.bf_diag_w32_launch.argtypes = [V, V, V, V, I, I, I, I, I, I, D, V]
lib.bf_diag_w32_table.argtypes = [I, V, V, V, V, I, I, I, I, I, I, D, V]
B, C, T, A, M = [int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (1, 4096, 256, 256, 64))]
Ctot = int(os.environ.get("DIAG_CTOT", "32768"))
ctx = accel.create_some_context()
q = ctx.create_command_queue()
nin, nout = B * A * C * T * 4, B * 2 * C * T * 2 * M
rng = np.random.default_rng(1)
xs = []
for _ in range(2):
    x = accel.DeviceArray(ctx, (nin,), np.uint8)
    x.set(q, rng.integers(0, 256, nin, dtype=np.uint8))
    xs.append(x)
ys = [accel.DeviceArray(ctx, (nout,), np.int8) for _ in range(2)]
d = np.zeros((M, A, 4), np.float32)
d[..., 0] = rng.uniform(0, 10 / 1712e6, (M, A))
d[..., 1] = rng.uniform(-1e-9, 1e-9, (M, A))
d[..., 2] = rng.uniform(-np.pi, np.pi, (M, A))
d[..., 3] = rng.uniform(-1, 1, (M, A))
dv = accel.DeviceArray(ctx, d.shape, np.float32)
dv.set(q, d)
words = B * C * ((M + 31) // 32) * (1024 * 8 + 256)
tb = accel.DeviceArray(ctx, (words + 4096,), np.uint32)


PARTS = {"gen W32 (q14_table_kernel)": -1, "gen W32H (q14_image_kernel)": -2, "contract w32t": 900}
for m, name in ((16, "w32h: frag_im halved (wrong)"),):  # (stamps: below)
    PARTS[name] = 960 + m
PARTS.update({"contract w64h (16 ch, NB 4)": 1200, "contract w64h (8 ch, NB 4)": 1201, "contract w64h (16 ch, NB 2)": 1202,
              "w64h no MFMA": 1210, "w64h no stores": 1211, "w64h no loads": 1212, "w64h no loads, no stores": 1213,
              "w64h no image DMA": 1215, "w64h reg-staged table NB2": 1220, "w64h reg-staged table NB4": 1221,
              "w64h no image DMA NB2": 1222})
if os.environ.get("W64_ONLY"):
    PARTS = {k: v for k, v in PARTS.items() if v >= 1200 or v == 900}
tbh = accel.DeviceArray(ctx, (words + 4096,), np.uint32)  # a kLayoutW32H table for the w32h contraction alone


def launch(i, form):
    os.environ.pop("BF_W32H", None)
    if form in PARTS or form == "contract w32h":
        mode = PARTS.get(form, 960)
        e = lib.bf_diag_w32_table(mode, xs[i % 2].ptr, dv.ptr, ys[i % 2].ptr, tbh.ptr if mode == -2 or mode >= 960 else tb.ptr,
                                  B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)
        assert e == 0, lib.bf_last_error()
        return
    if form == "w32h":
        os.environ["BF_W32H"] = "1"
    e = lib.bf_diag_w32_launch(xs[i % 2].ptr, dv.ptr, ys[i % 2].ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                               q.handle)
    assert e == 0, lib.bf_last_error()


def timeit_mode(mode, n=20):
    def run(i):
        tbl = tbh.ptr if mode == -2 or mode >= 960 else tb.ptr
        assert lib.bf_diag_w32_table(mode, xs[i % 2].ptr, dv.ptr, ys[i % 2].ptr, tbl, B, C, T, A, M, Ctot, 1 / 1712e6,
                                     q.handle) == 0
    for i in range(3):
        run(i)
    e0, e1 = accel.Event(), accel.Event()
    q.finish()
    e0.record(q)
    for i in range(n):
        run(i)
    e1.record(q)
    q.finish()
    return e1.time_since(e0) / n


def timeit(form, n=20):
    for i in range(3):
        launch(i, form)
    e0, e1 = accel.Event(), accel.Event()
    q.finish()
    e0.record(q)
    for i in range(n):
        launch(i, form)
    e1.record(q)
    q.finish()
    return e1.time_since(e0) / n


outs = {}
for form in ("w32t", "w32h"):
    _lib.call("bf_memset", ys[0].ptr, 0, nout, q.handle)
    launch(0, form)
    q.finish()
    outs[form] = ys[0].get(q).copy()
same = np.array_equal(outs["w32t"], outs["w32h"])
print(f"shape B={B} C={C} T={T} A={A} M={M}: w32h vs w32t int8 beams "
      f"{'bitwise equal' if same else 'DIFFERENT (%d bytes)' % int((outs['w32t'] != outs['w32h']).sum())}; "
      f"max |q| {np.abs(outs['w32t'].astype(int)).max()}", flush=True)
lib.bf_diag_w32_table(-1, xs[0].ptr, dv.ptr, ys[0].ptr, tb.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)
lib.bf_diag_w32_table(-2, xs[0].ptr, dv.ptr, ys[0].ptr, tbh.ptr, B, C, T, A, M, Ctot, 1 / 1712e6, q.handle)
for mode in (1200, 1202, 1220, 1221):  # the 64-beam-wave contraction on the same input and table: bitwise equal to w32t
    _lib.call("bf_memset", ys[0].ptr, 0, nout, q.handle)
    assert lib.bf_diag_w32_table(mode, xs[0].ptr, dv.ptr, ys[0].ptr, tbh.ptr, B, C, T, A, M, Ctot, 1 / 1712e6,
                                 q.handle) == 0, lib.bf_last_error()
    got = ys[0].get(q)
    print(f"  mode {mode} vs w32t: {'bitwise equal' if np.array_equal(got, outs['w32t']) else 'DIFFERENT (%d bytes)' % int((got != outs['w32t']).sum())}", flush=True)
    bad = np.flatnonzero(got != outs["w32t"])
    if bad.size:  # (b, p, c, t, col) of the differing bytes
        col = bad % (2 * M); t_ = (bad // (2 * M)) % T; c_ = (bad // (2 * M * T)) % C; p_ = (bad // (2 * M * T * C)) % 2
        for name, v in (("col", col), ("sample", t_), ("channel", c_), ("pol", p_)):
            u, n = np.unique(v, return_counts=True)
            print(f"    {name}: {len(u)} distinct; top {list(zip(u[np.argsort(-n)][:8].tolist(), np.sort(n)[::-1][:8].tolist()))}")
        print(f"    channel % 16: {np.unique(c_ % 16, return_counts=True)}; sample // 16: {np.unique(t_ // 16, return_counts=True)}")
        d = got[bad].astype(int) - outs["w32t"][bad].astype(int)
        print(f"    diff values: {np.unique(d, return_counts=True)}")
res = {f: [] for f in (() if os.environ.get("W64_ONLY") else ("w32t", "w32h", "contract w32h")) + tuple(PARTS)}
for r in range(int(os.environ.get("DIAG_ROUNDS", "5"))):
    for f in res:
        res[f].append(timeit(f))
for f, ts in res.items():
    ts = sorted(ts)
    print(f"  {f:28s}: median {ts[len(ts) // 2] * 1e6:8.1f} us  (all: "
          f"{', '.join(f'{t * 1e6:.1f}' for t in ts)})")

# per-wave phase cycles of the halved-image contraction (s_memtime, Mode 128)
lib.bf_diag_w32h_stamps.argtypes = [V, V, V, V, I, I, I, I, I, V]
ngrid = ((B * ((C + 7) // 8) + 7) // 8 * 8) * ((M + 31) // 32)
st = accel.DeviceArray(ctx, (ngrid * 4 * 4,), np.uint64)
_lib.call("bf_memset", st.ptr, 0, ngrid * 4 * 4 * 8, q.handle)
assert lib.bf_diag_w32h_stamps(xs[0].ptr, tbh.ptr, ys[0].ptr, st.ptr, B, C, T, A, M, q.handle) == 0
v = st.get(q).reshape(ngrid, 4, 4).astype(np.float64)
v = v[v.sum(axis=(1, 2)) > 0]
tot = v.sum(axis=2)
print(f"stamps over {v.shape[0]} workgroups x 4 waves (cycles per wave, mean): " + ", ".join(
    f"{n} {v[..., k].mean():.0f} ({100 * v[..., k].sum() / tot.sum():.1f} %)" for k, n in
    enumerate(("voltage wait", "steps (MFMA + LDS)", "requant + stores", "channel barrier"))))

# static-priority knobs (BF_KNOB): 1 | bit << 8 = prio 1 for w32t workgroups with that blockIdx bit; 2 = w64h waves 4-7
if os.environ.get("KNOB_AB"):
    kres = {}
    for r in range(5):
        for name, mode, knob in (("w32t", 900, 0), ("w32t prio bit3", 900, 1 | 3 << 8), ("w32t prio bit8", 900, 1 | 8 << 8),
                                 ("w32t prio bit0", 900, 1), ("w64h NB2", 1202, 0), ("w64h NB2 prio 4-7", 1202, 2)):
            os.environ["BF_KNOB"] = str(knob)
            kres.setdefault(name, []).append(timeit_mode(mode))
    os.environ.pop("BF_KNOB", None)
    for name, ts in kres.items():
        ts = sorted(ts)
        print(f"  knob {name:24s}: median {ts[len(ts) // 2] * 1e6:8.1f} us")

