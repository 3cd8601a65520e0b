"""Clock ramp: average int8 fused launch time over n back-to-back launches, from a fresh process (bench-like
inputs vs all-zero voltages).  The first ~30 ms of load run slower while the clocks ramp."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np
from dpdk_dc_sand_amd import accel
from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate

TS = 1 / 1712e6
ctx = accel.create_some_context()
q = ctx.create_command_queue()
A, M, C, T, B = 64, 16, 4096, 256, 8
mk = lambda dt: FusedBeamformerTemplate(ctx, B, C, C, T, A, M, sample_period=TS, delay_channels=1, sample_signed=True,
                                        out_int8=True, out_scale=1 / 64, t0=0.0, batch_dt=dt)
tmpl = mk(T * 2 * C * TS)
rng = np.random.default_rng(1)
d = np.zeros(tmpl.delay_shape, np.float32)
d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
d[..., 1] = rng.uniform(-1e-9, 1e-9, d.shape[:-1])
d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])
d[..., 3] = rng.uniform(-1, 1, d.shape[:-1])
dz = np.zeros_like(d)
dz[..., 0] = 1e-10
variants = {}
hosts = [rng.integers(-128, 128, size=tmpl.input_shape, dtype=np.int8) for _ in range(2)]
zero = np.zeros(tmpl.input_shape, np.int8)


def build(t, dv, data):
    ops = []
    for h in data:
        op = t.instantiate(q)
        op.ensure_all_bound()
        op.buffer("inSamples").set(q, h)
        op.buffer("delay_vals").set(q, dv)
        ops.append(op)
    return ops


variants["bench"] = build(tmpl, d, hosts)
variants["zero-delay"] = build(tmpl, dz, hosts)
variants["zero-data"] = build(tmpl, d, [zero, zero])
variants["batch_dt=0"] = build(mk(0.0), d, hosts)


def timeit(ops, n=20):
    for i in range(3):
        ops[i % 2]()
    e0, e1 = accel.Event(), accel.Event()
    q.finish(); e0.record(q)
    for i in range(n):
        ops[i % 2]()
    e1.record(q); q.finish()
    return e1.time_since(e0) / n

for n in (5, 20, 50, 200, 20, 5):
    print(f"n={n:4d} bench {timeit(variants['bench'], n)*1e6:8.1f} us   zero-data {timeit(variants['zero-data'], n)*1e6:8.1f} us", flush=True)
