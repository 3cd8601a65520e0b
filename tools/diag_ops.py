"""A/B timing of the drop-in chain's stand-alone kernels (diagnostic library build/libbf_diag.so): bf_reorder cache
policy x time chunk, bf_coeff_gen block form (non-temporal / plain stores) vs the per-(a, m) forms.  Variants are
selected through the diagnostic build's environment knobs (csrc/bf_reorder.hip, csrc/bf_coeff.hip); every variant's
output is checked equal to the first one's.  Interleaved rounds, HIP-event averages.

    python tools/diag_ops.py [--rounds 3] [--only cfg3,cfg4]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

TS = 1 / 1712e6
CONFIGS = {"cfg3": dict(A=64, M=16, C=4096, Ctot=4096, T=256, B=8),
           "cfg4": dict(A=256, M=64, C=4096, Ctot=32768, T=256, B=1)}
V, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double


def timeit(q, fn, n=10):
    for _ in range(3):
        fn()
    e0, e1 = accel.Event(), accel.Event()
    q.finish()
    e0.record(q)
    for _ in range(n):
        fn()
    e1.record(q)
    q.finish()
    return e1.time_since(e0) / n


def with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--only", default="cfg3,cfg4")
    args = p.parse_args()
    lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
    lib.bf_reorder.argtypes = [V, V, I, I, I, I, V]
    lib.bf_coeff_gen.argtypes = [V, V, I, I, I, I, I, I, I, D, V]
    ctx = accel.create_some_context()
    q = ctx.create_command_queue()
    rng = np.random.default_rng(0)
    for name in args.only.split(","):
        c = CONFIGS[name]
        A, M, C, Ctot, T, B = c["A"], c["M"], c["C"], c["Ctot"], c["T"], c["B"]
        vb = B * A * C * T * 4
        raw = accel.DeviceArray(ctx, (vb,), np.uint8)
        raw.set(q, rng.integers(0, 256, vb, dtype=np.uint8))
        ro = accel.DeviceArray(ctx, (vb,), np.uint8)
        reorder = {f"nt{nt} tt{tt}": {"BF_REORDER_NT": str(nt), "BF_REORDER_TT": str(tt)}
                   for nt in [int(v) for v in os.environ.get("REORDER_NT", "0,1,2,3").split(",")]
                   for tt in [int(v) for v in os.environ.get("REORDER_TT", "32,64,128,256").split(",")]}
        res = {k: [] for k in reorder}
        ref = None
        for k, env in reorder.items():  # equality first
            with_env(env, lambda: lib.bf_reorder(raw.ptr, ro.ptr, B, A, C, T, q.handle))
            got = ro.get(q)
            if ref is None:
                ref = got
            assert np.array_equal(got, ref), k
        del ref, got
        for _ in range(args.rounds):
            for k, env in reorder.items():
                res[k].append(with_env(env, lambda: timeit(q, lambda: lib.bf_reorder(raw.ptr, ro.ptr, B, A, C, T,
                                                                                       q.handle))))
        for k, ts in res.items():
            t = sorted(ts)[len(ts) // 2]
            print(f"{name} reorder {k:12s} median {t * 1e6:8.1f} us  {2 * vb / t / 1e9:7.1f} GB/s", flush=True)
        del raw, ro

        d = np.zeros((C, M, A, 4), np.float32)
        d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
        d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])
        dv = accel.DeviceArray(ctx, d.shape, np.float32)
        dv.set(q, d)
        tb = B * 2 * C * 2 * A * 2 * M * 4
        out = accel.DeviceArray(ctx, (tb // 4,), np.float32)
        forms = {"block nt": {"BF_COEFF_NT": "1"}, "block plain": {"BF_COEFF_NT": "0"},
                 "block nt bpg4": {"BF_COEFF_NT": "1", "BF_COEFF_BPG": "4"},
                 "block plain bpg4": {"BF_COEFF_NT": "0", "BF_COEFF_BPG": "4"},
                 "block nt bpg1": {"BF_COEFF_NT": "1", "BF_COEFF_BPG": "1"},
                 "block plain bpg1": {"BF_COEFF_NT": "0", "BF_COEFF_BPG": "1"},
                 "per-(a,m) thread": {"BF_COEFF_FORM": "thread"}, "per-(a,m) tile": {"BF_COEFF_FORM": "tile"}}
        ref = None
        for k, env in forms.items():
            with_env(env, lambda: lib.bf_coeff_gen(dv.ptr, out.ptr, B, 2, C, Ctot, A, M, 0, TS, q.handle))
            got = out.get(q)
            if ref is None:
                ref = got
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), k
        del ref, got
        res = {k: [] for k in forms}
        for _ in range(args.rounds):
            for k, env in forms.items():
                res[k].append(with_env(env, lambda: timeit(q, lambda: lib.bf_coeff_gen(
                    dv.ptr, out.ptr, B, 2, C, Ctot, A, M, 0, TS, q.handle))))
        alg = tb + C * M * A * 16
        for k, ts in res.items():
            t = sorted(ts)[len(ts) // 2]
            print(f"{name} coeff_gen {k:18s} median {t * 1e6:8.1f} us  {alg / t / 1e9:7.1f} GB/s", flush=True)
        del dv, out


if __name__ == "__main__":
    main()
