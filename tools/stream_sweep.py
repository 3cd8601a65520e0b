"""HBM stream-ceiling sweep (diagnostic library build/libbf_diag.so): the fused kernels' traffic mixes -- 2 GiB read +
2 GiB written (f32 beams, RW 1) and 2 GiB read + 0.5 GiB written (int8 beams, RW 4) -- streamed by the plain grid-stride
kernels bench.py takes its ceiling from and by chunked kernels (a workgroup reads a contiguous 4096 x U-byte chunk with
all its loads in flight, then writes the chunk's output), over grids, U, non-temporal loads / stores and chunk order.
Prints the time and rate of every variant and the best per mix.  usage: python tools/stream_sweep.py [GiB]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from dpdk_dc_sand_amd import _lib, accel  # noqa: E402

lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
V, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
lib.bf_diag_stream.argtypes = [V, V, S, S, I, I, V]
lib.bf_diag_stream_chunk.argtypes = [V, V, S, I, I, V]
ctx = accel.create_some_context()
q = ctx.create_command_queue()
nin = int(float(sys.argv[1]) * 2**30) if len(sys.argv) > 1 else 2**31
bufs = [(accel.DeviceArray(ctx, (nin,), np.uint8), accel.DeviceArray(ctx, (nin,), np.uint8)) for _ in range(2)]
rng = np.random.default_rng(1)
for xi, _ in bufs:  # random data: constant data runs at a higher clock (MI355X_MICROARCH.md)
    xi.set(q, rng.integers(0, 256, nin, dtype=np.uint8))


def timeit(fn, n=10):
    for i in range(2):
        assert fn(i) == 0
    e0, e1 = accel.Event(), accel.Event()
    q.finish()
    e0.record(q)
    for i in range(n):
        fn(i)
    e1.record(q)
    q.finish()
    return e1.time_since(e0) / n


NT = {0: "plain", 1: "nt-load", 2: "nt-store", 3: "nt-both"}
for rw in (1, 4):
    nout = nin // rw
    total = nin + nout
    res = []
    codes = [(1, "grid-stride plain"), (101, "grid-stride nt-store"), (102, "grid-stride nt-load"),
             (103, "grid-stride nt-both"), (8, "grid-stride U8")]
    if rw == 4:
        codes += [(200, "interleaved 4:1 nt-both"), (201, "interleaved 4:1 nt-load")]
    for grid in (1024, 2048, 4096):
        for code, nm in codes:
            t = timeit(lambda i: lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, nin, nout, grid, code,
                                                    q.handle))
            res.append((t, f"{nm:26s} grid {grid:5d}"))
    for order in (0, 1):
        for u in (4, 8, 16):
            for nt in (0, 1, 2, 3):
                for grid in (256, 512, 1024, 2048, 4096, 8192):
                    code = u + 100 * rw + 1000 * nt + 10000 * order
                    t = timeit(lambda i: lib.bf_diag_stream_chunk(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, nin, grid,
                                                                  code, q.handle))
                    res.append((t, f"chunk {'strided' if order == 0 else 'runs':7s} U {u:2d} {NT[nt]:8s} "
                                   f"grid {grid:5d}"))
    print(f"== read {nin / 2**30:.2f} GiB + write {nout / 2**30:.2f} GiB (RW {rw}) ==", flush=True)
    for t, nm in res:
        print(f"  {nm:50s} {t * 1e6:8.1f} us  {total / t / 1e9:7.1f} GB/s")
    best = sorted(res)[:5]
    print("  best:")
    for t, nm in best:
        print(f"    {nm:48s} {t * 1e6:8.1f} us  {total / t / 1e9:7.1f} GB/s")
