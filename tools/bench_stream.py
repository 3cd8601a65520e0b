"""Streaming ingest measurement: sustained Gsamples/s of host frames through
H2D -> fused beamform (int8 beams) -> D2H, against the PCIe copy rates measured on the same pinned buffers.

    python tools/bench_stream.py [--frames 24] [--depth 4] [--out-float]

Config 5: frames of config 3, (1, 64, 4096, 256, 2, 2) int8 = 256 MiB in, int8 beams (1, 2, 4096, 16, 16, 32) =
64 MiB out, pinned ring of `depth` frames.  Prints one JSON line.  depth=1 (no overlap) is measured too.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dpdk_dc_sand_amd import _lib, accel  # noqa: E402
from dpdk_dc_sand_amd.beamforming import StreamingBeamformerTemplate  # noqa: E402

TS = 1 / 1712e6


def copy_rate(ctx, host, dev_nbytes, direction, reps=8):
    """GB/s of hipMemcpyAsync between a pinned host array and a device buffer (one stream)."""
    q = ctx.create_command_queue()
    dev = accel.DeviceArray(ctx, (dev_nbytes,), np.uint8)
    fn = "bf_memcpy_h2d" if direction == "h2d" else "bf_memcpy_d2h"
    args = (dev.ptr, host.ptr) if direction == "h2d" else (host.ptr, dev.ptr)
    _lib.call(fn, *args, dev_nbytes, q.handle)
    q.finish()
    t = time.perf_counter()
    for _ in range(reps):
        _lib.call(fn, *args, dev_nbytes, q.handle)
    q.finish()
    return dev_nbytes * reps / (time.perf_counter() - t) / 1e9


def run(ctx, args, depth, frames_host, beams_host, d):
    A, M, C, T, B = 64, 16, 4096, 256, 1
    tmpl = StreamingBeamformerTemplate(ctx, B, C, C, T, A, M, delay_channels=1, sample_signed=True,
                                       out_int8=not args.out_float, out_scale=1 / 64, batch_dt=T * 2 * C * TS,
                                       depth=depth)
    with tmpl.instantiate() as sb:
        sb.set_delays(d)
        tickets = []
        for k in range(args.warmup):
            tickets.append(sb.submit(frames_host[k % len(frames_host)], beams_host[k % len(beams_host)]))
        sb.flush()
        tickets = []
        t = time.perf_counter()
        for k in range(args.frames):
            if k >= depth:
                sb.wait(tickets[k - depth])
            tickets.append(sb.submit(frames_host[k % depth], beams_host[k % depth]))
        sb.wait(tickets[-1])
        dt = time.perf_counter() - t
        stages = np.array([sb.stage_ms(tk) for tk in tickets[-depth:]])
    samples = A * 2 * C * T * B * args.frames
    return dict(depth=depth, seconds=dt, gsamples_per_s=samples / dt / 1e9,
                frames_per_s=args.frames / dt, in_gb_per_s=float(np.prod(tmpl.input_shape)) * args.frames / dt / 1e9,
                stage_ms_median={"h2d": float(np.median(stages[:, 0])), "compute": float(np.median(stages[:, 1])),
                                 "d2h": float(np.median(stages[:, 2]))})


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--frames", type=int, default=24)
    p.add_argument("--warmup", type=int, default=4)
    p.add_argument("--depth", type=int, default=4)
    p.add_argument("--out-float", action="store_true")
    args = p.parse_args()
    ctx = accel.create_some_context()
    A, M, C, T = 64, 16, 4096, 256
    in_shape, out_shape = (1, A, C, T, 2, 2), (1, 2, C, T // 16, 16, 2 * M)
    odt = np.float32 if args.out_float else np.int8
    rng = np.random.default_rng(0)
    frames_host = []
    for _ in range(args.depth):
        h = accel.HostArray(in_shape, np.int8, ctx)
        h[...] = rng.integers(-128, 128, in_shape, dtype=np.int8)
        frames_host.append(h)
    beams_host = [accel.HostArray(out_shape, odt, ctx) for _ in range(args.depth)]
    d = np.zeros((1, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, (1, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (1, M, A))
    h2d = copy_rate(ctx, frames_host[0], frames_host[0].nbytes, "h2d")
    d2h = copy_rate(ctx, frames_host[1 % args.depth], frames_host[0].nbytes, "d2h")
    overlapped = run(ctx, args, args.depth, frames_host, beams_host, d)
    serial = run(ctx, args, 1, frames_host, beams_host, d)
    samples_per_frame = A * 2 * C * T
    line = {
        "metric": "streaming int8 voltage Gsamples/s (host -> GPU -> host, config 5)",
        "value": round(overlapped["gsamples_per_s"], 2), "unit": "Gsamples/s",
        "frame": {"in_shape": in_shape, "in_bytes": int(np.prod(in_shape)), "out_shape": out_shape,
                  "out_dtype": np.dtype(odt).name, "out_bytes": int(np.prod(out_shape)) * np.dtype(odt).itemsize,
                  "samples": samples_per_frame},
        "frames": args.frames, "depth": args.depth,
        "overlapped": overlapped, "serial_depth1": serial,
        "pcie_copy_gb_per_s": {"h2d": round(h2d, 2), "d2h": round(d2h, 2)},
        "h2d_bound_gsamples_per_s": round(h2d * 1e9 / 2 / 1e9, 2),  # 2 bytes per complex sample
        "frac_of_h2d_bound": round(overlapped["gsamples_per_s"] / (h2d / 2), 4),
        "device": ctx.device.name,
    }
    print(json.dumps(line, default=float), flush=True)


if __name__ == "__main__":
    main()
