"""A/B: the config-4 int8 table path as one launch over C channels vs C / K launches of K channels each (the Q14
table of a chunk then stays in the 256 MB memory-side cache between its generator and its contraction).  Each chunk
call uses its own input / output buffers.  HIP-event averages, interleaved rounds.

    python tools/diag_chunk.py [--chunks 1,2,4,8] [--rounds 3]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from dpdk_dc_sand_amd import accel  # noqa: E402
from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate  # noqa: E402

TS = 1 / 1712e6


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--chunks", default="1,2,4,8")
    p.add_argument("--rounds", type=int, default=3)
    args = p.parse_args()
    B, C, T, A, M, Ctot = 1, 4096, 256, 256, 64, 32768
    ctx = accel.create_some_context()
    q = ctx.create_command_queue()
    rng = np.random.default_rng(0)
    d = np.zeros((1, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, (1, M, A))
    d[..., 2] = rng.uniform(-np.pi, np.pi, (1, M, A))
    raw = rng.integers(-128, 128, (B, A, C, T, 2, 2), dtype=np.int8)
    variants = {}
    for k in [int(v) for v in args.chunks.split(",")]:
        Ck = C // k
        ops = []
        for j in range(k):
            tmpl = FusedBeamformerTemplate(ctx, B, Ck, Ctot, T, A, M, xeng_id=j, delay_channels=1, sample_signed=True,
                                           out_int8=True, out_scale=1 / 64, sample_period=TS, t0=0.0, batch_dt=0.0)
            op = tmpl.instantiate(q)
            op.ensure_all_bound()
            op.buffer("inSamples").set(q, np.ascontiguousarray(raw[:, :, j * Ck:(j + 1) * Ck]))
            op.buffer("delay_vals").set(q, d)
            ops.append(op)
        variants[k] = ops
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, ops in variants.items():
            for _ in range(3):
                for op in ops:
                    op()
            q.finish()
            e0, e1 = accel.Event(), accel.Event()
            e0.record(q)
            for _ in range(10):
                for op in ops:
                    op()
            e1.record(q)
            q.finish()
            res[k].append(e1.time_since(e0) / 10)
    for k, ts in res.items():
        t = sorted(ts)[len(ts) // 2]
        print(f"cfg4 int8, {k} chunk(s) of {C // k} channels: {t * 1e6:8.1f} us per 4096 channels", flush=True)


if __name__ == "__main__":
    main()
