"""Per-operator timing on the GPU: the reference's three-pass chain (reorder, coefficient generator, table multiply,
OpSequence) next to the fused operator, at the SURVEY §8d configurations.  HIP-event averages on the launch
stream, random inputs, algorithmic bytes per launch and the achieved fraction of 8 TB/s.

    python tools/bench_ops.py [--reps 10] [--only cfg3,cfg4]     -> one JSON line per measurement
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from dpdk_dc_sand_amd import accel  # noqa: E402
from dpdk_dc_sand_amd.beamforming import (CoeffGeneratorTemplate, FusedBeamformerTemplate,  # noqa: E402
                                          MatrixMultiplyTemplate, OpSequenceTemplate, PreBeamformReorderTemplate)

TS = 1 / 1712e6
HBM = 8.0e12
CONFIGS = {
    "cfg1": dict(A=4, M=1, C=64, Ctot=1024, T=1024, B=1),
    "cfg2": dict(A=64, M=1, C=4096, Ctot=4096, T=256, B=8),
    "cfg3": dict(A=64, M=16, C=4096, Ctot=4096, T=256, B=8),
    "cfg4": dict(A=256, M=64, C=4096, Ctot=32768, T=256, B=1),
}


def timeit(queue, fn, reps, settle_s=0.2):
    # untimed clock settle first: the first ~30 ms of load run up to 35 % slower (profiles/r1_v6_clock_ramp.txt)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < settle_s:
        for _ in range(4):
            fn()
        queue.finish()
    e0, e1 = accel.Event(), accel.Event()
    e0.record(queue)
    for _ in range(reps):
        fn()
    e1.record(queue)
    queue.finish()
    return e1.time_since(e0) / reps


def emit(cfg, op, seconds, alg_bytes, **extra):
    line = {"config": cfg, "op": op, "us": round(seconds * 1e6, 2), "alg_bytes": int(alg_bytes),
            "achieved_GBps": round(alg_bytes / seconds / 1e9, 1), "frac_8TBps": round(alg_bytes / seconds / HBM, 4)}
    line.update(extra)
    print(json.dumps(line), flush=True)


def delays(C, M, A, rng):
    d = np.zeros((C, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
    d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])
    return d


def run_config(ctx, q, name, c, reps, rng, fused_only=False, tag=""):
    A, M, C, Ctot, T, B = c["A"], c["M"], c["C"], c["Ctot"], c["T"], c["B"]
    samples = A * 2 * C * T * B
    vbytes = 2 * samples
    raw = rng.integers(0, 256, (B, A, C, T, 2, 2), dtype=np.uint8)

    if fused_only:
        return run_fused(ctx, q, name, c, reps, rng, raw, samples, tag)
    # the reference's three-pass chain, op by op and as the OpSequence
    seq = OpSequenceTemplate(ctx, B, 2, C, Ctot, T // 16, 16, A, M, 0, TS, T).instantiate(q)
    seq.ensure_all_bound()
    seq.beamform_coeff.buffer("delay_vals").set(q, delays(C, M, A, rng))
    seq.prebeamform_reorder.buffer("inSamples").set(q, raw)
    table = B * 2 * C * 2 * A * 2 * M * 4
    out_f32 = 8 * M * 2 * C * T * B
    emit(name, "reorder", timeit(q, seq.prebeamform_reorder, reps), 2 * vbytes)
    emit(name, "coeff_gen", timeit(q, seq.beamform_coeff, reps), table + C * M * A * 16)
    emit(name, "matrix_multiply", timeit(q, seq.beamform_mult, reps), vbytes + table + out_f32)
    t_seq = timeit(q, seq, reps)
    emit(name, "op_sequence", t_seq, 3 * vbytes + 2 * table + out_f32 + C * M * A * 16,
         gsamples_per_s=round(samples / t_seq / 1e9, 2))
    del seq
    run_fused(ctx, q, name, c, reps, rng, raw, samples, tag)


def run_fused(ctx, q, name, c, reps, rng, raw, samples, tag):
    A, M, C, Ctot, T, B = c["A"], c["M"], c["C"], c["Ctot"], c["T"], c["B"]
    d1 = delays(1, M, A, rng)
    for label, kw in (("fused_f32_fast", {}), ("fused_f32_exact", dict(exact_coeffs=True)),
                      ("fused_int8", dict(out_int8=True, out_scale=1 / 64))):
        tmpl = FusedBeamformerTemplate(ctx, B, C, Ctot, T, A, M, sample_period=TS, delay_channels=1, t0=0.0,
                                       batch_dt=T * 2 * Ctot * TS, **kw)
        op = tmpl.instantiate(q)
        op.ensure_all_bound()
        op.buffer("inSamples").set(q, raw)
        op.buffer("delay_vals").set(q, d1)
        t = timeit(q, op, reps)
        emit(name, label + tag, t, tmpl.algorithmic_bytes(), gsamples_per_s=round(samples / t / 1e9, 2))
        del op


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--only", default=",".join(CONFIGS))
    p.add_argument("--fused-only", action="store_true")
    p.add_argument("--tag", default="", help="suffix for the op names (e.g. the env variant under test)")
    args = p.parse_args()
    ctx = accel.create_some_context()
    q = ctx.create_command_queue()
    rng = np.random.default_rng(0)
    for name in args.only.split(","):
        run_config(ctx, q, name, CONFIGS[name], args.reps, rng, args.fused_only, args.tag)


if __name__ == "__main__":
    main()
