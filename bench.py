"""Headline benchmark: int8 voltage Gsamples/s through the fused MI355X beamformer (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg2|cfg4] [--no-cpu-baseline] [--no-pmc]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

A "step" is one pass of the hot path over one batch block of synthetic input already resident in HBM: one
`bf_beamform_fused` launch = pre-beamform reorder (fused) + per-batch steering-coefficient regeneration from the
delay model + the antenna x beam complex contraction, for every (batch, pol, channel, sample) of the shard.
Workload cfg3 (default, BASELINE configs[2], the north-star target): 64 antennas, 16 beams, 4096 channels per
GPU, T = 256 samples, B = 8 batches, dual-pol int8 voltages, int8 requantised beams from the integer MFMA path
(bit-exact to the oracle's integer contract; `--output f32` gives float32 beams, `--int8-contract f32` int8 beams
requantised from the float32 path).  cfg2 (configs[1]): 1 beam.  cfg4 (configs[3], per GPU): 256 ants, 64 beams.

Multi-GPU: frequency channels shard across ranks with no data-path collective (rank r = X-engine r,
channels [C r, C (r+1)) of a C*N-channel band): scaling is weak.  The only collective is the root -> ranks channel
scatter of the full-band voltage cube, over RCCL (`torch.distributed` backend "nccl") on the GPUs: rank 0 builds
the band in its HBM, packs each rank's channel slice contiguously and scatters it; each rank's timed hot path then
runs on the slice it received.  The scatter is timed on its own (outside the hot-path timing) and reported in the
line's `scatter` block.  The timing bracket (barrier + max over ranks) runs over gloo.

Rank 0 prints ONE JSON line.  `value` = samples all ranks processed / max-over-ranks wall time of the K timed
steps (barrier + device sync on both sides).  `roofline.achieved` = algorithmic bytes per launch / average
launch duration from HIP events on the launch stream; `roofline.read_frac` = the voltage bytes alone / that time /
peak (the north star's "HBM-read roofline").  `roofline.traffic` = HBM bytes per launch from rocprofv3 PMC
counters (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, separate passes), rank 0, N = 1.  `ceiling` = the same
traffic mix as a plain streaming kernel on this box (diagnostic library), when it is built.
`cpu_baseline` = the oracle's vectorised NumPy restatement on a bounded channel sample, rank 0, N = 1.
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "int8 voltage Gsamples/s ingested + beams/s, 64-ant 4096-ch; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
TS = 1 / 1712e6

WORKLOADS = {
    "cfg3": dict(A=64, M=16, C=4096, T=256, B=8, desc="64 ants, 16 beams, 4096 ch/GPU, T=256, B=8, dual-pol int8, "
                 "per-batch coefficient regeneration fused (BASELINE configs[2])"),
    "cfg2": dict(A=64, M=1, C=4096, T=256, B=8, desc="64 ants, 1 beam, 4096 ch/GPU, T=256, B=8, dual-pol int8 "
                 "(BASELINE configs[1])"),
    "cfg4": dict(A=256, M=64, C=4096, T=256, B=1, Ctot=32768,
                 desc="256 ants, 64 beams, 4096 of 32768 ch per GPU (X-engine = rank), T=256, B=1, dual-pol int8 "
                      "(BASELINE configs[3], per GPU)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="cfg3")
    p.add_argument("--output", choices=("int8", "f32"), default="int8",
                   help="int8 requantised beams (bit-exact integer path, default) or float32 beams")
    p.add_argument("--int8-contract", choices=("q14", "f32"), default="q14",
                   help="int8 beams from the Q14 integer path (default) or requantised from the float32 path")
    p.add_argument("--out-int8", action="store_true", help="same as --output int8")
    p.add_argument("--out-f32", action="store_true", help="same as --output f32")
    p.add_argument("--settle-ms", type=float, default=300.0,
                   help="untimed clock-settle launches after the warmup steps (milliseconds of wall time)")
    p.add_argument("--unsigned", action="store_true", help="uint8 voltages (the reference slots' dtype) instead of int8")
    p.add_argument("--nbuf", type=int, default=2, help="rotating input/output buffer sets (defeat the 256 MB MALL)")
    p.add_argument("--scatter-backend", choices=("nccl", "gloo", "none"), default="nccl",
                   help="N > 1: how the full-band cube reaches the ranks (nccl = RCCL over xGMI, device to device; "
                        "gloo = host staging, for rehearsals with several ranks on one GPU; none = per-rank "
                        "synthetic input)")
    p.add_argument("--scatter-at-one", action="store_true",
                   help="run the scatter path at N = 1 as well (a one-rank RCCL communicator: exercises the device "
                        "band, the collective call and the binding of the received tensor on a one-GPU box)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--no-secondary", action="store_true")
    p.add_argument("--no-ceiling", action="store_true")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    a = p.parse_args()
    if a.out_f32:
        a.output = "f32"
    if a.out_int8:
        a.output = "int8"
    a.out_int8 = a.output == "int8"
    return a


class Dist:
    """Barrier + max-reduction across ranks (gloo, CPU) for the timing bracket, plus an RCCL group for the
    channel scatter.  torch is imported before libbf, so one HIP runtime serves both (its libamdhip64 SONAME is
    the one libbf.so links)."""

    def __init__(self, scatter_backend="none", force=False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.scatter_backend = scatter_backend if (self.world > 1 or force) else "none"
        self.nccl = None
        if self.world > 1 or (force and scatter_backend != "none"):
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("WORLD_SIZE", str(self.world))
            os.environ.setdefault("RANK", str(self.rank))
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            saved = os.dup(1)  # gloo prints its connection banner on stdout: keep stdout for the JSON line
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                if self.scatter_backend == "nccl":
                    torch.cuda.set_device(self.local_rank % max(torch.cuda.device_count(), 1))
                    self.nccl = dist.new_group(backend="nccl")
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v):
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def make_inputs(np, rng, shape, nbuf, unsigned=False):
    n = int(np.prod(shape))
    return [np.frombuffer(rng.bytes(n), np.uint8 if unsigned else np.int8).reshape(shape) for _ in range(nbuf)]


def scatter_inputs(args, dist, shape):
    """The channel scatter: rank 0 holds the full band (B, A, C*N, T, 2, 2) and sends rank r its
    packed channel slice [C r, C (r+1)).  Returns (per-rank slice, report).  nccl: device tensors over RCCL (the
    band is generated in rank 0's HBM); gloo: host arrays (rehearsal).  The slice is what this rank's timed hot
    path then processes."""
    import numpy as np
    import torch

    from dpdk_dc_sand_amd.shard import pack_channel_slices

    B, A, C, T = shape[:4]
    world, rank = dist.world, dist.rank
    per_rank = int(np.prod(shape))
    tdt = torch.uint8 if args.unsigned else torch.int8
    report = {"backend": dist.scatter_backend, "bytes_per_rank": per_rank, "ranks": world,
              "band_shape": [B, A, C * world, T, 2, 2]}
    if dist.scatter_backend == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
        parts = None
        if rank == 0:
            g = torch.Generator(device=dev)
            g.manual_seed(1)
            lo, hi = (0, 256) if args.unsigned else (-128, 128)
            band = torch.randint(lo, hi, (B, A, C * world, T, 2, 2), dtype=tdt, device=dev, generator=g)
            parts = [band[:, :, r * C:(r + 1) * C].contiguous() for r in range(world)]  # pack: B*A strided runs
            del band
        out = torch.empty(shape, dtype=tdt, device=dev)
        warm = torch.ones(1, device=dev)
        dist.dist.all_reduce(warm, group=dist.nccl)  # communicator set-up outside the timing
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            dist.dist.scatter(out, scatter_list=parts, src=0, group=dist.nccl)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        del parts
        t = dist.max(min(times))
        report["collective"] = "RCCL scatter (torch.distributed nccl) over xGMI, device to device"
    else:
        full = None
        if rank == 0:
            rng = np.random.default_rng(1)
            n = B * A * C * world * T * 4
            full = np.frombuffer(rng.bytes(n), np.uint8 if args.unsigned else np.int8).reshape(
                B, A, C * world, T, 2, 2)
        dist.barrier()
        t0 = time.perf_counter()
        ttype = torch.from_numpy(np.zeros(1, np.uint8 if args.unsigned else np.int8)).dtype
        out = torch.empty(shape, dtype=ttype)
        if rank == 0:
            dist.dist.scatter(out, scatter_list=[torch.from_numpy(p) for p in pack_channel_slices(full, world)], src=0)
        else:
            dist.dist.scatter(out, src=0)
        t = dist.max(time.perf_counter() - t0)
        out = out.numpy()
        report["collective"] = "gloo scatter through host memory (rehearsal backend)"
    report["seconds"] = round(t, 6)
    report["GBps_per_peer"] = round(per_rank / t / 1e9, 2)
    report["GBps_root_egress"] = round(per_rank * (world - 1) / t / 1e9, 2)
    return out, report


def template(args, dist, wl, int8_contract=None, kernel_path="auto"):
    from dpdk_dc_sand_amd.beamforming import FusedBeamformerTemplate
    A, M, C, T, B = wl["A"], wl["M"], wl["C"], wl["T"], wl["B"]
    Ctot = wl.get("Ctot", C * max(dist.world, 1))
    return FusedBeamformerTemplate(args.ctx, B, C, Ctot, T, A, M, xeng_id=dist.rank, sample_period=TS,
                                   delay_channels=1, sample_signed=not args.unsigned, out_int8=args.out_int8,
                                   out_scale=1 / 64, t0=0.0, batch_dt=T * 2 * Ctot * TS,
                                   int8_contract=int8_contract or args.int8_contract, kernel_path=kernel_path)


def delay_model(np, rng, shape):
    d = np.zeros(shape, np.float32)  # compact (1, M, A, 4) polynomial delay model with rates
    d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
    d[..., 1] = rng.uniform(-1e-9, 1e-9, d.shape[:-1])
    d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])
    d[..., 3] = rng.uniform(-1, 1, d.shape[:-1])
    return d


def run_gpu(args, dist, wl, tmpl=None, inputs=None):
    """Time K launches of the fused operator.  `inputs`: this rank's resident input (a torch device tensor from
    the RCCL scatter, or a host array), else synthetic host data."""
    import numpy as np

    from dpdk_dc_sand_amd import accel

    queue = args.queue
    tmpl = tmpl or template(args, dist, wl)
    rng = np.random.default_rng(1 + dist.rank)
    d = delay_model(np, rng, tmpl.delay_shape)
    ops = []
    hosts = None
    if inputs is None:
        hosts = make_inputs(np, rng, tmpl.input_shape, args.nbuf, args.unsigned)
    for i in range(args.nbuf):
        op = tmpl.instantiate(queue)
        if inputs is not None and hasattr(inputs, "data_ptr"):
            # the scattered device tensor itself for buffer 0, a device-side copy for the others
            src = inputs if i == 0 else inputs.clone()
            op.bind(inSamples=accel.DeviceArray(args.ctx, tmpl.input_shape, op.slots["inSamples"].dtype,
                                                ptr=src.data_ptr(), owner=False))
            op._keep = src
        op.ensure_all_bound()
        if hosts is not None:
            op.buffer("inSamples").set(queue, hosts[i])
        elif not hasattr(inputs, "data_ptr"):
            op.buffer("inSamples").set(queue, inputs)
        op.buffer("delay_vals").set(queue, d)
        ops.append(op)
    del hosts
    if inputs is not None and hasattr(inputs, "data_ptr"):
        import torch
        torch.cuda.synchronize()  # the clones are on torch's stream
    for i in range(args.warmup):
        ops[i % len(ops)]()
    queue.finish()
    # Clock settle (untimed, before the timed region): the GPU ramps its clocks over the first ~30 ms of load
    # (the first launches of a fresh process run up to 35 % slower, profiles/r1_v6_clock_ramp.txt); a streaming
    # beamformer runs continuously, so the steady state is the number that matters.
    t_settle = time.perf_counter()
    i = 0
    while time.perf_counter() - t_settle < args.settle_ms / 1e3:
        for _ in range(8):
            ops[i % len(ops)]()
            i += 1
        queue.finish()

    e0, e1 = accel.Event(), accel.Event()
    dist.barrier()
    queue.finish()
    t0 = time.perf_counter()
    e0.record(queue)
    for i in range(args.steps):
        ops[i % len(ops)]()
    e1.record(queue)
    queue.finish()
    t_local = time.perf_counter() - t0
    dist.barrier()
    kernel_s = e1.time_since(e0) / args.steps
    t_max = dist.max(t_local)
    A, M, C, T, B = wl["A"], wl["M"], wl["C"], wl["T"], wl["B"]
    return dict(t_max=t_max, kernel_s=kernel_s, samples_per_step=A * 2 * C * T * B, beams_per_step=M * 2 * C * T * B,
                alg_bytes=tmpl.algorithmic_bytes(), read_bytes=A * 2 * C * T * B * 2, ops=ops, tmpl=tmpl, delays=d)


def contract_check(args, dist, wl, r):
    """Q14 integer contract vs requantise(float32 beams) on the headline's own input: the cost of the integer
    contract in output values (at most one LSB by construction; the rate is measured here)."""
    import numpy as np
    op = r["ops"][0]
    op()
    args.queue.finish()
    q14 = op.buffer("outData").get(args.queue)
    alt = template(args, dist, wl, int8_contract="f32").instantiate(args.queue)
    alt.bind(inSamples=op.buffer("inSamples"), delay_vals=op.buffer("delay_vals"))
    alt.ensure_all_bound()
    alt()
    qf = alt.buffer("outData").get(args.queue)
    diff = np.abs(q14.astype(np.int16) - qf.astype(np.int16))
    return {"compared": "Q14 integer int8 beams vs int8 requantised from the float32 path, same input",
            "values": int(diff.size), "mismatch_rate": float(np.count_nonzero(diff)) / diff.size,
            "max_abs_lsb": int(diff.max())}


def stream_ceiling(args, in_bytes, out_bytes):
    """The same traffic mix (in_bytes read, out_bytes written) as plain streaming kernels from the diagnostic
    library (build/libbf_diag.so: 16-byte lanes, plain / non-temporal loads and stores, 4:1 interleaved mix for
    the int8 path): the best of them is this box's achievable ceiling for the fused kernel's traffic."""
    import ctypes

    from dpdk_dc_sand_amd import accel
    path = os.path.join(ROOT, "build", "libbf_diag.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    V, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.bf_diag_stream.argtypes = [V, V, S, S, I, I, V]
    bufs = [(accel.DeviceArray(args.ctx, (in_bytes,), "u1"), accel.DeviceArray(args.ctx, (max(out_bytes, 16),), "u1"))
            for _ in range(2)]
    best = None
    codes = [1, 101, 102, 103]
    if out_bytes * 4 == in_bytes:
        codes += [200, 201]
    for grid in (1024, 2048):
        for code in codes:
            for i in range(3):
                lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, in_bytes, out_bytes, grid, code,
                                   args.queue.handle)
            e0 = accel.Event(args.queue)
            n = 10
            for i in range(n):
                lib.bf_diag_stream(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, in_bytes, out_bytes, grid, code,
                                   args.queue.handle)
            e1 = accel.Event(args.queue)
            args.queue.finish()
            t = e1.time_since(e0) / n
            if best is None or t < best[0]:
                best = (t, grid, code)
    return {"us": round(best[0] * 1e6, 2), "GBps": round((in_bytes + out_bytes) / best[0] / 1e9, 1),
            "kernel": f"bf_diag_stream grid {best[1]} mode {best[2]}",
            "note": "best plain streaming kernel over the same read/write byte mix on this box"}


def cpu_baseline(wl, out_int8, seconds=10.0):
    """The oracle's vectorised NumPy restatement (reorder -> per-batch coefficients -> f32 matmul) timed on
    this host on a bounded channel sample of the same workload (kind "port")."""
    import numpy as np

    import oracle as O
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    A, M, T, B = wl["A"], wl["M"], wl["T"], wl["B"]
    rng = np.random.default_rng(7)
    d = np.zeros((1, M, A, 4), np.float32)
    d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
    d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])

    def once(c):
        raw = rng.integers(-128, 128, size=(B, A, c, T, 2, 2), dtype=np.int8)
        t = time.perf_counter()
        Ctot = wl.get("Ctot", wl["C"])
        y = O.fused_beamform(raw, d, Ctot, signed=True, batch_dt=T * 2 * Ctot * TS)
        if out_int8:
            O.requantise(y, 1 / 64)
        return time.perf_counter() - t

    c = 16
    dt = once(c)  # warm-up + rate estimate
    c = int(min(max(16, c * seconds / max(dt, 1e-3)), wl["C"]))
    dt = once(c)
    rate = A * 2 * c * T * B / dt / 1e9
    return {"value": round(rate, 4), "unit": "Gsamples/s", "cores": int(threads), "kind": "port",
            "sample": f"{c} of {wl['C']} channels x B={B} x T={T} x A={A} x 2 pols ({dt:.1f} s): oracle.fused_beamform "
                      f"(NumPy reorder + float64-phase coefficients + float32 matmul{' + requantise' if out_int8 else ''}, "
                      f"BLAS threads={threads})"}


def pmc_traffic(args):
    """HBM bytes per fused launch from rocprofv3 counters: FETCH_SIZE and WRITE_SIZE in separate passes
    (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reads 1/2 of a wide coalesced stream -> x2; WRITE_SIZE exact; KiB).
    Calibrated in-repo (tools/pmc_calibrate.py, profiles/r2_v_pmc_calibration.jsonl): a 1 GiB streaming read gives
    FETCH_SIZE = 0.500 x the bytes (every request a 128-byte TCC_EA0_RDREQ_128B, tallied at 64 B), a 1 GiB write
    WRITE_SIZE = 1.000 x, and a 1 GiB + 256 MiB mix the same two ratios."""
    exe = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 not found"
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        out = tempfile.mkdtemp(prefix="bfpmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload,
               "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--output", args.output,
               "--int8-contract", args.int8_contract] + (["--unsigned"] if args.unsigned else [])
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
        files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            return None, f"rocprofv3 {counter} failed rc={r.returncode}: {r.stderr[-300:]}"
        per = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if "beamform_fused" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    per.append(float(row["Counter_Value"]))
        if not per:
            return None, f"no {counter} rows for the fused kernel"
        vals[counter] = sorted(per)[len(per) // 2]
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, vals


def compute_desc(out_int8, int8_contract):
    if out_int8 and int8_contract == "q14":
        return "Q14 two-limb int8 coefficients on v_mfma_i32_16x16x64_i8, exact int32 accumulation, int8 beams"
    desc = "f16 hi/lo-split coefficients on v_mfma_f32_16x16x32_f16, f32 accumulation"
    return desc + (", int8 beams requantised in-kernel from the float32 beams" if out_int8 else ", float32 beams")


def mfma_util(wl, out_int8, int8_contract, kernel_s):
    """Matrix-core utilisation of the dominant kernel: algorithmic ops (8 A M per (b, p, c, t): the complex MAC)
    and the ops the MFMAs actually issue (two coefficient limbs, K = 2A padded to the MFMA depth, N = 2M padded
    to 16), both against the dense peak.  The path is HBM-bound by design (SURVEY §7 hard part 1): this shows the
    headroom, not a target."""
    A, M, C, T, B = wl["A"], wl["M"], wl["C"], wl["T"], wl["B"]
    integer = out_int8 and int8_contract == "q14"
    kg = 64 if integer else 32
    kpad, npad = -(-2 * A // kg) * kg, -(-2 * M // 16) * 16
    alg = 8.0 * A * M * 2 * C * T * B
    issued = 2.0 * 2 * kpad * npad * T * 2 * C * B
    peak, unit, instr = ((5000.0, "TOPS", "v_mfma_i32_16x16x64_i8 (2x the dense BF16 rate, MI355X_MICROARCH.md)")
                         if integer else (2500.0, "TFLOP/s", "v_mfma_f32_16x16x32_f16 (dense F16 = BF16 rate)"))
    return {"instruction": instr, "unit": unit, "peak": peak, "algorithmic": round(alg / kernel_s / 1e12, 1),
            "issued": round(issued / kernel_s / 1e12, 1), "frac_issued": round(issued / kernel_s / 1e12 / peak, 4)}


def kernel_name(wl, out_int8, int8_contract="q14"):
    """The launch's dominant kernel (bf_fused.hip dispatch): item kernels for A <= 64 and T <= 256, else the wide
    kernels."""
    integer = out_int8 and int8_contract == "q14"
    if wl["A"] <= 64 and wl["T"] <= 256:
        return "beamform_fused_i8_item_kernel" if integer else "beamform_fused_item_kernel"
    return "beamform_fused_i8_w32_kernel" if integer else "beamform_fused_wide_kernel"


def secondary(args, dist, workload, out_int8, int8_contract="q14"):
    sub = argparse.Namespace(**{**vars(args), "workload": workload, "out_int8": out_int8,
                                "int8_contract": int8_contract})
    wl = WORKLOADS[workload]
    r = run_gpu(sub, dist, wl)
    r.pop("ops")
    out = {"workload": workload + ": " + wl["desc"],
           "output": ("int8" + ("" if int8_contract == "q14" else " (requantised from float32 beams)"))
           if out_int8 else "float32",
           "kernel": kernel_name(wl, out_int8, int8_contract),
           "value": round(r["samples_per_step"] * args.steps / r["t_max"] / 1e9, 2), "unit": "Gsamples/s",
           "roofline_frac": round(r["alg_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
           "read_frac": round(r["read_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
           "avg_launch_us": round(r["kernel_s"] * 1e6, 2), "alg_bytes_per_launch": r["alg_bytes"]}
    if not args.no_ceiling:
        ceil = stream_ceiling(args, r["read_bytes"], int(r["alg_bytes"] - r["read_bytes"]))
        if ceil:
            out["ceiling"] = ceil
            out["frac_of_ceiling"] = round(ceil["us"] / out["avg_launch_us"], 4)
    return out


def main():
    args = parse()
    wl = WORKLOADS[args.workload]
    dist = Dist(args.scatter_backend, force=args.scatter_at_one)
    from dpdk_dc_sand_amd import accel

    n_dev = accel.device_count()
    if n_dev < 1:
        raise RuntimeError("no HIP device visible")
    args.ctx = accel.create_some_context(device=dist.local_rank % n_dev)
    args.queue = args.ctx.create_command_queue()
    if args.pmc_child:
        run_gpu(args, dist, wl)
        return
    tmpl = template(args, dist, wl)
    scatter = None
    inputs = None
    if dist.scatter_backend != "none":
        # the scatter is reported beside the hot path, not part of it: if the collective raises (on every rank),
        # the ranks agree over gloo and generate their shards in place, so the timed line is still produced
        err = None
        try:
            inputs, scatter = scatter_inputs(args, dist, tmpl.input_shape)
        except Exception as e:  # noqa: BLE001 -- reported in the line's scatter block
            err = f"{type(e).__name__}: {str(e)[:300]}"
        if dist.max(1.0 if err else 0.0) > 0:
            inputs = None
            scatter = {"backend": dist.scatter_backend, "error": err or "failed on another rank",
                       "note": "scatter failed; each rank generated its shard in place"}
    r = run_gpu(args, dist, wl, tmpl=tmpl, inputs=inputs)
    total_samples = r["samples_per_step"] * args.steps * dist.world
    value = total_samples / r["t_max"] / 1e9
    achieved = r["alg_bytes"] / r["kernel_s"] / 1e9
    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "Gsamples/s", "n_gpus": dist.world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(r["t_max"] / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int8",
        "data": "synthetic (uniform random %s voltages, random delay/phase polynomials)" % ("uint8" if args.unsigned else "int8"),
        "config": {"workload": args.workload + ": " + wl["desc"], "n_ants": wl["A"], "n_beams": wl["M"],
                   "n_channels_per_gpu": wl["C"], "n_samples_per_channel": wl["T"], "n_batches": wl["B"],
                   "n_pols": 2, "output": "int8" if args.out_int8 else "float32",
                   "int8_contract": args.int8_contract if args.out_int8 else None,
                   "parallelism": f"channel-shard x{dist.world} (xeng_id = rank), no data-path collective"},
        "beams_per_s": round(r["beams_per_step"] * args.steps * dist.world / r["t_max"], 1),
        "compute": compute_desc(args.out_int8, args.int8_contract),
        "device": args.ctx.device.name,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "read_frac": round(r["read_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel": kernel_name(wl, args.out_int8, args.int8_contract),
                     "avg_launch_us": round(r["kernel_s"] * 1e6, 2), "alg_bytes_per_launch": r["alg_bytes"],
                     "read_bytes_per_launch": r["read_bytes"]},
        "mfma": mfma_util(wl, args.out_int8, args.int8_contract, r["kernel_s"]),
        "scatter": scatter or {"backend": None, "note": "no scatter: single rank, or --scatter-backend none "
                                                        "(each rank generates its shard in place)"},
        "cpu_baseline": None,
    }
    if dist.rank == 0 and dist.world == 1 and args.out_int8 and args.int8_contract == "q14":
        line["int8_contract_check"] = contract_check(args, dist, wl, r)
    r.pop("ops")
    if dist.rank == 0 and dist.world == 1 and not args.no_ceiling:
        ceil = stream_ceiling(args, r["read_bytes"], int(r["alg_bytes"] - r["read_bytes"]))
        if ceil:
            line["ceiling"] = ceil
            line["roofline"]["frac_of_ceiling"] = round(ceil["us"] / line["roofline"]["avg_launch_us"], 4)
    if dist.rank == 0 and dist.world == 1 and not args.no_secondary and args.workload == "cfg3":
        line["secondary"] = []
        cases = [("cfg2", args.out_int8, "q14"), ("cfg3", not args.out_int8, "q14"), ("cfg3", True, "f32"),
                 ("cfg4", True, "q14"), ("cfg4", False, "q14")]
        for workload, out_int8, contract in cases:
            if (workload, out_int8, contract if out_int8 else "q14") == (args.workload, args.out_int8,
                                                                          args.int8_contract if args.out_int8 else "q14"):
                continue
            try:
                line["secondary"].append(secondary(args, dist, workload, out_int8, contract))
            except Exception as e:  # secondary lines are informational
                line["secondary"].append({"workload": workload, "error": str(e)[:200]})
    if dist.rank == 0 and dist.world == 1 and not args.no_pmc:
        try:
            traffic, info = pmc_traffic(args)
            line["roofline"]["traffic"] = traffic
            line["roofline"]["traffic_counters"] = info
        except Exception as e:
            line["roofline"]["traffic_counters"] = f"unavailable: {str(e)[:200]}"
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(wl, args.out_int8)
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
