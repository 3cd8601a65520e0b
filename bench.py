"""Headline benchmark: int8 voltage Gsamples/s through the fused MI355X beamformer (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg3|cfg2|cfg4] [--no-cpu-baseline] [--no-pmc]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N

`--gpus N` alone starts the N ranks itself (N child processes of this script, one per GPU, RANK / WORLD_SIZE /
MASTER_* set; the parent never touches a GPU); under an external launcher `--gpus` must equal WORLD_SIZE.

A "step" is one pass of the hot path over one batch block of synthetic input already resident in HBM: one
`bf_beamform_fused` launch = pre-beamform reorder (fused) + per-batch steering-coefficient regeneration from the
delay model + the antenna x beam complex contraction, for every (batch, pol, channel, sample) of the shard.
Workload cfg3 (default, BASELINE configs[2], the north-star target): 64 antennas, 16 beams, 4096 channels per
GPU, T = 256 samples, B = 8 batches, dual-pol int8 voltages, int8 requantised beams from the integer MFMA path
(bit-exact to the oracle's integer contract; `--output f32` gives float32 beams, `--int8-contract f32` int8 beams
requantised from the float32 path).  cfg2 (configs[1]): 1 beam.  cfg4 (configs[3], per GPU): 256 ants, 64 beams.

Multi-GPU: frequency channels shard across ranks with no data-path collective (rank r = X-engine r,
channels [C r, C (r+1)) of a C*N-channel band): scaling is weak.  The only collective is the root -> ranks channel
scatter of the full-band voltage cube, device to device over RCCL/xGMI through libbf (bf_channel_scatter): rank 0
fills the band in its HBM, packs each rank's channel slice and sends it; each rank receives its slice straight into
the fused operator's input buffer and its timed hot path runs on it.  The scatter is timed on its own (outside the
hot-path timing) and reported in the line's `scatter` block.  The timing bracket (barrier + max over ranks) and the
RCCL id hand-out run over a plain TCP group (dpdk_dc_sand_amd.rendezvous): no torch in the ranks, so every rank
runs libbf on one HIP runtime.  At N > 1 the line's `secondary` also times config 4 channel-sharded (256 ants,
64 beams, 4096 channels per rank of the 32768-channel band, xeng_id = rank: BASELINE configs[3] at N = 8).

Rank 0 prints ONE JSON line.  `value` = samples all ranks processed / max-over-ranks wall time of the K timed
steps (barrier + device sync on both sides).  `roofline.achieved` = algorithmic bytes per launch / average
launch duration from HIP events on the launch stream; `roofline.read_frac` = the voltage bytes alone / that time /
peak (the north star's "HBM-read roofline"), and `read_frac_ceiling` the same for this box's plain streaming kernel
over the kernel's whole read + write byte mix: the read fraction the beams' writes leave reachable.  `roofline.traffic` = HBM bytes per launch from rocprofv3 PMC
counters (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, separate passes), rank 0, N = 1.  `ceiling` = the same
traffic mix as a plain streaming kernel on this box (build/libbf_stream.so), with `target_reachable`: whether the
north star's 0.70 of 8 TB/s is within that stream for the byte mix.  A `kind: streaming` secondary (rank 0, N = 1) is
config 5: 256 MiB frames through the native pinned-ring pipeline against this process's own H2D copy rate.
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


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU).  Without an external launcher, N > 1 starts N child ranks of this script "
                        "itself; under torch.distributed.run it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
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
    p.add_argument("--scatter-backend", choices=("rccl", "host", "none", "nccl", "gloo"), default="rccl",
                   help="N > 1: how the full-band cube reaches the ranks (rccl = libbf bf_channel_scatter over "
                        "RCCL/xGMI, device to device; host = TCP through host memory, for rehearsals with several "
                        "ranks on one GPU; none = per-rank synthetic input; nccl / gloo: aliases of rccl / host)")
    p.add_argument("--scatter-at-one", action="store_true",
                   help="run the scatter path at N = 1 as well (a one-rank RCCL communicator: exercises the device "
                        "band, the libbf scatter and the binding of the received slice on a one-GPU box)")
    p.add_argument("--coeff-table", choices=("on", "off"), default="on",
                   help="int8 wide path (config 4): Q14 coefficients from the generated table (on) or in-kernel")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--no-secondary", action="store_true")
    p.add_argument("--no-stream", action="store_true",
                   help="skip the config-5 streaming secondary (host ring -> H2D -> fused -> D2H, rank 0, N = 1)")
    p.add_argument("--stream-frames", type=int, default=64, help="timed frames of the config-5 streaming secondary")
    p.add_argument("--no-ceiling", action="store_true")
    p.add_argument("--no-rocprof", action="store_true",
                   help="skip the rocprofv3 --kernel-trace re-run that checks the event timings (rank 0, N = 1)")
    p.add_argument("--prof-out", default=None,
                   help="directory for that re-run's trace, timed_kernel_stats.csv and prof_bench.json")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--prof-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--rank-probe", action="store_true", help=argparse.SUPPRESS)  # CPU test of the rank launch
    p.add_argument("--probe-sleep", type=float, default=0.0, help=argparse.SUPPRESS)
    a = p.parse_args(argv)
    if a.out_f32:
        a.output = "f32"
    if a.out_int8:
        a.output = "int8"
    a.out_int8 = a.output == "int8"
    return a


def resolve_world(args, env=None):
    """The ranks of this invocation (one process per GPU, rank r = X-engine r).  Returns (world, launch):
    `launch` is True when this process must start the ranks itself (`--gpus N > 1` and no external launcher, i.e. no
    WORLD_SIZE in the environment).  Under an external launcher (torch.distributed.run) `--gpus` must equal WORLD_SIZE:
    a mismatch would silently time a different number of ranks than the command line names."""
    env = os.environ if env is None else env
    if env.get("WORLD_SIZE") is not None:
        world = int(env["WORLD_SIZE"])
        if args.gpus is not None and args.gpus != world:
            raise ValueError(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        args.gpus = world
        return world, False
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise ValueError(f"--gpus must be >= 1, got {n}")
    args.gpus = n
    return n, n > 1


def free_port_pair(host="127.0.0.1", tries=64):
    """A port p with p and p + 1 both free on `host` (the rendezvous group listens on MASTER_PORT + 1)."""
    import socket
    for _ in range(tries):
        s = socket.socket()
        s.bind((host, 0))
        p = s.getsockname()[1]
        t = socket.socket()
        try:
            t.bind((host, p + 1))
            return p
        except OSError:
            continue
        finally:
            t.close()
            s.close()
    raise RuntimeError("no free port pair for the rank rendezvous")


def launch_ranks(n, argv, poll_s=0.05, grace_s=20.0):
    """`bench.py --gpus N` with no launcher: start N fresh child processes of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set -- the reference's one worker per device
    (utilities/pcie_bandwidth_tests/main.cpp:214-224), each rank X-engine `rank` (coeff_generator.py:53).  This
    process never touches the GPU; the children inherit stdout, so rank 0's JSON line is the run's output.  If a rank
    fails, the others are stopped (they would wait in a collective) and its exit status is returned."""
    import signal
    port = free_port_pair()

    def die_with_parent():  # a rank must not outlive this process (a killed launcher would leave GPUs busy)
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass

    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), BF_BENCH_LAUNCHER="bench.py")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env, cwd=ROOT,
                                      preexec_fn=die_with_parent))

    def forward(signum, _frame):  # SIGTERM / SIGINT to the launcher: stop the ranks, then exit with the signal
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        raise SystemExit(128 + signum)

    signal.signal(signal.SIGTERM, forward)
    signal.signal(signal.SIGINT, forward)
    rc = 0
    try:
        pending = list(range(n))
        while pending and rc == 0:
            for r in list(pending):
                c = procs[r].poll()
                if c is None:
                    continue
                pending.remove(r)
                if c != 0:
                    rc = c if c > 0 else 128 - c  # a signal -> the shell's 128 + signal
                    print(f"bench.py: rank {r} exited with status {c}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    break
            time.sleep(poll_s)
    finally:
        live = [p for p in procs if p.poll() is None]
        for p in live:
            p.terminate()
        deadline = time.monotonic() + grace_s
        for p in live:
            try:
                p.wait(timeout=max(0.1, deadline - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


class Dist:
    """The ranks' host-side group (rendezvous.HostGroup over TCP: barrier + max for the timing bracket, the RCCL id
    hand-out, the host scatter) and, for the RCCL channel scatter, libbf's communicator (shard.ChannelScatter,
    opened once the rank's device is current).  No torch."""

    def __init__(self, scatter_backend="rccl", force=False):
        from dpdk_dc_sand_amd.rendezvous import HostGroup
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        backend = {"nccl": "rccl", "gloo": "host"}.get(scatter_backend, scatter_backend)
        self.scatter_backend = backend if (self.world > 1 or force) else "none"
        self.group = HostGroup(self.rank, self.world) if self.world > 1 else None
        self.comm = None

    def open_comm(self, ctx):
        from dpdk_dc_sand_amd.rendezvous import HostGroup
        from dpdk_dc_sand_amd.shard import ChannelScatter
        self.comm = ChannelScatter(self.group or HostGroup(0, 1), ctx)

    def barrier(self):
        if self.group:
            self.group.barrier()

    def max(self, v):
        return self.group.allreduce_max(v) if self.group else v

    def close(self):
        if self.comm:
            self.comm.close()
        if self.group:
            self.group.close()


def make_inputs(np, rng, shape, nbuf, unsigned=False):
    n = int(np.prod(shape))
    return [np.frombuffer(rng.bytes(n), np.uint8 if unsigned else np.int8).reshape(shape) for _ in range(nbuf)]


def scatter_inputs(args, dist, shape):
    """The channel scatter: rank 0 holds the full band (B, A, C*N, T, 2, 2) and sends rank r its
    packed channel slice [C r, C (r+1)).  Returns (per-rank slice, report).  rccl: the band is filled in rank 0's
    HBM (bf_fill_random) and each slice lands in a device array (libbf bf_channel_scatter over RCCL); host: numpy
    band, slices through the TCP group (rehearsal).  The slice is what this rank's timed hot path then processes."""
    import numpy as np

    from dpdk_dc_sand_amd import _lib, accel
    from dpdk_dc_sand_amd.shard import pack_channel_slices, scatter_channel_slices

    B, A, C, T = shape[:4]
    world, rank = dist.world, dist.rank
    per_rank = int(np.prod(shape))
    dt = np.uint8 if args.unsigned else np.int8
    report = {"backend": dist.scatter_backend, "bytes_per_rank": per_rank, "ranks": world,
              "band_shape": [B, A, C * world, T, 2, 2]}
    if dist.scatter_backend == "rccl":
        band, err = None, None
        try:  # every rank's buffers first: the communicator's set-up is a blocking collective
            if rank == 0:
                band = accel.DeviceArray(args.ctx, (B, A, C * world, T, 2, 2), dt)
                _lib.call("bf_fill_random", band.ptr, band.nbytes, 1, args.queue.handle)
            out = accel.DeviceArray(args.ctx, shape, dt)
        except Exception as e:  # noqa: BLE001
            err = e
        if dist.max(1.0 if err else 0.0) > 0:  # agree before any rank enters bf_comm_create or posts its ncclRecv
            raise err or RuntimeError("scatter set-up failed on another rank")
        dist.open_comm(args.ctx)
        times = []
        for _ in range(3):
            args.queue.finish()
            dist.barrier()
            t0 = time.perf_counter()
            dist.comm.scatter(band, out, B, A, C, T, args.queue)
            args.queue.finish()
            times.append(time.perf_counter() - t0)
        t = dist.max(min(times))
        # what arrived is what the root sent: per-rank slice checksums against the root's band (on the devices)
        ok, sums = dist.comm.verify(band, out, B, A, C, T, args.queue)
        sent, received = dist.comm.stats()
        del band
        report["verified"] = ok
        if sums is not None:
            report["checksums"] = sums
        report["rccl_bytes_received_this_rank"] = received
        report["rccl_bytes_sent_root"] = sent if rank == 0 else None
        report["collective"] = ("RCCL grouped ncclSend/ncclRecv over xGMI via libbf bf_channel_scatter, device to "
                                "device (root: one 2-D pack per peer, its own slice by a 2-D copy -- at one rank by a self send/recv)")
    else:
        full = None
        if rank == 0:
            rng = np.random.default_rng(1)
            full = np.frombuffer(rng.bytes(B * A * C * world * T * 4), dt).reshape(B, A, C * world, T, 2, 2)
        dist.barrier()
        t0 = time.perf_counter()
        out = scatter_channel_slices(full, shape, dt, dist.group)
        t = dist.max(time.perf_counter() - t0)
        del full, pack_channel_slices
        report["collective"] = "host memory over the TCP rendezvous group (rehearsal backend)"
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
                                   int8_contract=int8_contract or args.int8_contract, kernel_path=kernel_path,
                                   coeff_table=args.coeff_table == "on")


def delay_model(np, rng, shape):
    d = np.zeros(shape, np.float32)  # compact (1, M, A, 4) polynomial delay model with rates
    d[..., 0] = rng.uniform(0, 10 * TS, d.shape[:-1])
    d[..., 1] = rng.uniform(-1e-9, 1e-9, d.shape[:-1])
    d[..., 2] = rng.uniform(-np.pi, np.pi, d.shape[:-1])
    d[..., 3] = rng.uniform(-1, 1, d.shape[:-1])
    return d


def run_gpu(args, dist, wl, tmpl=None, inputs=None):
    """Time K launches of the fused operator.  `inputs`: this rank's resident input (an accel.DeviceArray from the
    RCCL scatter, or a host array from the host scatter), else synthetic host data."""
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
    on_device = isinstance(inputs, accel.DeviceArray)
    for i in range(args.nbuf):
        op = tmpl.instantiate(queue)
        if on_device and i == 0:
            op.bind(inSamples=inputs)  # the scattered slice itself (received in place), no copy
        op.ensure_all_bound()
        if hosts is not None:
            op.buffer("inSamples").set(queue, hosts[i])
        elif on_device:
            if i > 0:
                op.buffer("inSamples").copy_region(queue, inputs)  # a device-side copy for the other buffers
        else:
            op.buffer("inSamples").set(queue, inputs)
        op.buffer("delay_vals").set(queue, d)
        ops.append(op)
    del hosts
    queue.finish()
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
    queue.trace_mark(1)  # the timed region's bounds in a profiler trace (tools/kernel_stats.py), outside the timing
    dist.barrier()
    queue.finish()
    t0 = time.perf_counter()
    e0.record(queue)
    for i in range(args.steps):
        ops[i % len(ops)]()
    e1.record(queue)
    queue.finish()
    t_local = time.perf_counter() - t0
    queue.trace_mark(2)
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
    """The same traffic mix (in_bytes read, out_bytes written) as plain streaming kernels from the stream-ceiling
    library (build/libbf_stream.so, tools/stream_ceiling.hip: 16-byte lanes, plain / non-temporal loads and stores,
    4:1 interleaved mix for the int8 path): the best of them is this box's achievable ceiling for the fused kernel's
    traffic."""
    import ctypes

    from dpdk_dc_sand_amd import accel
    path = os.path.join(ROOT, "build", "libbf_stream.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    V, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.bf_stream_ceiling.argtypes = [V, V, S, S, I, I, V]
    bufs = [(accel.DeviceArray(args.ctx, (in_bytes,), "u1"), accel.DeviceArray(args.ctx, (max(out_bytes, 16),), "u1"))
            for _ in range(2)]
    best = None
    codes = [1, 101, 102, 103]
    if out_bytes * 4 == in_bytes:
        codes += [200, 201]
    for grid in (1024, 2048):
        for code in codes:
            for i in range(3):
                lib.bf_stream_ceiling(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, in_bytes, out_bytes, grid, code,
                                      args.queue.handle)
            e0 = accel.Event(args.queue)
            n = 10
            for i in range(n):
                lib.bf_stream_ceiling(bufs[i % 2][0].ptr, bufs[i % 2][1].ptr, in_bytes, out_bytes, grid, code,
                                      args.queue.handle)
            e1 = accel.Event(args.queue)
            args.queue.finish()
            t = e1.time_since(e0) / n
            if best is None or t < best[0]:
                best = (t, grid, code)
    return {"us": round(best[0] * 1e6, 2), "GBps": round((in_bytes + out_bytes) / best[0] / 1e9, 1),
            "kernel": f"bf_stream_ceiling grid {best[1]} mode {best[2]}",
            "note": "best plain streaming kernel over the same read/write byte mix on this box"}


def copy_rate(args, host, direction, reps=8):
    """GB/s of bf_memcpy_{h2d,d2h} between a pinned host array and a device buffer on one stream (this process)."""
    import numpy as np

    from dpdk_dc_sand_amd import _lib, accel
    dev = accel.DeviceArray(args.ctx, (host.nbytes,), np.uint8)
    fn = "bf_memcpy_h2d" if direction == "h2d" else "bf_memcpy_d2h"
    ptrs = (dev.ptr, host.ctypes.data) if direction == "h2d" else (host.ctypes.data, dev.ptr)
    _lib.call(fn, *ptrs, host.nbytes, args.queue.handle)
    args.queue.finish()
    t = time.perf_counter()
    for _ in range(reps):
        _lib.call(fn, *ptrs, host.nbytes, args.queue.handle)
    args.queue.finish()
    return host.nbytes * reps / (time.perf_counter() - t) / 1e9


def stream_secondary(args, depth=4):
    """Config 5 (BASELINE configs[4]): the sustained rate of host frames through the native streaming pipeline
    (bf_pipeline: pinned host ring -> H2D stream -> fused coefficient regeneration + beamform + int8 requantisation ->
    D2H stream, `depth` frames in flight), against this process's own pinned H2D copy rate on the same buffers -- the
    PCIe bound, since a frame's voltages (256 MiB) are 4x its int8 beams.  The reference moves the same data in
    back-to-back phases (common/UnitTest.cpp:28-57; cudaPcieRateTest.cpp:63-123)."""
    import numpy as np

    from dpdk_dc_sand_amd import accel
    from dpdk_dc_sand_amd.beamforming import StreamingBeamformerTemplate
    A, M, C, T, B = 64, 16, 4096, 256, 1
    tmpl = StreamingBeamformerTemplate(args.ctx, B, C, C, T, A, M, delay_channels=1, sample_signed=True,
                                       out_int8=True, out_scale=1 / 64, batch_dt=T * 2 * C * TS, depth=depth)
    rng = np.random.default_rng(11)
    frames = []
    for _ in range(depth):
        h = accel.HostArray(tmpl.input_shape, np.int8, args.ctx)
        h[...] = np.frombuffer(rng.bytes(h.nbytes), np.int8).reshape(h.shape)
        frames.append(h)
    beams = [accel.HostArray(tmpl.output_shape, np.int8, args.ctx) for _ in range(depth)]
    h2d = copy_rate(args, frames[0], "h2d")
    d2h = copy_rate(args, frames[1 % depth], "d2h")
    d = delay_model(np, rng, tmpl.delay_shape)
    with tmpl.instantiate() as sb:
        sb.set_delays(d)
        for k in range(2 * depth):  # warm-up: pipeline, clocks
            sb.submit(frames[k % depth], beams[k % depth])
        sb.flush()
        tickets = []
        t = time.perf_counter()
        for k in range(args.stream_frames):
            if k >= depth:
                sb.wait(tickets[k - depth])
            tickets.append(sb.submit(frames[k % depth], beams[k % depth]))
        sb.wait(tickets[-1])
        dt = time.perf_counter() - t
        stages = np.array([sb.stage_ms(tk) for tk in tickets[-depth:]])
    samples = A * 2 * C * T * B * args.stream_frames
    rate = samples / dt / 1e9
    bound = h2d / 2  # 2 bytes per complex 8-bit sample
    return {"workload": "cfg5: streaming ingest, config-3 frames (64 ants, 16 beams, 4096 ch, T=256, B=1: 256 MiB "
                        "int8 voltages in, 64 MiB int8 beams out) through the pinned host ring (BASELINE configs[4])",
            "kind": "streaming", "output": "int8", "value": round(rate, 2), "unit": "Gsamples/s", "n_gpus": 1,
            "frames": args.stream_frames, "depth": depth, "seconds": round(dt, 4),
            "frames_per_s": round(args.stream_frames / dt, 1),
            "pcie_copy_GBps": {"h2d": round(h2d, 2), "d2h": round(d2h, 2),
                               "note": "bf_memcpy_{h2d,d2h} of one pinned 256 MiB frame, one stream, this process"},
            "h2d_bound_Gsamples_s": round(bound, 2), "frac_of_h2d_bound": round(rate / bound, 4),
            "stage_ms_median": {"h2d": round(float(np.median(stages[:, 0])), 3),
                                "compute": round(float(np.median(stages[:, 1])), 3),
                                "d2h": round(float(np.median(stages[:, 2])), 3)},
            "pipeline": "bf_pipeline (csrc/bf_pipeline.cpp): H2D / compute / D2H HIP streams, per-slot events"}


def host_cpus():
    """(CPUs in this process's affinity mask, the cgroup CPU quota in cores or None)."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        affinity = os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return int(affinity), quota


def cpu_baseline(wl, out_int8, seconds=10.0):
    """The oracle's vectorised NumPy restatement (reorder -> per-batch coefficients -> f32 matmul) timed on
    this host on a bounded channel sample of the same workload (kind "port"): the same delay model as the timed GPU
    run (bench.delay_model: delays, delay rates, phases, phase rates), BLAS threads = every CPU in the affinity
    mask (the baseline uses the host's cores; `cores` is that thread count)."""
    import numpy as np

    import oracle as O
    affinity, quota = host_cpus()
    try:
        from threadpoolctl import threadpool_limits
        limiter = threadpool_limits(limits=affinity, user_api="blas")
    except Exception:  # noqa: BLE001 -- threadpoolctl missing: the BLAS default (reported below)
        limiter = None
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("user_api") == "blas"] or [1])
    except Exception:  # noqa: BLE001
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    A, M, T, B = wl["A"], wl["M"], wl["T"], wl["B"]
    Ctot = wl.get("Ctot", wl["C"])
    rng = np.random.default_rng(7)
    d = delay_model(np, rng, (1, M, A, 4))

    def once(c):
        raw = rng.integers(-128, 128, size=(B, A, c, T, 2, 2), dtype=np.int8)
        t = time.perf_counter()
        y = O.fused_beamform(raw, d, Ctot, signed=True, t0=0.0, batch_dt=T * 2 * Ctot * TS)
        if out_int8:
            O.requantise(y, 1 / 64)
        return time.perf_counter() - t

    try:
        c = 16
        once(c)  # warm-up
        dt = once(c)  # rate estimate
        c = int(min(max(16, c * seconds / max(dt, 1e-3)), wl["C"]))
        dt = once(c)
    finally:
        if limiter is not None:
            limiter.unregister()
    rate = A * 2 * c * T * B / dt / 1e9
    return {"value": round(rate, 4), "unit": "Gsamples/s", "cores": int(threads), "blas_threads": int(threads),
            "host_cpus_in_affinity": affinity, "cgroup_cpu_quota_cores": quota, "kind": "port",
            "threads_note": "BLAS threads = the affinity mask's CPUs, capped by the BLAS library's own thread maximum; "
                            "the cgroup quota bounds the CPU time those threads get",
            "sample": f"{c} of {wl['C']} channels x B={B} x T={T} x A={A} x 2 pols ({dt:.1f} s), extrapolated "
                      f"linearly in channels: oracle.fused_beamform (NumPy reorder + float64-phase coefficients "
                      f"with delay/phase rates + float32 matmul{' + requantise' if out_int8 else ''}, "
                      f"BLAS threads={threads})"}


def pmc_pass(args, counters, workload, output, contract):
    """One rocprofv3 --pmc pass over a short child run of the fused launch (3 timed + 1 warm-up dispatches): the
    median per-dispatch value of each counter over the `beamform_fused*` kernels, or (None, error)."""
    exe = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 not found"
    out = tempfile.mkdtemp(prefix="bfpmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = [exe, "--pmc", *counters, "--output-format", "csv", "-d", out, "-o", "pmc", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", workload,
           "--steps", "3", "--warmup", "1", "--settle-ms", "0", "--output", output,
           "--int8-contract", contract] + (["--unsigned"] if args.unsigned else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    files = glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True)
    if r.returncode != 0 or not files:
        return None, f"rocprofv3 {' '.join(counters)} failed rc={r.returncode}: {r.stderr[-300:]}"
    vals = {}
    for counter in counters:
        per = []
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if "beamform_fused" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    per.append(float(row["Counter_Value"]))
        if not per:
            return None, f"no {counter} rows for the fused kernel"
        vals[counter] = sorted(per)[len(per) // 2]
    return vals, None


MFMA_COUNTERS = ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")


def pmc_traffic(args):
    """HBM bytes per fused launch from rocprofv3 counters: FETCH_SIZE and WRITE_SIZE in separate passes
    (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reads 1/2 of a wide coalesced stream -> x2; WRITE_SIZE exact; KiB).
    Calibrated in-repo (tools/pmc_calibrate.py, profiles/r2_v_pmc_calibration.jsonl): a 1 GiB streaming read gives
    FETCH_SIZE = 0.500 x the bytes (every request a 128-byte TCC_EA0_RDREQ_128B, tallied at 64 B), a 1 GiB write
    WRITE_SIZE = 1.000 x, and a 1 GiB + 256 MiB mix the same two ratios.  A third pass takes the matrix pipe's busy
    cycles (summed over the 1024 SIMDs) and the GPU-active cycles (summed over the 8 XCDs): the measured MFMA-busy
    fraction and the clock the chip held (MI355X_MICROARCH.md, DVFS); it is informational."""
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        v, err = pmc_pass(args, (counter,), args.workload, args.output, args.int8_contract)
        if err:
            return None, err
        vals.update(v)
    v, err = pmc_pass(args, MFMA_COUNTERS, args.workload, args.output, args.int8_contract)
    if not err:
        vals.update(v)
    traffic = (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0
    return traffic, vals


def pmc_mfma_busy(vals, kernel_s):
    """The measured matrix-pipe busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over 1024 SIMDs x the kernel's GPU-active
    cycles, GRBM_GUI_ACTIVE / 8 XCDs) and the clock the chip held (those cycles over the event-timed launch)."""
    if not isinstance(vals, dict) or "SQ_VALU_MFMA_BUSY_CYCLES" not in vals or not vals.get("GRBM_GUI_ACTIVE"):
        return None
    cycles = vals["GRBM_GUI_ACTIVE"] / 8.0
    return {"busy_frac": round(vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024.0 * cycles), 4),
            "clock_GHz": round(cycles / kernel_s / 1e9, 3),
            "counters": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), profiled pass"}


ADC_SAMPLE_RATE, FFT_SIZE = 1712e6, 8192  # MeerKAT L-band (BeamformerParameters.h:15-16)


def realtime(wl, n_gpus, value_gsps):
    """Real-time factor against MeerKAT ingest, as the reference's harness reports GPU utilisation
    (BeamformerCoefficientTest.cu:422-465: kernel time / the wall time the processed spectra represent): the band
    needs A * 2 pols * C * N channels * (ADC rate / FFT size) samples/s; `gpus_per_band` is that need over this
    run's whole-job rate x N (the reference's "GPUs required")."""
    spectra_per_s = ADC_SAMPLE_RATE / FFT_SIZE
    need = wl["A"] * 2 * wl["C"] * n_gpus * spectra_per_s / 1e9
    return {"ingest_need_Gsamples_s": round(need, 2), "realtime_factor": round(value_gsps / need, 2),
            "gpus_per_band": round(need / value_gsps * n_gpus, 4),
            "basis": f"{wl['A']} ants x 2 pols x {wl['C'] * n_gpus} channels x {spectra_per_s:.1f} spectra/s "
                     "(ADC 1712 MHz / FFT 8192, BeamformerParameters.h:15-16; BeamformerCoefficientTest.cu:422-465)"}


def rocprof_check(args, n_secondary):
    """The same bench (headline + secondaries, no PMC / CPU baseline / ceiling) re-run as a child under
    `rocprofv3 --kernel-trace`; each timed region (bracketed by bf_trace_mark dispatches) summarised per kernel by
    tools/kernel_stats.py.  Returns ([region stats], the child's own JSON line) -- the child's events and its
    profiled kernel durations come from the same process, so they must agree."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_stats
    exe = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, None, "rocprofv3 not found"
    out = args.prof_out or tempfile.mkdtemp(prefix="bfprof_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(out, exist_ok=True)
    cmd = [exe, "--kernel-trace", "--stats", "--output-format", "csv", "-d", out, "-o", "bench", "--", sys.executable,
           os.path.abspath(__file__), "--prof-child", "--workload", args.workload, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--settle-ms", str(args.settle_ms), "--output", args.output,
           "--int8-contract", args.int8_contract, "--coeff-table", args.coeff_table, "--no-pmc", "--no-cpu-baseline",
           "--no-ceiling", "--no-stream"]
    cmd += (["--unsigned"] if args.unsigned else []) + (["--no-secondary"] if n_secondary == 0 else [])
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    files = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not files:
        return None, None, f"rocprofv3 failed rc={r.returncode}: {r.stderr[-300:]}"
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    child = json.loads(lines[-1]) if lines else None
    regions = kernel_stats.region_stats(files[0])
    kernel_stats.write_csv(regions, os.path.join(out, "timed_kernel_stats.csv"))
    if child is not None:
        with open(os.path.join(out, "prof_bench.json"), "w") as f:
            f.write(json.dumps(child) + "\n")
    return regions, child, None


def short_kernel(name):
    """'void bf::(anonymous namespace)::k<true, 2>(bf::FusedArgs)' -> 'k<true, 2>'."""
    name = name.replace("(anonymous namespace)::", "")
    name = name[5:] if name.startswith("void ") else name
    return name.split("(")[0].split("::")[-1][:70]


def rocprof_entry(regions, i, kernel, alg_bytes):
    """The timed dispatches of `kernel` in region i: count, average / median duration, roofline fraction."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import kernel_stats
    if regions is None or i >= len(regions):
        return None
    name, s = kernel_stats.dominant(regions[i], "::" + kernel + "<")
    if s is None:
        return {"error": f"no {kernel} dispatches in timed region {i}"}
    steps = s["Calls"]
    # every kernel of the timed steps (config 4's int8 path: the coefficient generator + the contraction)
    per_step_ns = sum(v["TotalDurationNs"] for v in regions[i].values()) / steps
    out = {"kernel_instance": name, "timed_dispatches": steps, "avg_us": round(s["AverageNs"] / 1e3, 2),
           "median_us": round(s["MedianNs"] / 1e3, 2), "max_us": round(s["MaxNs"] / 1e3, 2),
           "frac": round(alg_bytes / (per_step_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)}
    if len(regions[i]) > 1:
        out["per_step_us_all_kernels"] = round(per_step_ns / 1e3, 2)
        out["kernels_us_per_step"] = {short_kernel(k): round(v["TotalDurationNs"] / steps / 1e3, 2)
                                      for k, v in regions[i].items()}
    return out


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


def mfma_split(sec, ent):
    """A two-kernel step (config 4's int8 path: the Q14 generator, then the contraction): the matrix-core rates of the
    contraction alone, over its own rocprof time, and the generator's share of the step."""
    per = ent.get("kernels_us_per_step")
    if not per or "mfma" not in sec or "avg_us" not in ent:
        return
    contraction_us = ent["avg_us"]
    total_us = ent.get("per_step_us_all_kernels") or sum(per.values())
    scale = sec["avg_launch_us"] / contraction_us  # the rates scale with 1 / time
    m = sec["mfma"]
    m["contraction_only"] = {"kernel_us": contraction_us, "algorithmic": round(m["algorithmic"] * scale, 1),
                             "issued": round(m["issued"] * scale, 1),
                             "frac_issued": round(m["frac_issued"] * scale, 4)}
    m["generator_share_of_step"] = round(1.0 - contraction_us / total_us, 4)


def kernel_name(wl, out_int8, int8_contract="q14", coeff_table="on", signed=True):
    """The launch's dominant kernel (bf_fused.hip dispatch): item kernels for A <= 64 and T <= 256, else the wide
    kernels; the int8 32-beam path with a coefficient table (A <= 256) is a table-driven contraction after its
    generator (q14_table_kernel, reported per step beside it): at config 4's shape with int8 samples the LDS-DMA
    ring kernel (w32r: 224 < A <= 256, T = 256, M % 32 == 0), else the register-ring kernel (w32t).  Float beams at
    A = 256, T = 256, M % 32 == 0 (one delay model, no weights, fast coefficients): the persistent wide kernel."""
    integer = out_int8 and int8_contract == "q14"
    if wl["A"] <= 64 and wl["T"] <= 256:
        return "beamform_fused_i8_item_kernel" if integer else "beamform_fused_item_kernel"
    if integer:
        if coeff_table != "on" or wl["A"] > 256:
            return "beamform_fused_i8_w32_kernel"
        if signed and 224 < wl["A"] <= 256 and wl["T"] == 256 and wl["M"] % 32 == 0:
            return "beamform_fused_i8_w32r_kernel"
        return "beamform_fused_i8_w32t_kernel"
    if not out_int8 and wl["A"] == 256 and wl["T"] == 256 and wl["M"] % 32 == 0:
        return "beamform_fused_wide_p2_kernel"
    return "beamform_fused_wide_kernel"


def secondary(args, dist, workload, out_int8, int8_contract="q14"):
    sub = argparse.Namespace(**{**vars(args), "workload": workload, "out_int8": out_int8,
                                "int8_contract": int8_contract})
    wl = WORKLOADS[workload]
    r = run_gpu(sub, dist, wl)
    r.pop("ops")
    out = {"workload": workload + ": " + wl["desc"],
           "output": ("int8" + ("" if int8_contract == "q14" else " (requantised from float32 beams)"))
           if out_int8 else "float32",
           "kernel": kernel_name(wl, out_int8, int8_contract, args.coeff_table, not args.unsigned),
           "value": round(r["samples_per_step"] * args.steps * dist.world / r["t_max"] / 1e9, 2),
           "unit": "Gsamples/s", "n_gpus": dist.world,
           "roofline_frac": round(r["alg_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
           "read_frac": round(r["read_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
           "avg_launch_us": round(r["kernel_s"] * 1e6, 2), "alg_bytes_per_launch": r["alg_bytes"],
           "mfma": mfma_util(wl, out_int8, int8_contract, r["kernel_s"])}
    if dist.group:  # every rank's own launch time (each rank its own X-engine's channels)
        out["per_rank_avg_launch_us"] = dist.group.gather_json(round(r["kernel_s"] * 1e6, 2))
    if not args.no_ceiling and dist.world == 1:
        ceil = stream_ceiling(args, r["read_bytes"], int(r["alg_bytes"] - r["read_bytes"]))
        if ceil:
            out["ceiling"] = ceil
            out["frac_of_ceiling"] = round(ceil["us"] / out["avg_launch_us"], 4)
            out["read_frac_ceiling"] = round(r["read_bytes"] / (ceil["us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
            out.update(target_block(r["alg_bytes"], ceil["us"]))
    return out


NORTH_STAR_FRAC = 0.70  # BASELINE.json north_star: >= 70 % of the HBM roofline at 1 GPU


def target_block(alg_bytes, ceiling_us, target=NORTH_STAR_FRAC):
    """Whether the north star's 0.70 of 8 TB/s is reachable for this byte mix on this box: `ceiling_frac` is the
    roofline fraction a kernel running exactly at the box's best plain stream over the same read/write bytes would
    show; `target_needs_frac_of_ceiling` what fraction of that stream the target asks for (> 1: above any stream)."""
    ceiling_frac = alg_bytes / (ceiling_us * 1e-6) / 1e9 / HBM_PEAK_GBS
    return {"target_frac": target, "ceiling_frac": round(ceiling_frac, 4),
            "target_reachable": bool(ceiling_frac >= target),
            "target_needs_frac_of_ceiling": round(target / ceiling_frac, 4)}


def main():
    args = parse()
    world, launch = resolve_world(args)
    if launch:  # before anything touches the GPU: this process only starts and waits for the ranks
        sys.exit(launch_ranks(world, sys.argv[1:]))
    wl = WORKLOADS[args.workload]
    dist = Dist(args.scatter_backend, force=args.scatter_at_one)
    if args.rank_probe:  # the ranks' rendezvous and timing-bracket collectives only, no GPU (tests/test_bench_logic.py)
        dist.barrier()
        top = dist.max(float(dist.rank))
        got = dist.group.gather_json({"rank": dist.rank, "local_rank": dist.local_rank, "pid": os.getpid()}) \
            if dist.group else [{"rank": 0, "local_rank": 0, "pid": os.getpid()}]
        if dist.rank == 0:
            print(json.dumps({"n_gpus": dist.world, "gpus_arg": args.gpus, "max_rank": top, "ranks": got,
                              "ranks_launched_by": os.environ.get("BF_BENCH_LAUNCHER")}), flush=True)
        time.sleep(args.probe_sleep)
        dist.close()
        return
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
        # the ranks agree over the TCP group and generate their shards in place, so the timed line is still produced
        err = None
        try:
            inputs, scatter = scatter_inputs(args, dist, tmpl.input_shape)
        except Exception as e:  # noqa: BLE001 -- reported in the line's scatter block
            err = f"{type(e).__name__}: {str(e)[:300]}"
        if dist.max(1.0 if err else 0.0) > 0:
            inputs = None
            scatter = {"backend": dist.scatter_backend, "error": err or "failed on another rank",
                       "note": "scatter failed; each rank generated its shard in place"}
    # top level, so a failed or unverified collective cannot pass for a clean scaling point (None: no scatter)
    scatter_ok = None if scatter is None else ("error" not in scatter and scatter.get("verified", True) is not False)
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
                   "parallelism": f"channel-shard x{dist.world} (xeng_id = rank), no data-path collective",
                   "ranks_launched_by": os.environ.get("BF_BENCH_LAUNCHER") or
                   ("external launcher (WORLD_SIZE)" if "WORLD_SIZE" in os.environ else "single process")},
        "beams_per_s": round(r["beams_per_step"] * args.steps * dist.world / r["t_max"], 1),
        "compute": compute_desc(args.out_int8, args.int8_contract),
        "device": args.ctx.device.name,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "read_frac": round(r["read_bytes"] / r["kernel_s"] / 1e9 / HBM_PEAK_GBS, 4),
                     "kernel": kernel_name(wl, args.out_int8, args.int8_contract, args.coeff_table,
                                           not args.unsigned),
                     "avg_launch_us": round(r["kernel_s"] * 1e6, 2), "alg_bytes_per_launch": r["alg_bytes"],
                     "read_bytes_per_launch": r["read_bytes"]},
        "mfma": mfma_util(wl, args.out_int8, args.int8_contract, r["kernel_s"]),
        "scatter_ok": scatter_ok,
        "scatter": scatter or {"backend": None, "note": "no scatter: single rank, or --scatter-backend none "
                                                        "(each rank generates its shard in place)"},
        "realtime": realtime(wl, dist.world, value),
        "cpu_baseline": None,
    }
    if dist.group:
        line["per_rank_avg_launch_us"] = dist.group.gather_json(round(r["kernel_s"] * 1e6, 2))
    if dist.rank == 0 and dist.world == 1 and args.out_int8 and args.int8_contract == "q14" and not args.prof_child:
        line["int8_contract_check"] = contract_check(args, dist, wl, r)
    r.pop("ops")
    if dist.rank == 0 and dist.world == 1 and not args.no_ceiling:
        ceil = stream_ceiling(args, r["read_bytes"], int(r["alg_bytes"] - r["read_bytes"]))
        if ceil:
            line["ceiling"] = ceil
            line["roofline"]["frac_of_ceiling"] = round(ceil["us"] / line["roofline"]["avg_launch_us"], 4)
            # the north star's "HBM-read roofline": with the beams written too, a read-only fraction of 1 is not
            # reachable; the best this box allows is the voltage bytes over its own stream time for the same mix
            line["roofline"]["read_frac_ceiling"] = round(r["read_bytes"] / (ceil["us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
            line["roofline"].update(target_block(r["alg_bytes"], ceil["us"]))
    if not args.no_secondary and args.workload == "cfg3":
        # every rank runs the secondaries (each is timed between barriers, max over ranks); at N > 1 config 4
        # channel-sharded: 4096 channels per rank of the 32768-channel band (BASELINE configs[3] at N = 8)
        line["secondary"] = []
        cases = [("cfg2", args.out_int8, "q14"), ("cfg3", not args.out_int8, "q14"), ("cfg3", True, "f32"),
                 ("cfg4", True, "q14"), ("cfg4", False, "q14")]
        if dist.world > 1:
            cases = [("cfg4", True, "q14"), ("cfg4", False, "q14")]
        for workload, out_int8, contract in cases:
            if (workload, out_int8, contract if out_int8 else "q14") == (args.workload, args.out_int8,
                                                                          args.int8_contract if args.out_int8 else "q14"):
                continue
            try:
                line["secondary"].append(secondary(args, dist, workload, out_int8, contract))
            except Exception as e:  # secondary lines are informational
                line["secondary"].append({"workload": workload, "error": str(e)[:200]})
    if dist.rank == 0 and dist.world == 1 and not (args.no_stream or args.prof_child):
        try:
            line.setdefault("secondary", []).append(stream_secondary(args))
        except Exception as e:  # noqa: BLE001 -- informational
            line.setdefault("secondary", []).append({"workload": "cfg5", "kind": "streaming",
                                                     "error": f"{type(e).__name__}: {str(e)[:200]}"})
    if dist.rank == 0 and dist.world == 1 and not (args.no_rocprof or args.prof_child):
        # the timed regions of the profiled child: the headline, then each device-resident secondary in order
        secs = [s for s in line.get("secondary", []) if "error" not in s and s.get("kind") != "streaming"]
        try:
            regions, child, err = rocprof_check(args, len(secs))
        except Exception as e:  # informational: the live event timing above is the measurement
            regions, child, err = None, None, f"{type(e).__name__}: {str(e)[:200]}"
        if err:
            line["roofline"]["rocprof"] = {"error": err}
        else:
            ent = rocprof_entry(regions, 0, line["roofline"]["kernel"], r["alg_bytes"]) or {}
            ent.update({"profiled_run_ms_per_step": child.get("ms_per_step") if child else None,
                        "profiled_run_event_avg_us": child["roofline"]["avg_launch_us"] if child else None,
                        "source": "rocprofv3 --kernel-trace re-run of this bench (same args, child process): the "
                                  "timed dispatches only, between the two bf_trace_mark dispatches of each timed "
                                  "region (tools/kernel_stats.py)"})
            line["roofline"]["rocprof"] = ent
            for i, s in enumerate(secs):
                e = rocprof_entry(regions, i + 1, s["kernel"], s["alg_bytes_per_launch"])
                if e:
                    s["rocprof"] = e
                    mfma_split(s, e)
    if dist.rank == 0 and dist.world == 1 and not args.no_pmc:
        try:
            traffic, info = pmc_traffic(args)
            line["roofline"]["traffic"] = traffic
            line["roofline"]["traffic_counters"] = info
            busy = pmc_mfma_busy(info, r["kernel_s"])
            if busy and isinstance(line.get("mfma"), dict):
                line["mfma"]["pmc"] = busy
            # config 4 (the MFMA-heavy shape): the same measured busy fraction for its secondary lines' kernels
            for sec in line.get("secondary", []):
                if "error" in sec or not sec["workload"].startswith("cfg4") or not isinstance(sec.get("mfma"), dict):
                    continue
                out_int8 = sec["output"].startswith("int8")
                contract = "f32" if "requantised" in sec["output"] else "q14"
                v, err = pmc_pass(args, MFMA_COUNTERS, "cfg4", "int8" if out_int8 else "f32", contract)
                # the counters cover the beamform_fused* kernel only: the int8 line's contraction, not its generator
                kernel_us = sec["mfma"].get("contraction_only", {}).get("kernel_us", sec["avg_launch_us"])
                busy = None if err else pmc_mfma_busy(v, kernel_us * 1e-6)
                sec["mfma"]["pmc"] = busy or {"error": err or "no counters"}
        except Exception as e:
            line["roofline"]["traffic_counters"] = f"unavailable: {str(e)[:200]}"
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(wl, args.out_int8)
    if dist.rank == 0:
        print(json.dumps(line), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
