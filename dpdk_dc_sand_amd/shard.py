"""Frequency-channel sharding across X-engines (one process per GPU).

The reference's only parallel axis is the X-engine index: engine `xeng_id` owns `n_channels_per_stream` channels
whose absolute index is `c + n_channels_per_stream * xeng_id` (coeff_generator.py:49-53,
coeff_generator_cpu.py:134-141).  Here rank r of a world of N is X-engine r.  Beamforming itself needs no collective;
the only data movement is the root -> ranks channel scatter of a full-band voltage cube, kept out of
the timed hot path:
  * `ChannelScatter`: device to device over RCCL/xGMI through libbf (bf_comm_create + bf_channel_scatter,
    include/bf.h) -- the multi-GPU path;
  * `scatter_channel_slices` / `gather_channel_slices`: host memory over a `rendezvous.HostGroup` -- rehearsals with
    several ranks on one GPU (RCCL refuses two ranks on one device) and verification.
No torch: every rank runs libbf on one HIP runtime.
"""
import ctypes
import json

import numpy as np

from . import _lib


def shard_channels(n_channels, world_size):
    """Per-rank (xeng_id, first channel, n_channels_per_stream).  The reference's absolute-channel formula needs
    equal shards, so n_channels must divide evenly."""
    if world_size < 1 or n_channels % world_size:
        raise ValueError(f"n_channels={n_channels} does not split evenly over {world_size} X-engines")
    per = n_channels // world_size
    return [(r, r * per, per) for r in range(world_size)]


def pack_channel_slices(raw, world_size):
    """Split a full-band raw cube (B, A, Ctot, T, 2, 2) into per-rank contiguous (B, A, C, T, 2, 2) cubes.
    A channel slice of the raw layout is B*A strided runs of C*T*4 bytes; packing makes each rank's part one
    contiguous message (bf_channel_scatter does the same on the device with one 2-D copy per peer)."""
    raw = np.asarray(raw)
    Ctot = raw.shape[2]
    return [np.ascontiguousarray(raw[:, :, s:s + n]) for _, s, n in shard_channels(Ctot, world_size)]


def scatter_channel_slices(raw, shape, dtype, group):
    """Root (rank 0 of `group`, a rendezvous.HostGroup) scatters the packed channel slices of `raw`
    (B, A, Ctot, T, 2, 2) through host memory; every rank returns its (B, A, Ctot / N, T, 2, 2) slice.  `shape` is
    the per-rank slice shape (all ranks know it); `raw` is only read on rank 0."""
    parts = [p.tobytes() for p in pack_channel_slices(raw, group.world)] if group.rank == 0 else None
    mine = group.scatter_bytes(parts)
    return np.frombuffer(mine, np.dtype(dtype)).reshape(shape).copy()


def gather_channel_slices(part, group):
    """Inverse of the scatter for beams (B, 2, C, T/16, 16, 2M) (verification only): rank 0 returns the full band,
    the other ranks None."""
    part = np.ascontiguousarray(part)
    got = group.gather_bytes(part.tobytes())
    if got is None:
        return None
    return np.concatenate([np.frombuffer(g, part.dtype).reshape(part.shape) for g in got], axis=2)


class ScatterOp(ctypes.Structure):
    """include/bf.h bf_scatter_op."""
    _fields_ = [("kind", ctypes.c_int), ("peer", ctypes.c_int), ("group", ctypes.c_int), ("src_space", ctypes.c_int),
                ("dst_space", ctypes.c_int), ("reserved", ctypes.c_int), ("src_off", ctypes.c_ulonglong),
                ("src_pitch", ctypes.c_ulonglong), ("dst_off", ctypes.c_ulonglong), ("dst_pitch", ctypes.c_ulonglong),
                ("width", ctypes.c_ulonglong), ("height", ctypes.c_ulonglong)]


SCATTER_COPY2D, SCATTER_SEND, SCATTER_RECV = 1, 2, 3
SPACE_BAND, SPACE_STAGING, SPACE_SLICE = 1, 2, 3


def scatter_plan(nranks, rank, root, B, A, C, T, chunk=0):
    """libbf's operation list for one rank's part of bf_channel_scatter (bf_scatter_plan: host arithmetic only, the
    list the scatter executes).  Returns ([op dicts], staging bytes)."""
    n, staging = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.call("bf_scatter_plan", nranks, rank, root, B, A, C, T, chunk, None, 0, ctypes.byref(n), ctypes.byref(staging))
    ops = (ScatterOp * max(n.value, 1))()
    _lib.call("bf_scatter_plan", nranks, rank, root, B, A, C, T, chunk, ops, n.value, ctypes.byref(n),
              ctypes.byref(staging))
    return [{f: getattr(o, f) for f, _ in ScatterOp._fields_} for o in ops[:n.value]], staging.value


class ChannelScatter:
    """The RCCL channel scatter of libbf (bf_comm_* / bf_channel_scatter).  Rank 0 makes the communicator id and
    `group` (a rendezvous.HostGroup) hands it to every rank; the communicator lives on `context`'s device.

    bf_comm_create is a blocking RCCL collective, so every rank first checks its local preconditions (the device can
    be made current, RCCL loads) and the ranks agree over `group` before any of them calls it: a rank that fails
    early makes every rank raise instead of leaving the others waiting inside ncclCommInitRank."""

    def __init__(self, group, context):
        self.group, self.context = group, context
        self.rank, self.world = group.rank, group.world
        self.handle = None
        uid, err = None, None
        if self.rank == 0:
            buf = ctypes.create_string_buffer(128)
            try:
                _lib.call("bf_comm_unique_id", buf, 128)
                uid = buf.raw
            except _lib.BeamformerError as e:  # every rank must learn it, or the others wait for an id forever
                uid, err = b"", e
        uid = group.broadcast_bytes(uid)
        if not uid:
            raise err or RuntimeError("rank 0 could not create the RCCL communicator id")
        local = None
        try:
            context.activate()
            _lib.call("bf_comm_load")
        except Exception as e:  # noqa: BLE001 -- reported on every rank below
            local = e
        if group.allreduce_any(local is not None):
            raise local or RuntimeError("RCCL communicator set-up failed on another rank")
        h = ctypes.c_void_p()
        _lib.call("bf_comm_create", ctypes.byref(h), uid, len(uid), self.world, self.rank)
        self.handle = h.value

    def scatter(self, band, out, B, A, C, T, queue, root=0):
        """Stream-ordered on `queue`: band (B, A, C*N, T, 2, 2) device array on `root` (None elsewhere) -> `out`
        (B, A, C, T, 2, 2) device array on every rank: the peers' slices through RCCL (ncclSend/ncclRecv), the
        root's own by a 2-D copy -- at one rank by a self send/recv instead, so one GPU runs the RCCL path too."""
        _lib.call("bf_channel_scatter", self.handle, _lib.ptr(band), _lib.ptr(out), B, A, C, T, root, queue.handle)

    def stats(self):
        """(bytes handed to ncclSend, bytes received through ncclRecv) on this rank so far."""
        s, r = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        _lib.call("bf_comm_stats", self.handle, ctypes.byref(s), ctypes.byref(r))
        return s.value, r.value

    def verify(self, band, out, B, A, C, T, queue, root=0):
        """Check every rank's received slice against the root's band without moving either to the host: each rank
        checksums its slice (bf_checksum), the root checksums each rank's strided region of the band, rank 0 (the
        host group's hub) compares them and every rank learns the outcome.  Returns (ok on every rank, [per-rank
        dict] on the root else None)."""
        if not 0 <= root < self.world:
            raise ValueError(f"root {root} of {self.world} ranks")
        payload = {"rank": self.rank, "checksum": device_checksum(out, C * T * 4 * B * A, 0, 1, queue)}
        if self.rank == root:
            run = C * T * 4
            payload["want"] = [device_checksum(_lib.ptr(band) + run * r, run, run * self.world, B * A, queue)
                               for r in range(self.world)]
        got = self.group.gather_json(payload)
        report = None
        if self.rank == 0:
            want = next(g["want"] for g in got if g["rank"] == root)
            report = [{"rank": g["rank"], "checksum": f"{g['checksum']:016x}", "match": g["checksum"] == want[g["rank"]]}
                      for g in sorted(got, key=lambda g: g["rank"])]
        report = json.loads(self.group.broadcast_bytes(json.dumps(report).encode() if self.rank == 0 else None))
        return all(r["match"] for r in report), (report if self.rank == root else None)

    def allreduce_max(self, value):
        v = ctypes.c_double(float(value))
        _lib.call("bf_comm_allreduce_max", self.handle, ctypes.byref(v))
        return v.value

    def close(self):
        if getattr(self, "handle", None):
            _lib.call("bf_comm_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_checksum(src, run_bytes, pitch_bytes, rows, queue):
    """bf_checksum of a 2-D device region (rows x run_bytes, pitch_bytes apart) on `queue`'s stream."""
    out = ctypes.c_ulonglong()
    _lib.call("bf_checksum", _lib.ptr(src), run_bytes, pitch_bytes, rows, ctypes.byref(out), queue.handle)
    return out.value


def host_checksum(words):
    """CPU restatement of bf_checksum over a packed array of uint32 words (tests)."""
    w = np.ascontiguousarray(words).reshape(-1).view(np.uint32).astype(np.uint64)
    i = np.arange(w.size, dtype=np.uint64)
    return int(np.sum(_splitmix64(_splitmix64(i) ^ w), dtype=np.uint64))


def _splitmix64(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))
