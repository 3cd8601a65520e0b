"""Multi-rank (X-engine) logic on CPU: world-2 and world-3 process groups over the TCP rendezvous.

Checks the channel-shard arithmetic, the host group's collectives (barrier, max, broadcast -- the RCCL id hand-out
--, scatter, gather), the root -> ranks channel scatter / gather helpers, that beamforming each shard with
xeng_id = rank reproduces the full-band result exactly (the reference's absolute-channel convention,
coeff_generator.py:49-53), bench.py's timing bracket (barrier + max over ranks), and the C ABI's communicator
argument checks (no GPU needed: they fail before RCCL is touched)."""
import ctypes
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dpdk_dc_sand_amd import _lib  # noqa: E402
from dpdk_dc_sand_amd.shard import pack_channel_slices, shard_channels  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_channels():
    assert shard_channels(4096 * 8, 8)[3] == (3, 3 * 4096, 4096)
    with pytest.raises(ValueError):
        shard_channels(1000, 3)


def test_pack_channel_slices_roundtrip():
    raw = np.arange(2 * 3 * 8 * 16 * 4, dtype=np.int64).reshape(2, 3, 8, 16, 2, 2)
    parts = pack_channel_slices(raw, 4)
    assert all(p.flags.c_contiguous and p.shape == (2, 3, 2, 16, 2, 2) for p in parts)
    np.testing.assert_array_equal(np.concatenate(parts, axis=2), raw)


def _run_world(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return sorted(results)


def _group_worker(rank, world, port, q):
    from dpdk_dc_sand_amd.rendezvous import HostGroup
    try:
        g = HostGroup(rank, world, "127.0.0.1", port)
        g.barrier()
        mx = g.allreduce_max(10.0 - rank)
        uid = g.broadcast_bytes(bytes(range(128)) if rank == 0 else None)  # the RCCL id hand-out
        part = g.scatter_bytes([bytes([r]) * (r + 1) for r in range(world)] if rank == 0 else None)
        got = g.gather_bytes(bytes([rank + 100]))
        js = g.gather_json({"rank": rank})
        anyf = g.allreduce_any(rank == world - 1)
        g.barrier()
        g.close()
        q.put((rank, "ok", mx, uid == bytes(range(128)), part == bytes([rank]) * (rank + 1),
               got == [bytes([r + 100]) for r in range(world)] if rank == 0 else got is None,
               js == [{"rank": r} for r in range(world)] if rank == 0 else js is None, anyf))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error " + repr(e), None, None, None, None, None, None))


@pytest.mark.parametrize("world", [2, 3])
def test_host_group_collectives(world):
    for rank, status, mx, uid_ok, part_ok, gather_ok, json_ok, anyf in _run_world(_group_worker, world):
        assert status == "ok", status
        assert mx == 10.0 and uid_ok and part_ok and gather_ok and json_ok and anyf, rank


def _shard_worker(rank, world, port, q):
    import oracle as O
    from dpdk_dc_sand_amd.rendezvous import HostGroup
    from dpdk_dc_sand_amd.shard import gather_channel_slices, scatter_channel_slices
    try:
        g = HostGroup(rank, world, "127.0.0.1", port)
        B, A, M, T, Ctot = 2, 5, 3, 32, 8
        C = Ctot // world
        raw = O.u8_voltages((B, A, Ctot, T, 2, 2), seed=11) if rank == 0 else None
        d = np.zeros((1, M, A, 4), np.float32)
        rng = np.random.default_rng(3)
        d[..., 0] = rng.uniform(0, 10 * O.TS_MEERKAT, (1, M, A))
        d[..., 2] = rng.uniform(-np.pi, np.pi, (1, M, A))
        mine = scatter_channel_slices(raw, (B, A, C, T, 2, 2), np.uint8, g)
        beams = O.fused_beamform(mine, d, Ctot, xeng_id=rank)  # this X-engine's channels
        full = gather_channel_slices(beams, g)

        # bench.py's timing bracket: barrier + max over ranks, on the same kind of group
        from bench import Dist
        dd = Dist.__new__(Dist)
        dd.world, dd.rank, dd.local_rank, dd.group, dd.comm = world, rank, rank, g, None
        dd.barrier()
        mx = dd.max(float(rank + 1))
        equal = None
        if rank == 0:
            equal = bool(np.array_equal(full, O.fused_beamform(raw, d, Ctot, xeng_id=0)))
        g.close()
        q.put((rank, "ok", equal, mx))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error " + repr(e), None, None))


def test_channel_sharded_beamforming_matches_full_band():
    world = 2
    res = _run_world(_shard_worker, world)
    assert all(r[1] == "ok" for r in res), res
    assert res[0][2], "sharded beams differ from the full-band result"
    assert all(r[3] == float(world) for r in res)


def test_comm_argument_validation_without_gpu():
    h = ctypes.c_void_p()
    uid = bytes(128)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_comm_create", None, uid, 128, 2, 0)
    with pytest.raises(_lib.BeamformerError, match="128 bytes"):
        _lib.call("bf_comm_create", ctypes.byref(h), uid, 64, 2, 0)
    with pytest.raises(_lib.BeamformerError, match="rank 2 of 2"):
        _lib.call("bf_comm_create", ctypes.byref(h), uid, 128, 2, 2)
    with pytest.raises(_lib.BeamformerError, match="128-byte buffer"):
        _lib.call("bf_comm_unique_id", ctypes.create_string_buffer(16), 16)
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_channel_scatter", None, None, None, 1, 1, 1, 16, 0, None)
    assert _lib.load().bf_comm_destroy(None) == 0


def _stray_worker(rank, world, port, q):
    """Rank 0 of a world-2 group; before rank 1 connects, two strays do: one claiming rank 7 (out of range) and one
    claiming rank 0 (the root's own id).  Both must be dropped and the real rank 1 accepted."""
    import struct
    import time
    from dpdk_dc_sand_amd.rendezvous import HostGroup
    try:
        if rank == 0:
            g = HostGroup(0, world, "127.0.0.1", port)
            v = g.allreduce_max(1.0)
            rejected = list(g.rejected)
            g.close()
            q.put((rank, "ok", v, rejected))
        else:
            strays = []
            for bad in (7, 0):
                deadline = time.monotonic() + 60
                while True:
                    try:
                        s = socket.create_connection(("127.0.0.1", port), timeout=5.0)
                        break
                    except OSError:
                        if time.monotonic() > deadline:
                            raise
                        time.sleep(0.05)
                s.sendall(struct.pack("!I", bad))
                strays.append(s)
            time.sleep(0.5)
            g = HostGroup(1, world, "127.0.0.1", port)
            v = g.allreduce_max(2.0)
            g.close()
            for s in strays:
                s.close()
            q.put((rank, "ok", v, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error " + repr(e), None, None))


def test_rendezvous_rejects_stray_and_duplicate_rank_ids():
    res = _run_world(_stray_worker, 2)
    assert all(r[1] == "ok" for r in res), res
    assert res[0][2] == res[1][2] == 2.0
    assert sorted(res[0][3]) == [0, 7]


def test_host_checksum_restatement():
    """The CPU restatement of bf_checksum (shard.host_checksum, what the GPU kernel is tested against): position
    sensitive, and the strided band region of a rank equals its packed slice."""
    from dpdk_dc_sand_amd.shard import host_checksum
    rng = np.random.default_rng(2)
    band = rng.integers(0, 256, (2, 3, 4 * 8, 16, 2, 2), dtype=np.uint8)
    parts = pack_channel_slices(band, 4)
    sums = [host_checksum(p) for p in parts]
    assert len(set(sums)) == 4
    w = parts[1].reshape(-1).view(np.uint32).copy()
    w[[3, 5]] = w[[5, 3]]
    assert w[3] == w[5] or host_checksum(w) != sums[1]
    assert host_checksum(np.zeros(0, np.uint32)) == 0


def test_checksum_and_comm_stats_argument_validation_without_gpu():
    out = ctypes.c_ulonglong(5)
    with pytest.raises(_lib.BeamformerError, match="4-byte"):
        _lib.call("bf_checksum", 1 << 20, 6, 8, 2, ctypes.byref(out), None)
    assert out.value == 0
    _lib.call("bf_checksum", 1 << 20, 0, 0, 3, ctypes.byref(out), None)  # empty region: 0, no device touched
    with pytest.raises(_lib.BeamformerError, match="null pointer"):
        _lib.call("bf_comm_stats", None, ctypes.byref(out), ctypes.byref(out))


class _FakeDev:
    """A host array standing in for a device buffer: `ptr` is a fake address resolved by _fake_checksum."""
    registry = {}

    def __init__(self, arr, base):
        self.arr, self.ptr = np.ascontiguousarray(arr).reshape(-1).view(np.uint8), base
        _FakeDev.registry[base] = self


def _fake_checksum(src, run_bytes, pitch_bytes, rows, queue):
    from dpdk_dc_sand_amd.shard import host_checksum
    addr = src.ptr if isinstance(src, _FakeDev) else int(src)
    base = max(b for b in _FakeDev.registry if b <= addr)
    buf = _FakeDev.registry[base].arr[addr - base:]
    pitch = pitch_bytes or run_bytes
    return host_checksum(np.concatenate([buf[i * pitch:i * pitch + run_bytes] for i in range(rows)]))


def _verify_worker(rank, world, port, q, root, bad_rank):
    """ChannelScatter.verify over a world-`world` host group with the device checksums replaced by the host
    restatement: every rank's slice is compared with the root's band region, whichever rank is the root."""
    from dpdk_dc_sand_amd import shard
    from dpdk_dc_sand_amd.rendezvous import HostGroup
    try:
        shard.device_checksum = _fake_checksum
        g = HostGroup(rank, world, "127.0.0.1", port)
        B, A, C, T = 2, 3, 4, 8
        band = np.random.default_rng(1).integers(0, 256, (B, A, C * world, T, 2, 2), dtype=np.uint8)
        mine = pack_channel_slices(band, world)[rank].copy()
        if rank == bad_rank:
            mine[1, 2, 3, 4, 1, 0] ^= 1
        cs = shard.ChannelScatter.__new__(shard.ChannelScatter)
        cs.group, cs.rank, cs.world, cs.handle = g, rank, world, None
        ok, report = cs.verify(_FakeDev(band, 1 << 40) if rank == root else None, _FakeDev(mine, 1 << 41), B, A, C,
                               T, None, root=root)
        g.close()
        q.put((rank, "ok", ok, report))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, "error " + repr(e), None, None))


@pytest.mark.parametrize("root,bad_rank", [(0, None), (1, None), (2, 0), (1, 2)])
def test_scatter_verify_any_root(root, bad_rank):
    world = 3
    res = _run_world(_verify_worker, world, root, bad_rank)
    assert all(r[1] == "ok" for r in res), res
    assert all(r[2] == (bad_rank is None) for r in res), res
    for rank, _, _, report in res:
        if rank != root:
            assert report is None
        else:
            assert [x["rank"] for x in report] == [0, 1, 2]
            assert [x["match"] for x in report] == [r != bad_rank for r in range(world)]


def _replay_scatter(N, root, B, A, C, T, chunk):
    """Replay every rank's bf_scatter_plan (libbf's own operation list for bf_channel_scatter) on host buffers:
    COPY2D as strided byte copies, each SEND queued on its (root -> peer) link, each RECV taking the next message of
    its link in order (RCCL point-to-point matching).  Returns (band, per-rank slices, per-rank write counts of the
    slices, root staging write counts, bytes sent / received per rank)."""
    from dpdk_dc_sand_amd.shard import (SCATTER_COPY2D, SCATTER_RECV, SCATTER_SEND, SPACE_BAND, SPACE_SLICE,
                                        SPACE_STAGING, scatter_plan)
    rng = np.random.default_rng(N * 100 + root)
    run = C * T * 4
    slice_bytes = B * A * run
    band = rng.integers(0, 256, B * A * run * N, dtype=np.uint8)
    plans = {r: scatter_plan(N, r, root, B, A, C, T, chunk) for r in range(N)}
    staging = np.zeros(plans[root][1], np.uint8)
    staging_writes = np.zeros(plans[root][1], np.int32)
    slices = {r: np.zeros(slice_bytes, np.uint8) for r in range(N)}
    writes = {r: np.zeros(slice_bytes, np.int32) for r in range(N)}
    links = {r: [] for r in range(N)}  # root -> r, in send order
    sent = {r: 0 for r in range(N)}
    received = {r: 0 for r in range(N)}
    for r in range(N):
        assert plans[r][1] == (slice_bytes * (max(N - 1, 1)) if r == root else 0)

    def space(r, s):
        return {SPACE_BAND: (band, None), SPACE_STAGING: (staging, staging_writes),
                SPACE_SLICE: (slices[r], writes[r])}[s]

    def run_ops(r, ops):
        last_group, copies_open = -1, True
        for o in ops:
            assert o["group"] >= last_group
            if o["group"] != last_group:
                last_group, copies_open = o["group"], True
            if o["kind"] == SCATTER_COPY2D:
                assert r == root and copies_open, "a copy after its group's sends"
                src, _ = space(r, o["src_space"])
                dst, cnt = space(r, o["dst_space"])
                for h in range(o["height"]):
                    s0, d0 = o["src_off"] + h * o["src_pitch"], o["dst_off"] + h * o["dst_pitch"]
                    dst[d0:d0 + o["width"]] = src[s0:s0 + o["width"]]
                    cnt[d0:d0 + o["width"]] += 1
            elif o["kind"] == SCATTER_SEND:
                copies_open = False
                assert r == root and o["src_space"] == SPACE_STAGING
                src, _ = space(r, o["src_space"])
                links[o["peer"]].append(src[o["src_off"]:o["src_off"] + o["width"]].copy())
                sent[r] += o["width"]
            else:
                assert o["kind"] == SCATTER_RECV and o["peer"] == root and o["dst_space"] == SPACE_SLICE
                copies_open = False
                msg = links[r].pop(0)
                assert len(msg) == o["width"], "a receive paired with a send of another size"
                dst, cnt = space(r, o["dst_space"])
                dst[o["dst_off"]:o["dst_off"] + o["width"]] = msg
                cnt[o["dst_off"]:o["dst_off"] + o["width"]] += 1
                received[r] += o["width"]

    run_ops(root, plans[root][0])
    for r in range(N):
        if r != root:
            run_ops(r, plans[r][0])
    assert all(not q for q in links.values()), "sends left without a receive"
    return band.reshape(B, A, C * N, T * 4), slices, writes, staging_writes, sent, received


@pytest.mark.parametrize("N", [1, 2, 3, 4])
@pytest.mark.parametrize("root_at", ["first", "last", "middle"])
@pytest.mark.parametrize("chunk", [0, 256, 100, 48], ids=["one-piece", "row-blocks", "ragged-blocks", "row-segments"])
def test_scatter_plan_moves_every_band_byte_once(N, root_at, chunk):
    """the scatter's piece and staging-slot planning and its send/receive pairing, on CPU.  For N = 1..4
    ranks, roots first / middle / last, whole-row pieces, ragged row blocks and rows longer than a piece (sub-row
    segments): every rank's slice equals its channel block [C r, C (r + 1)) of the band, every slice byte and every
    staging byte is written exactly once, and the byte counts match what bf_comm_stats reports."""
    root = {"first": 0, "last": N - 1, "middle": N // 2}[root_at]
    B, A, C, T = 2, 3, 2, 16  # run = 128 bytes, 6 rows
    band, slices, writes, staging_writes, sent, received = _replay_scatter(N, root, B, A, C, T, chunk)
    for r in range(N):
        want = np.ascontiguousarray(band[:, :, C * r:C * (r + 1)]).reshape(-1)
        np.testing.assert_array_equal(slices[r], want, err_msg=f"rank {r}")
        assert (writes[r] == 1).all(), f"rank {r}: slice bytes written {np.unique(writes[r])} times"
        # the root's own slice is one 2-D copy at N > 1 (a self send/receive only at one rank)
        assert received[r] == (0 if (r == root and N > 1) else want.size)
    assert (staging_writes == 1).all()
    assert sent[root] == B * A * C * T * 4 * max(N - 1, 1)
    assert all(sent[r] == 0 for r in range(N) if r != root)


def test_scatter_plan_argument_checks():
    from dpdk_dc_sand_amd.shard import ScatterOp, scatter_plan
    with pytest.raises(_lib.BeamformerError, match="root 2 of 2"):
        scatter_plan(2, 0, 2, 1, 1, 1, 16)
    with pytest.raises(_lib.BeamformerError, match="bad shape"):
        scatter_plan(2, 0, 0, 0, 1, 1, 16)
    n, stg = ctypes.c_size_t(), ctypes.c_size_t()
    ops = (ScatterOp * 1)()
    with pytest.raises(_lib.BeamformerError, match="capacity"):
        _lib.call("bf_scatter_plan", 3, 0, 0, 2, 2, 1, 16, 64, ops, 1, ctypes.byref(n), ctypes.byref(stg))
    assert n.value > 1
    # the product piece: a 2 GiB cfg3 slice (8 x 64 rows of 1 MiB) moves in 8 groups of 256 MiB
    plan, staging = scatter_plan(2, 1, 0, 8, 64, 4096, 256)
    assert len(plan) == 8 and all(o["width"] == 256 << 20 for o in plan) and staging == 0
