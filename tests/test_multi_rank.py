"""Multi-rank (X-engine) logic on CPU: world_size-2 gloo process groups.

Checks the channel-shard arithmetic, the root -> ranks channel scatter / gather helpers, that beamforming each
shard with xeng_id = rank reproduces the full-band result exactly (the reference's absolute-channel convention,
coeff_generator.py:49-53), and bench.py's gloo timing bracket (barrier + max over ranks)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

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


def _worker(rank, world, port, result_q):
    import torch.distributed as dist

    import oracle as O
    from dpdk_dc_sand_amd.shard import gather_channel_slices, scatter_channel_slices

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, A, M, T, Ctot = 2, 5, 3, 32, 8
        C = Ctot // world
        raw = O.u8_voltages((B, A, Ctot, T, 2, 2), seed=11) if rank == 0 else None
        d = np.zeros((1, M, A, 4), np.float32)
        rng = np.random.default_rng(3)
        d[..., 0] = rng.uniform(0, 10 * O.TS_MEERKAT, (1, M, A))
        d[..., 2] = rng.uniform(-np.pi, np.pi, (1, M, A))
        mine = scatter_channel_slices(raw, (B, A, C, T, 2, 2), np.uint8, rank, world)
        beams = O.fused_beamform(mine, d, Ctot, xeng_id=rank)  # this X-engine's channels
        full = gather_channel_slices(beams, rank, world)

        # bench.py's timing bracket: barrier + max over ranks
        from bench import Dist
        os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank))
        dd = Dist.__new__(Dist)
        dd.world, dd.rank, dd.local_rank, dd.dist = world, rank, rank, dist
        dd.barrier()
        mx = dd.max(float(rank + 1))
        if rank == 0:
            ref = O.fused_beamform(raw, d, Ctot, xeng_id=0)
            result_q.put(("ok", bool(np.array_equal(full, ref)), mx))
    except Exception as e:  # pragma: no cover - reported to the parent
        result_q.put(("error", repr(e), None))
    finally:
        dist.destroy_process_group()


def test_channel_sharded_beamforming_matches_full_band_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, equal, mx = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert status == "ok", equal
    assert equal, "sharded beams differ from the full-band result"
    assert mx == float(world)
