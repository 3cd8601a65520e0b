"""Frequency-channel sharding across X-engines (one process per GPU).

The reference's only parallel axis is the X-engine index: engine `xeng_id` owns `n_channels_per_stream` channels
whose absolute index is `c + n_channels_per_stream * xeng_id` (coeff_generator.py:49-53,
coeff_generator_cpu.py:134-141).  Here rank r of a world of N is X-engine r.  Beamforming itself needs no collective;
the only data movement is the optional root -> ranks channel scatter of a full-band voltage cube, done
with `torch.distributed` (gloo on CPU, nccl = RCCL over xGMI on GPUs) and kept out of the timed hot path.
"""
import numpy as np


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
    contiguous message."""
    raw = np.asarray(raw)
    Ctot = raw.shape[2]
    return [np.ascontiguousarray(raw[:, :, s:s + n]) for _, s, n in shard_channels(Ctot, world_size)]


def scatter_channel_slices(raw, shape, dtype, rank, world_size, group=None, device=None):
    """Root (rank 0) scatters the packed channel slices of `raw` (B, A, Ctot, T, 2, 2); every rank returns its
    (B, A, Ctot / N, T, 2, 2) slice as a numpy array (CPU / gloo) or a torch tensor on `device` (nccl).

    `shape` is the per-rank slice shape (all ranks must know it); `raw` is only read on rank 0."""
    import torch
    import torch.distributed as dist

    tdtype = torch.from_numpy(np.zeros(1, dtype)).dtype
    out = torch.empty(shape, dtype=tdtype, device=device)
    if rank == 0:
        parts = [torch.from_numpy(p).to(device) if device is not None else torch.from_numpy(p)
                 for p in pack_channel_slices(raw, world_size)]
        dist.scatter(out, scatter_list=parts, src=0, group=group)
    else:
        dist.scatter(out, src=0, group=group)
    return out if device is not None else out.numpy()


def gather_channel_slices(part, rank, world_size, group=None):
    """Inverse of scatter for beams (B, 2, C, T/16, 16, 2M) (verification only): rank 0 returns the full band."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(np.ascontiguousarray(part))
    if rank == 0:
        parts = [torch.empty_like(t) for _ in range(world_size)]
        dist.gather(t, gather_list=parts, dst=0, group=group)
        return np.concatenate([p.numpy() for p in parts], axis=2)
    dist.gather(t, dst=0, group=group)
    return None
