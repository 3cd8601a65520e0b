"""GPU box: the one-rank RCCL channel scatter (bf_channel_scatter, self send/recv) at growing sizes, each checked
byte for byte on the host and by the device checksums.  Prints one JSON line per size.
Usage: python tools/diag_scatter.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402
from dpdk_dc_sand_amd.rendezvous import HostGroup  # noqa: E402
from dpdk_dc_sand_amd.shard import ChannelScatter, device_checksum  # noqa: E402


def main():
    ctx = accel.create_some_context(device=0)
    q = ctx.create_command_queue()
    comm = ChannelScatter(HostGroup(0, 1), ctx)
    shapes = [(2, 3, 5, 32), (8, 64, 64, 256), (8, 64, 1024, 256), (8, 64, 2047, 256), (8, 64, 2048, 256),
              (8, 64, 4095, 256), (8, 64, 4096, 256)]
    try:
        for B, A, C, T in shapes:
            band = accel.DeviceArray(ctx, (B, A, C, T, 2, 2), np.int8)
            _lib.call("bf_fill_random", band.ptr, band.nbytes, 5, q.handle)
            out = accel.DeviceArray(ctx, (B, A, C, T, 2, 2), np.int8)
            _lib.call("bf_fill_random", out.ptr, out.nbytes, 9, q.handle)
            comm.scatter(band, out, B, A, C, T, q)
            q.finish()
            h_band, h_out = band.get(q), out.get(q)
            diff = np.flatnonzero(h_band.reshape(-1) != h_out.reshape(-1))
            cs_out = device_checksum(out, out.nbytes, 0, 1, q)
            run = C * T * 4
            cs_band = device_checksum(band, run, run, B * A, q)
            cs_band1 = device_checksum(band, band.nbytes, 0, 1, q)
            ok, rep = comm.verify(band, out, B, A, C, T, q)
            print(json.dumps({"shape": [B, A, C, T], "bytes": band.nbytes, "n_diff": int(diff.size),
                              "first_diff": int(diff[0]) if diff.size else None,
                              "last_diff": int(diff[-1]) if diff.size else None,
                              "cs_out": f"{cs_out:016x}", "cs_band_2d": f"{cs_band:016x}",
                              "cs_band_1d": f"{cs_band1:016x}", "verify": ok, "stats": comm.stats()}), flush=True)
            del band, out, h_band, h_out
    finally:
        comm.close()


if __name__ == "__main__":
    main()
