"""GPU box: the one-rank RCCL channel scatter (bf_channel_scatter, self send/recv) at growing sizes, each checked
byte for byte on the host and by the device checksums.  Prints one JSON line per size.

--attribute (diagnostic library build/libbf_diag.so): which stage of the unchunked scatter lost the second GiB in
round 4 (profiles/r4_sc_scatter_unchunked.txt) -- at the 2 GiB slice, each stage alone, checksummed on the device:
  pack   : one hipMemcpy2DAsync of the whole slice (bf_diag_memcpy2d, the scatter's pack) into a staging block;
  p2p    : one self ncclSend/ncclRecv group of the whole 2 GiB (bf_diag_p2p_self) from the band into the slice;
  scatter: bf_channel_scatter with the piece size raised above the slice (bf_diag_scatter_chunk), and at the
           product's 256 MiB pieces.
Usage: python tools/diag_scatter.py [--attribute]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpdk_dc_sand_amd import _lib, accel  # noqa: E402
from dpdk_dc_sand_amd.rendezvous import HostGroup  # noqa: E402
from dpdk_dc_sand_amd.shard import ChannelScatter, device_checksum  # noqa: E402


def attribute():
    import ctypes
    lib = _lib.load(os.path.join(os.path.dirname(_lib.LIB_PATH), "..", "build", "libbf_diag.so"))
    V, S = ctypes.c_void_p, ctypes.c_size_t
    lib.bf_diag_scatter_chunk.argtypes = [S]
    lib.bf_diag_memcpy2d.argtypes = [V, S, V, S, S, S, V]
    lib.bf_diag_p2p_self.argtypes = [V, V, V, S, V]
    # route every libbf call of this process (accel, shard) through the diagnostic library
    _lib._lib = lib
    ctx = accel.create_some_context(device=0)
    q = ctx.create_command_queue()
    comm = ChannelScatter(HostGroup(0, 1), ctx)
    try:
        for B, A, C, T in [(8, 64, 2048, 256), (8, 64, 4095, 256), (8, 64, 4096, 256)]:
            run, rows = C * T * 4, B * A
            nbytes = run * rows
            band = accel.DeviceArray(ctx, (nbytes,), np.uint8)
            _lib.call("bf_fill_random", band.ptr, nbytes, 5, q.handle)
            want = device_checksum(band, nbytes, 0, 1, q)
            out = accel.DeviceArray(ctx, (nbytes,), np.uint8)

            def check(stage, fn):
                _lib.call("bf_fill_random", out.ptr, nbytes, 9, q.handle)
                fn()
                q.finish()
                got = device_checksum(out, nbytes, 0, 1, q)
                bad = None
                if got != want:  # first bad row, from per-row checksums (no 2 GiB host copy)
                    for r in range(rows):
                        if device_checksum(out.ptr + r * run, run, run, 1, q) != device_checksum(band.ptr + r * run,
                                                                                             run, run, 1, q):
                            bad = r
                            break
                print(json.dumps({"shape": [B, A, C, T], "bytes": nbytes, "stage": stage, "ok": got == want,
                                  "first_bad_row": bad, "first_bad_byte": None if bad is None else bad * run}),
                      flush=True)

            check("pack: one hipMemcpy2DAsync of the slice",
                  lambda: _lib.call("bf_diag_memcpy2d", out.ptr, run, band.ptr, run, run, rows, q.handle))
            check("p2p: one self ncclSend/ncclRecv group of the slice",
                  lambda: _lib.call("bf_diag_p2p_self", comm.handle, band.ptr, out.ptr, nbytes, q.handle))
            _lib.call("bf_diag_scatter_chunk", 8 << 30)
            check("scatter, unchunked (pack + self send/recv, one group)",
                  lambda: comm.scatter(band, out, B, A, C, T, q))
            _lib.call("bf_diag_scatter_chunk", 0)
            check("scatter, 256 MiB pieces (the product)", lambda: comm.scatter(band, out, B, A, C, T, q))
            del band, out
    finally:
        comm.close()


def main():
    if "--attribute" in sys.argv:
        return attribute()
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
