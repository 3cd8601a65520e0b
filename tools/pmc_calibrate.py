"""In-repo calibration of the PMC byte counters the bench's `roofline.traffic` uses (the x2 FETCH_SIZE
factor came from MI355X_MICROARCH.md, not from a measurement here).  A plain streaming kernel of the diagnostic
library reads (or writes) a known byte count; rocprofv3 collects FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ per
dispatch in separate passes, and this prints counter x unit / known bytes.

    python tools/pmc_calibrate.py [outdir]           (parent: no GPU use; each pass is a rocprofv3 child)
    python tools/pmc_calibrate.py --child MODE N      (child: N launches of the stream kernel, MODE read|write|mix)
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NBYTES = 1 << 30  # 1 GiB: far beyond L2 and the 256 MB Infinity Cache


def child(mode, n):
    sys.path.insert(0, ROOT)
    import ctypes
    import numpy as np
    from dpdk_dc_sand_amd import _lib, accel
    lib = _lib.load(os.path.join(ROOT, "build", "libbf_diag.so"))
    V, S, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.bf_diag_stream.argtypes = [V, V, S, S, I, I, V]
    ctx = accel.create_some_context()
    q = ctx.create_command_queue()
    a = accel.DeviceArray(ctx, (NBYTES,), np.uint8)
    b = accel.DeviceArray(ctx, (NBYTES,), np.uint8)
    ri, wo = {"read": (NBYTES, 0), "write": (0, NBYTES), "mix": (NBYTES, NBYTES // 4)}[mode]
    for _ in range(n):  # unroll 102: non-temporal 16-B loads, plain 16-B stores (the bench's ceiling kernel shape)
        assert lib.bf_diag_stream(a.ptr, b.ptr, ri, wo, 2048, 102, q.handle) == 0
    q.finish()


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_cal")
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    rows = []
    for mode, counters in (("read", "FETCH_SIZE"), ("read", "TCC_EA0_RDREQ TCC_EA0_RDREQ_128B"), ("write", "WRITE_SIZE"),
                           ("mix", "FETCH_SIZE"), ("mix", "WRITE_SIZE")):
        d = os.path.join(out, f"{mode}_{counters.split()[0]}")
        cmd = ["timeout", "-s", "KILL", "120", "/opt/rocm/bin/rocprofv3", "--pmc", *counters.split(), "--output-format", "csv",
               "-d", d, "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--child", mode, "5"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if r.returncode != 0 or not files:
            print(f"{mode} {counters}: failed rc={r.returncode} {r.stderr[-300:]}")
            continue
        vals = {}
        with open(files[0]) as f:
            for row in csv.DictReader(f):
                if "stream_kernel" in row.get("Kernel_Name", ""):
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        for name, v in vals.items():
            v.sort()
            med = v[len(v) // 2]
            # FETCH_SIZE / WRITE_SIZE are in KiB; TCC_EA0_RDREQ counts requests (x 64 B, as FETCH_SIZE tallies them),
            # TCC_EA0_RDREQ_128B the 128-byte ones (x 128 B)
            got = med * 1024 if name in ("FETCH_SIZE", "WRITE_SIZE") else med * (128 if name.endswith("128B") else 64)
            known = {"read": {"r": NBYTES, "w": 0}, "write": {"r": 0, "w": NBYTES},
                     "mix": {"r": NBYTES, "w": NBYTES // 4}}[mode]["w" if name == "WRITE_SIZE" else "r"]
            rows.append({"kernel_bytes": mode, "counter": name, "median_per_dispatch": med, "bytes_from_counter": got,
                         "known_bytes": known, "ratio": round(got / known, 4) if known else None})
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
    else:
        main()
