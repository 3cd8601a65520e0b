"""Which HIP runtime libbf runs on inside the test process.

The product (libbf.so, RUNPATH /opt/rocm-7.2.0/lib) and bench.py run on /opt/rocm's HIP runtime.  If anything maps
torch's bundled libamdhip64 (ROCm 7.0) into a process before libbf is loaded, the dynamic loader reuses it for
libbf's NEEDED `libamdhip64.so.7` and every kernel then runs under the other runtime.  Round 4's GPU suite did exactly
that through one collection-time `torch.cuda.device_count()`; these tests pin that it cannot happen again: the GPU
suite's own process (the `gpu` test, run after collection of the whole suite) and a fresh process (CPU test).
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROCM = os.path.realpath("/opt/rocm")


def _mapped(name, maps_text):
    paths = set()
    for line in maps_text.splitlines():
        parts = line.split(None, 5)
        if len(parts) == 6 and name in os.path.basename(parts[5]):
            paths.add(os.path.realpath(parts[5].strip()))
    return sorted(paths)


def _check_hip_runtime(paths):
    assert len(paths) == 1, f"expected exactly one libamdhip64 mapping, got {paths}"
    assert paths[0].startswith(ROCM + os.sep), f"libamdhip64 mapped from {paths[0]}, not from {ROCM}"
    assert "torch" not in paths[0]


def test_fresh_process_binds_libbf_to_rocm_runtime():
    """Loading libbf alone (no device needed) maps /opt/rocm's libamdhip64 and nothing from torch/lib."""
    code = ("import sys; sys.path.insert(0, %r); from dpdk_dc_sand_amd import _lib; _lib.load(); "
            "print(open('/proc/self/maps').read())") % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    _check_hip_runtime(_mapped("libamdhip64", r.stdout))


@pytest.mark.gpu
def test_hip_runtime_is_the_products():
    """In the GPU suite's own process, after the device is initialised through libbf: the one HIP runtime mapped is
    /opt/rocm's, and torch was never imported (collection included)."""
    sys.path.insert(0, ROOT)
    from dpdk_dc_sand_amd import accel
    assert accel.device_count() >= 1
    ctx = accel.create_some_context(device=0)
    ctx.create_command_queue().finish()
    with open("/proc/self/maps") as f:
        _check_hip_runtime(_mapped("libamdhip64", f.read()))
    assert "torch" not in sys.modules, "torch was imported into the GPU test process"
