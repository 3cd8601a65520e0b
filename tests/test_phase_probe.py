"""Host check of the integer path's fast Q14 phasor (bf_phase.hpp q14_fast, restated in
tools/probes/q14_fast_check.c): its error against the exact reference-order phasor stays below the decision
guard, and every coefficient the fast rule decides equals the exact Q14 value."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_q14_fast_rule_is_exact(tmp_path):
    exe = tmp_path / "q14"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "probes", "q14_fast_check.c"), "-lm"],
                   check=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "wrong unflagged 0" in r.stdout


def _run_probe(tmp_path, name, n):
    exe = tmp_path / name
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tools", "probes", name + ".c"), "-lm"], check=True)
    r = subprocess.run([str(exe), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_markstein_division_is_correctly_rounded(tmp_path):
    """bf_phase.hpp div_denom (reciprocal + one Markstein step) == IEEE a / (Ctot*Ts) on steering quotients."""
    assert "0 differ from the IEEE division" in _run_probe(tmp_path, "div_check", 5000000)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_sincos_pio2_float32_roundings_equal_libm(tmp_path):
    """bf_phase.hpp sincos_pio2: the float32 roundings of sin/cos equal libm's (the coefficient contract)."""
    assert "differing from libm: 0," in _run_probe(tmp_path, "sincos_check", 3000000)
