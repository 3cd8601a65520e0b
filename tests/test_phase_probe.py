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
