"""C callers of the ABI (the reference's native harness, common/UnitTest.cpp:28-57 and
BeamformerCoefficientTest.cu:278-420).

* tests/c/bf_smoke.c -- simulate -> HtoD -> kernels -> DtoH -> verify against the oracle's fixture
  (tests/golden/c_smoke.bin, from tests/golden/make_c_fixture.py): reorder, coefficients and int8 beams bit-exact,
  f32 beams within the tolerance, the three-pass chain == the fused operator with exact coefficients.
* tests/c/bf_stream_doc.c -- INTEGRATION.md's streaming example, compiled from the markdown block itself.
Both are built by `make` (target cabi) with plain gcc against include/bf.h and the in-tree libbf.so.
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "c_smoke.bin")
BINS = [os.path.join(ROOT, "build", b) for b in ("bf_smoke", "bf_stream_doc")]


def _build():
    r = subprocess.run(["make", "-s", "cabi"], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_c_callers_compile_and_link():
    """Both C programs (and the INTEGRATION.md snippet inside one) compile warning-free and link to libbf.so."""
    for b in BINS + [os.path.join(ROOT, "build", "stream_snippet.inc")]:
        if os.path.exists(b):
            os.remove(b)
    _build()
    assert all(os.path.exists(b) for b in BINS)
    snippet = open(os.path.join(ROOT, "build", "stream_snippet.inc")).read()
    assert "bf_pipeline_submit" in snippet and "bf_pipeline_destroy" in snippet


def test_fixture_matches_oracle():
    """The committed fixture is what make_c_fixture.py writes (regenerated here, byte for byte)."""
    import importlib.util
    import shutil
    import tempfile
    spec = importlib.util.spec_from_file_location("mk", os.path.join(ROOT, "tests", "golden", "make_c_fixture.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    with tempfile.TemporaryDirectory() as d:
        saved = mk.HERE
        mk.HERE = d
        try:
            mk.main()
        finally:
            mk.HERE = saved
        assert open(os.path.join(d, "c_smoke.bin"), "rb").read() == open(FIXTURE, "rb").read()
        shutil.rmtree(d, ignore_errors=True)
    hdr = np.fromfile(FIXTURE, "<i4", count=8)
    assert list(hdr[:7]) == [mk.B, mk.A, mk.C, mk.T, mk.M, mk.Ctot, mk.XENG]


@pytest.mark.gpu
def test_c_smoke_on_gpu():
    if not all(os.path.exists(b) for b in BINS):
        _build()
    r = subprocess.run([BINS[0], FIXTURE], capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bf_smoke OK" in r.stdout
    print(r.stdout.strip())


@pytest.mark.gpu
def test_integration_stream_example_on_gpu():
    if not all(os.path.exists(b) for b in BINS):
        _build()
    r = subprocess.run([BINS[1], FIXTURE, "13"], capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bf_stream_doc OK: 13 frames" in r.stdout
    print(r.stdout.strip())
