"""Test configuration.

* `gpu` marker: needs a real MI355X (run with `-m gpu`); everything else runs on CPU.
* `combinations` marker + `--all-combinations`: the reference's parameter-grid plugin
  (beamformer/unit_test/conftest.py:44-101), restated.
* The in-tree libbf.so is (re)built by `make` at session start when sources are newer.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config) -> None:
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "combinations(names, *values): test combinations of values")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_addoption(parser) -> None:
    group = parser.getgroup("combinations")
    group.addoption("--all-combinations", action="store_true", help="Test the full Cartesian product of parameters")


def pytest_generate_tests(metafunc) -> None:
    """`combinations` marker: by default max(len) combos cycling each list, the last one using every list's
    last value; the full product with --all-combinations (reference unit_test/conftest.py:61-101)."""
    all_combinations = metafunc.config.option.all_combinations
    for marker in metafunc.definition.iter_markers("combinations"):
        if isinstance(marker.args[0], (tuple, list)):
            names = list(marker.args[0])
        else:
            names = [n.strip() for n in marker.args[0].split(",") if n.strip()]
        values = marker.args[1:]
        if len(names) != len(values):
            pytest.fail(f"{metafunc.definition.nodeid}: combinations needs one value list per name", pytrace=False)
        if not names:
            continue
        if all_combinations:
            for name, value_list in zip(names, values):
                metafunc.parametrize(name, value_list)
        else:
            n = max(len(v) for v in values)
            combos = []
            for i in range(n):
                if i == n - 1:
                    combos.append(tuple(v[-1] for v in values))
                else:
                    combos.append(tuple(v[i % len(v)] for v in values))
            metafunc.parametrize(names, combos)


def pytest_sessionstart(session) -> None:
    if os.environ.get("BF_SKIP_MAKE"):
        return
    r = subprocess.run(["make", "-s", "-j8"], cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        raise pytest.UsageError("building libbf.so failed:\n" + r.stdout + r.stderr)


@pytest.fixture(scope="session")
def context():
    from dpdk_dc_sand_amd import accel
    return accel.create_some_context(device_filter=lambda x: x.is_cuda, interactive=False)


@pytest.fixture(scope="session")
def command_queue(context):
    return context.create_command_queue()
