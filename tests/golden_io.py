"""Access to tests/golden/golden.npz (made by tests/golden/make_golden.py from the reference's CPU oracles)."""
import hashlib
import os

import numpy as np

from oracle import u8_voltages

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")
_G = None


def golden():
    global _G
    if _G is None:
        _G = np.load(PATH, allow_pickle=False)
    return _G


def cases(prefix):
    return sorted({k.split("/")[0] for k in golden().files if k.startswith(prefix)})


def get(case, key):
    return golden()[f"{case}/{key}"]


def sha256(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def voltages(case, shape):
    """Regenerate a golden case's u8 voltages (default_rng(2021)) and check them against the stored digest."""
    x = u8_voltages(shape)
    assert sha256(x) == str(get(case, "input_sha256")), f"{case}: regenerated input differs from the golden's"
    return x
