"""The stated float tolerance for beamformed outputs.

The reference tests compare with rtol = atol = 1e-4 (beamform_mult_kernel_test.py:267-269).  An absolute 1e-4
is below the fp32 resolution of the dot products' partial sums (|partial| ~ 1e3-1e4 -> ulp 1e-4-1e-3): with
non-uniform delays the reference's own fp32 CPU oracle misses it against the exact product in ~0.02-0.1 % of
outputs (tools/precision_probe.py; tests/test_oracle_golden.py::test_reference_tolerance_is_not_fp32_attainable).
So the contract adds the fp32 dot-product term: two fp32 evaluations of y = sum_k x_k w_k may differ by
2^-20 * sum_k |x_k w_k| (measured: GPU <= 1.5e-7 * sum|xw| vs exact, the CPU oracle <= 3.8e-7).
"""
import numpy as np

import oracle as O

RTOL = 1e-4
ATOL = 1e-4
FP32_DOT = 2.0 ** -20


def fp32_tolerance(desired, x_reordered, w, signed=False):
    """Elementwise bound ATOL + RTOL*|desired| + FP32_DOT * sum_k |x_k w_k| (float64)."""
    desired = np.asarray(desired, np.float64)
    mag = O.dot_magnitude(x_reordered, w, signed=signed).reshape(desired.shape)
    return ATOL + RTOL * np.abs(desired) + FP32_DOT * mag


def assert_beams_allclose(actual, desired, x_reordered, w, signed=False):
    """|actual - desired| <= ATOL + RTOL*|desired| + FP32_DOT * sum_k |x_k w_k|, elementwise."""
    actual = np.asarray(actual, np.float64)
    desired = np.asarray(desired, np.float64)
    assert actual.shape == desired.shape, (actual.shape, desired.shape)
    err = np.abs(actual - desired)
    tol = fp32_tolerance(desired, x_reordered, w, signed)
    bad = err > tol
    if bad.any():
        i = np.unravel_index(np.argmax(err / tol), err.shape)
        raise AssertionError(f"{int(bad.sum())}/{err.size} beams outside the fp32 tolerance; worst at {i}: "
                             f"actual {actual[i]!r} desired {desired[i]!r} |err| {err[i]:.3e} tol {tol[i]:.3e}")
