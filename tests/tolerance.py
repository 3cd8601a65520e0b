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
from oracle.beamform_oracle import _as_real

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


def assert_reference_bar(actual, desired, x_reordered, w, signed=False, max_fraction=1e-5):
    """The reference's own assertion, np.testing.assert_allclose(cpu, gpu, rtol=1e-4, atol=1e-4)
    (beamform_mult_kernel_test.py:267-269, beamform_op_sequence_test.py:198-199), against its float32 CPU result.

    That CPU result is itself rounded at the scale of its partial sums (|partial| ~ 1e3 -> ulp ~ 1e-4), so an output
    that cancels to near zero can sit 1e-4 from the exact value on the CPU side alone.  Every element that misses the
    bar must therefore (a) meet the same bar against the exact (float64) product, or (b) be no farther from the exact
    product than the reference's float32 result is, or (c) lie within the float32 dot-product rounding bound
    2^-20 * sum_k |x_k w_k| of the exact product (the same accumulation-order term as assert_beams_allclose: an fp32
    sum whose partials reach ~1e3 can land 1e-4 from a near-zero exact result in either implementation); and such
    elements must be rare (<= max_fraction).
    Returns the number of elements that missed the plain bar (reported by the caller)."""
    a = np.asarray(actual, np.float64)
    d = np.asarray(desired, np.float64)
    assert a.shape == d.shape, (a.shape, d.shape)
    miss = np.abs(a - d) > ATOL + RTOL * np.abs(d)
    n = int(miss.sum())
    if not n:
        return 0
    assert n <= max(1, max_fraction * a.size), f"{n}/{a.size} beams miss the reference's rtol=atol=1e-4 bar"
    # exact products of the missing elements only: a = (B, P, C, NB, 16, 2M) <-> x (B, P, C, NB, 16, A, 2), w (B,P,C,2A,2M)
    B, P, C, NB, S, A, Z = x_reordered.shape
    X = _as_real(x_reordered, signed).reshape(B, P, C, NB * S, 2 * A).astype(np.float64)
    W = np.asarray(w, np.float64)
    for idx in zip(*np.nonzero(miss.reshape(B, P, C, NB * S, -1))):
        b, p, c, t, col = (int(v) for v in idx)
        exact = float(np.dot(X[b, p, c, t], W[b, p, c, :, col]))
        mag = float(np.dot(np.abs(X[b, p, c, t]), np.abs(W[b, p, c, :, col])))
        got = float(a.reshape(B, P, C, NB * S, -1)[b, p, c, t, col])
        ref = float(d.reshape(B, P, C, NB * S, -1)[b, p, c, t, col])
        err = abs(got - exact)
        ok = err <= ATOL + RTOL * abs(exact) or err <= abs(ref - exact) or err <= 2.0 ** -20 * mag
        assert ok, (f"beam {idx}: gpu {got!r}, reference f32 {ref!r}, exact {exact!r}, sum|x w| {mag!r}: the GPU "
                    "misses the bar against the exact product, is farther from it than the reference's own float32 "
                    "result and outside the fp32 dot-product rounding bound")
    return n
