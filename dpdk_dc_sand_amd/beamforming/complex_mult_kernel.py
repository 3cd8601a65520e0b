"""Beamformer complex multiplication launcher (drop-in for beamformer/beamforming/complex_mult_kernel.py).

The reference launches the numba kernel `run_complex_mult` with one thread per (row, k) element, each thread
redoing the whole 2M x 2A row (complex_mult_kernel.py:11-100), then blocks on cuda.synchronize() (:162).
Here the same call runs the HIP MFMA kernel `bf_beamform` (dpdk_dc_sand_amd/csrc/bf_beamform.hip) on the
operation's stream, asynchronously (stream-ordered; DeviceArray.get synchronises).
"""
import numpy as np

from .. import _lib


class ComplexMultKernel:
    """Class for beamform complex multiplication (complex_mult_kernel.py:103-162)."""

    def complex_mult(self, data_matrix, coeff_matrix, out):
        """Launch the beamform multiply for `self` (a MatrixMultiply operation).

        data_matrix: DeviceArray 8-bit (B, P, C, NB, 16, A, 2); coeff_matrix: float32 (B, P, C, 2A, 2M);
        out: float32 (B, P, C, NB, 16, 2M).
        """
        B, P, C, NB, S, A, Z = data_matrix.shape
        M2 = coeff_matrix.shape[4]
        if Z != 2 or S != 16 or M2 % 2:
            raise ValueError(f"unexpected data shape {data_matrix.shape} / coeff shape {coeff_matrix.shape}")
        if coeff_matrix.shape != (B, P, C, 2 * A, M2) or out.shape != (B, P, C, NB, S, M2):
            raise ValueError("data, coefficient and output shapes disagree")
        if np.dtype(coeff_matrix.dtype) != np.float32 or np.dtype(out.dtype) != np.float32:
            raise ValueError("coefficients and output must be float32")
        signed = np.dtype(data_matrix.dtype) == np.int8
        queue = self.command_queue
        _lib.call("bf_beamform", data_matrix.ptr, coeff_matrix.ptr, out.ptr, B, P, C, NB, A, M2 // 2, int(signed),
                  queue.handle)
