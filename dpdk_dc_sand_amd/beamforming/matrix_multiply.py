"""Beamformer multiplication (drop-in for beamformer/beamforming/matrix_multiply.py).

Same template/operation names, constructor signature and slots (matrix_multiply.py:16-163).  `_run` goes
through ComplexMultKernel.complex_mult -> the HIP MFMA kernel `bf_beamform` (see complex_mult_kernel.py).
"""
import numpy as np

from .. import accel
from .complex_mult_kernel import ComplexMultKernel


class MatrixMultiplyTemplate:
    """Template for beamform multiplication (matrix_multiply.py:16-115).

    Input  [batch][pol][n_channels_per_stream][n_blocks][n_samples_per_block][n_ants][complexity], 8-bit
    Output [batch][pol][n_channels_per_stream][n_blocks][n_samples_per_block][2*n_beams], float32
    Coeffs [batch][pol][n_channels_per_stream][2*n_ants][2*n_beams], float32

    `sample_signed` (MI355X extension, default False = the reference's uint8 slot): read voltages as int8.
    """

    def __init__(self, context, n_ants: int, n_channels_per_stream: int, n_samples_per_channel: int, n_beams: int,
                 n_batches: int, sample_signed: bool = False) -> None:
        for name, v in dict(n_ants=n_ants, n_channels_per_stream=n_channels_per_stream,
                            n_samples_per_channel=n_samples_per_channel, n_beams=n_beams,
                            n_batches=n_batches).items():
            if int(v) <= 0:
                raise ValueError(f"{name} must be positive, got {v}")
        self.context = context
        self.n_ants = n_ants
        self.n_channels_per_stream = n_channels_per_stream
        self.n_samples_per_channel = n_samples_per_channel
        self.n_batches = n_batches
        self._sample_bitwidth = 8
        self.n_pols = 2  # Hardcoded to 2 in the reference (matrix_multiply.py:70)
        self.complexity = 2
        self.beams = n_beams
        self.sample_signed = bool(sample_signed)
        self.n_samples_per_block = 128 // self._sample_bitwidth  # 16 (matrix_multiply.py:76)
        if self.n_samples_per_channel % self.n_samples_per_block != 0:
            raise ValueError(f"n_samples_per_channel must be a multiple of {self.n_samples_per_block}")
        self.n_blocks = self.n_samples_per_channel // self.n_samples_per_block
        self.length = self.n_batches * self.n_pols * self.n_channels_per_stream * self.n_blocks * \
            self.n_samples_per_block

        self.input_data_dimensions = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_blocks, exact=True),
            accel.Dimension(self.n_samples_per_block, exact=True),
            accel.Dimension(self.n_ants, exact=True),
            accel.Dimension(self.complexity, exact=True),
        )
        self.output_data_dimensions = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_blocks, exact=True),
            accel.Dimension(self.n_samples_per_block, exact=True),
            accel.Dimension(self.beams * self.complexity, exact=True),
        )
        self.coeff_data_dimensions = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_ants * 2, exact=True),
            accel.Dimension(self.beams * 2, exact=True),
        )

    def instantiate(self, command_queue):
        """Initialise the complex multiplication class."""
        return MatrixMultiply(self, command_queue)


class MatrixMultiply(accel.Operation):
    """Beamform complex multiplication (matrix_multiply.py:118-163).

    .. rubric:: Slots
    inData: (batches, n_pols, n_channels_per_stream, n_blocks, n_samples_per_block, n_ants, complexity), uint8
        (int8 with sample_signed)
    outData: (batches, n_pols, n_channels_per_stream, n_blocks, n_samples_per_block, 2*n_beams), float32
    inCoeffs: (batches, n_pols, n_channels_per_stream, 2*n_ants, 2*n_beams), float32
    """

    def __init__(self, template: MatrixMultiplyTemplate, command_queue):
        super().__init__(command_queue)
        self.template = template
        self.slots["inData"] = accel.IOSlot(dimensions=self.template.input_data_dimensions,
                                            dtype=np.int8 if template.sample_signed else np.uint8)
        self.slots["outData"] = accel.IOSlot(dimensions=self.template.output_data_dimensions, dtype=np.float32)
        self.slots["inCoeffs"] = accel.IOSlot(dimensions=self.template.coeff_data_dimensions, dtype=np.float32)

    def _run(self):
        """Run the beamform computation."""
        ComplexMultKernel.complex_mult(self, self.buffer("inData").buffer, self.buffer("inCoeffs").buffer,
                                       self.buffer("outData").buffer)
