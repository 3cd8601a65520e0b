"""Drop-in for the reference package `beamformer/beamforming` (magnate3/dpdk_dc_sand), on HIP/gfx950.

Reference module -> here:
    beamforming.prebeamform_reorder   -> PreBeamformReorderTemplate / PreBeamformReorder
    beamforming.coeff_generator       -> CoeffGeneratorTemplate / CoeffGenerator
    beamforming.matrix_multiply       -> MatrixMultiplyTemplate / MatrixMultiply
    beamforming.complex_mult_kernel   -> ComplexMultKernel
    beamforming.beamform_op_sequence  -> OpSequenceTemplate / OpSequence
New (MI355X-native): beamforming.fused -> FusedBeamformerTemplate / FusedBeamformer (one-pass reorder +
coefficient regeneration + multiply, optional ?beam-weights gains), beamforming.requant -> RequantTemplate /
Requant, beamforming.streaming -> StreamingBeamformerTemplate / StreamingBeamformer (host -> GPU -> host frames
with H2D, compute and D2H overlapped).
The CPU reference helpers the reference tests import (beamforming/reorder.py, unit_test/*_cpu.py) live in the
repository's `oracle/` package, which the product path never imports.
"""
from .beamform_op_sequence import OpSequence, OpSequenceTemplate  # noqa: F401
from .coeff_generator import CoeffGenerator, CoeffGeneratorTemplate  # noqa: F401
from .complex_mult_kernel import ComplexMultKernel  # noqa: F401
from .fused import FusedBeamformer, FusedBeamformerTemplate  # noqa: F401
from .matrix_multiply import MatrixMultiply, MatrixMultiplyTemplate  # noqa: F401
from .prebeamform_reorder import PreBeamformReorder, PreBeamformReorderTemplate  # noqa: F401
from .requant import Requant, RequantTemplate  # noqa: F401
from .streaming import StreamingBeamformer, StreamingBeamformerTemplate  # noqa: F401
