"""Reorder -> coefficient generation -> multiply (drop-in for beamformer/beamforming/beamform_op_sequence.py).

Same template/sequence names, constructor signature, sub-operation attributes and compound slot names as the
reference (beamform_op_sequence.py:16-157).  For the one-pass MI355X path (no reorder round trip through HBM,
coefficients regenerated in-kernel) see `fused.FusedBeamformerTemplate`.
"""
from .. import accel
from .coeff_generator import CoeffGeneratorTemplate
from .matrix_multiply import MatrixMultiplyTemplate
from .prebeamform_reorder import PreBeamformReorderTemplate


class OpSequenceTemplate:
    """Template linking pre-beamform reorder, coefficient generation and beamform multiply
    (beamform_op_sequence.py:16-114).

    Input  [n_batches][antennas][n_channels][samples_per_channel][polarisations][complexity]
    Output [n_batches][polarisations][n_channels][n_blocks][samples_per_block][2*n_beams]
    """

    def __init__(self, context, n_batches, n_pols, n_channels_per_stream, n_channels, n_blocks, n_samples_per_block,
                 n_ants, n_beams, xeng_id, sample_period, n_samples_per_channel) -> None:
        self.preBeamformReorder_template = PreBeamformReorderTemplate(
            context, n_ants, n_channels_per_stream, n_samples_per_channel, n_batches)
        self.beamform_coeff_template = CoeffGeneratorTemplate(
            context, n_batches, n_pols, n_channels_per_stream, n_channels, n_blocks, n_samples_per_block, n_ants,
            n_beams, xeng_id, sample_period)
        self.beamform_mult_template = MatrixMultiplyTemplate(
            context=context, n_ants=n_ants, n_channels_per_stream=n_channels_per_stream,
            n_samples_per_channel=n_samples_per_channel, n_beams=n_beams, n_batches=n_batches)

    def instantiate(self, queue):
        """Instantiate and return OpSequence object."""
        return OpSequence(self, queue)


class OpSequence(accel.OperationSequence):
    """1. pre-beamform reorder, 2. beamform coefficient generator, 3. beamforming
    (beamform_op_sequence.py:117-157)."""

    def __init__(self, template, queue):
        self.prebeamform_reorder = template.preBeamformReorder_template.instantiate(queue)
        self.beamform_coeff = template.beamform_coeff_template.instantiate(queue)
        self.beamform_mult = template.beamform_mult_template.instantiate(queue)
        operations = [
            ("prebeamform_reorder", self.prebeamform_reorder),
            ("beamform_coeff", self.beamform_coeff),
            ("beamform_mult", self.beamform_mult),
        ]
        compounds = {
            "bufin_delay_vals": ["beamform_coeff:delay_vals"],
            "bufint_coeff": ["beamform_coeff:outCoeffs", "beamform_mult:inCoeffs"],
            "bufin_reorder": ["prebeamform_reorder:inSamples"],
            "bufint_data": ["prebeamform_reorder:outReordered", "beamform_mult:inData"],
            "bufout_mult": ["beamform_mult:outData"],
        }
        super().__init__(queue, operations, compounds)
        self.template = template
