"""Pre-beamform reorder (drop-in for beamformer/beamforming/prebeamform_reorder.py).

Same template/operation names, constructor signature, attributes and slots (prebeamform_reorder.py:15-186).
The reference compiles a mako CUDA kernel per shape through katsdpsigproc/PyCUDA (:107-119); here one
precompiled HIP kernel (`bf_reorder`, LDS-tiled, 16-byte coalesced in and out) serves every shape.
"""
import numpy as np

from .. import _lib, accel


class PreBeamformReorderTemplate:
    """Template for the pre-beamform reorder (prebeamform_reorder.py:15-125).

    Input  [n_batches][n_ants][n_channels_per_stream][n_samples_per_channel][n_pols][complexity], 8-bit
    Output [n_batches][n_pols][n_channels_per_stream][n_blocks][n_samples_per_block][n_ants][complexity]
    Raises ValueError unless n_samples_per_channel is a multiple of 16 (the reference's check at :62-65 is
    meant to enforce this but does not).
    """

    def __init__(self, context, n_ants: int, n_channels_per_stream: int, n_samples_per_channel: int,
                 n_batches: int) -> None:
        for name, v in dict(n_ants=n_ants, n_channels_per_stream=n_channels_per_stream,
                            n_samples_per_channel=n_samples_per_channel, n_batches=n_batches).items():
            if int(v) <= 0:
                raise ValueError(f"{name} must be positive, got {v}")
        self.context = context
        self.n_ants = n_ants
        self.n_channels_per_stream = n_channels_per_stream
        self.n_samples_per_channel = n_samples_per_channel
        self.n_pols = 2  # Hardcoded to 2. No other values are supported (reference :53)
        self.n_batches = n_batches
        self._sample_bitwidth = 8
        self.complexity = 2
        self.n_samples_per_block = 128 // self._sample_bitwidth
        if self.n_samples_per_channel % self.n_samples_per_block != 0:
            raise ValueError(f"samples_per_channel must be divisible by {self.n_samples_per_block}.")
        self.n_blocks = self.n_samples_per_channel // self.n_samples_per_block

        self.inputDataShape = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_ants, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_samples_per_channel, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.complexity, exact=True),
        )
        self.outputDataShape = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_blocks, exact=True),
            accel.Dimension(self.n_samples_per_block, exact=True),
            accel.Dimension(self.n_ants, exact=True),
            accel.Dimension(self.complexity, exact=True),
        )
        self.matrix_size = self.n_ants * self.n_channels_per_stream * self.n_samples_per_channel * self.n_pols

    def instantiate(self, command_queue) -> "PreBeamformReorder":
        """Create a PreBeamformReorder object using this template."""
        return PreBeamformReorder(self, command_queue)


class PreBeamformReorder(accel.Operation):
    """Pre-beamform reorder operation (prebeamform_reorder.py:128-186).

    .. rubric:: Slots
    inSamples: (n_batches, n_ants, n_channels_per_stream, n_samples_per_channel, n_pols, complexity), uint8
    outReordered: (n_batches, n_pols, n_channels_per_stream, n_blocks, n_samples_per_block, n_ants, complexity),
        uint8
    """

    def __init__(self, template: PreBeamformReorderTemplate, command_queue) -> None:
        super().__init__(command_queue)
        self.template = template
        self.slots["inSamples"] = accel.IOSlot(dimensions=self.template.inputDataShape, dtype=np.uint8)
        self.slots["outReordered"] = accel.IOSlot(dimensions=self.template.outputDataShape, dtype=np.uint8)

    def _run(self) -> None:
        t = self.template
        _lib.call("bf_reorder", self.buffer("inSamples").ptr, self.buffer("outReordered").ptr, t.n_batches,
                  t.n_ants, t.n_channels_per_stream, t.n_samples_per_channel, self.command_queue.handle)
