"""Beamformer steering-coefficient generation (drop-in for beamformer/beamforming/coeff_generator.py).

Same template/operation names, constructor signature and slots as the reference
(coeff_generator.py:106-207); `_run` launches the HIP kernel `bf_coeff_gen` instead of the numba kernel
`run_coeff_gen` (:12-103).  The phase is evaluated in float64 in the reference's operation order, so the
output is bit-exact to the CPU oracle (unit_test/coeff_generator_cpu.py:78-187), including its
delay_vals[c][m][a] -> (antenna a, beam m) mapping (the numba kernel transposes it).
"""
import numpy as np

from .. import _lib, accel


class CoeffGeneratorTemplate:
    """Template for the beamform coefficient generator (coeff_generator.py:106-181).

    Parameters are the reference's: context, n_batches, n_pols, n_channels_per_stream, n_channels (whole band),
    n_blocks, n_samples_per_block, n_ants, n_beams, xeng_id (selects the absolute channel offset
    n_channels_per_stream * xeng_id), sample_period (ADC period, seconds).
    """

    def __init__(self, context, n_batches: int, n_pols: int, n_channels_per_stream: int, n_channels: int,
                 n_blocks: int, n_samples_per_block: int, n_ants: int, n_beams: int, xeng_id: int,
                 sample_period: float) -> None:
        for name, v in dict(n_batches=n_batches, n_pols=n_pols, n_channels_per_stream=n_channels_per_stream,
                            n_channels=n_channels, n_ants=n_ants, n_beams=n_beams).items():
            if int(v) <= 0:
                raise ValueError(f"{name} must be positive, got {v}")
        if int(xeng_id) < 0:
            raise ValueError(f"xeng_id must be >= 0, got {xeng_id}")
        if not sample_period > 0:
            raise ValueError(f"sample_period must be > 0, got {sample_period}")
        self.context = context
        self.n_batches = n_batches
        self.n_pols = n_pols
        self.n_channels_per_stream = n_channels_per_stream
        self.n_channels = n_channels
        self.n_blocks = n_blocks
        self.n_samples_per_block = n_samples_per_block
        self.n_ants = n_ants
        self.n_beams = n_beams
        self.xeng_id = xeng_id
        self.sample_period = sample_period

        self.delay_vals_data_dimensions = (
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_beams, exact=True),
            accel.Dimension(self.n_ants, exact=True),
            accel.Dimension(4, exact=True),
        )
        self.coeff_data_dimensions = (
            accel.Dimension(self.n_batches, exact=True),
            accel.Dimension(self.n_pols, exact=True),
            accel.Dimension(self.n_channels_per_stream, exact=True),
            accel.Dimension(self.n_ants * 2, exact=True),
            accel.Dimension(self.n_beams * 2, exact=True),
        )

    def instantiate(self, command_queue):
        """Initialise the coefficient generation class."""
        return CoeffGenerator(self, command_queue)


class CoeffGenerator(accel.Operation):
    """Beamform coefficient generation (coeff_generator.py:184-250).

    .. rubric:: Slots
    delay_vals: (n_channels_per_stream, n_beams, n_ants, 4), float32 -- (delay_s, delay_rate, phase_rad,
        phase_rate); only [0] and [2] are used, as in the reference.
    outCoeffs: (n_batches, n_pols, n_channels_per_stream, 2*n_ants, 2*n_beams), float32 -- per (a, m) the
        real 2x2 block [[cos, sin], [-sin, cos]], replicated over batches and pols.
    """

    def __init__(self, template: CoeffGeneratorTemplate, command_queue):
        super().__init__(command_queue)
        self.template = template
        self.slots["delay_vals"] = accel.IOSlot(dimensions=self.template.delay_vals_data_dimensions,
                                                dtype=np.float32)
        self.slots["outCoeffs"] = accel.IOSlot(dimensions=self.template.coeff_data_dimensions, dtype=np.float32)

    def _run(self):
        t = self.template
        _lib.call("bf_coeff_gen", self.buffer("delay_vals").ptr, self.buffer("outCoeffs").ptr, t.n_batches,
                  t.n_pols, t.n_channels_per_stream, t.n_channels, t.n_ants, t.n_beams, t.xeng_id,
                  float(t.sample_period), self.command_queue.handle)
