"""8-bit requantiser for beamformed output (no reference counterpart; SURVEY §7 build step 7).

Contract (oracle.requantise): q = clamp(round_half_even(y * scale), -127, 127) as int8, elementwise on the
float32 beams -- bit-exact given the same float32 input.
"""
import numpy as np

from .. import _lib, accel


class RequantTemplate:
    def __init__(self, context, shape, scale: float = 1.0):
        self.context = context
        self.shape = tuple(int(s) for s in shape)
        self.scale = float(scale)

    def instantiate(self, command_queue):
        return Requant(self, command_queue)


class Requant(accel.Operation):
    """.. rubric:: Slots
    inData: float32 `shape`;  outData: int8 `shape`
    """

    def __init__(self, template: RequantTemplate, command_queue):
        super().__init__(command_queue)
        self.template = template
        self.slots["inData"] = accel.IOSlot(template.shape, np.float32)
        self.slots["outData"] = accel.IOSlot(template.shape, np.int8)

    def _run(self):
        n = int(np.prod(self.template.shape, dtype=np.int64))
        _lib.call("bf_requant", self.buffer("inData").ptr, self.buffer("outData").ptr, n, self.template.scale,
                  self.command_queue.handle)
