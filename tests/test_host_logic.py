"""Host-side logic that needs no GPU: template shapes/attributes mirror the reference, ValueError behaviour,
accel slot binding and the OpSequence compound-slot aliasing (beamform_op_sequence.py:148-156)."""
import os

import numpy as np
import pytest

from dpdk_dc_sand_amd import accel
from dpdk_dc_sand_amd.beamforming import (CoeffGeneratorTemplate, FusedBeamformerTemplate, MatrixMultiplyTemplate,
                                          OpSequenceTemplate, PreBeamformReorderTemplate)

TS = 1 / 1712e6
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeQueue:
    """Stands in for a CommandQueue: the operators only touch it when they run."""
    context = None
    handle = None


class FakeBuf:
    def __init__(self, shape, dtype):
        self.shape, self.dtype = tuple(shape), np.dtype(dtype)


def dims(d):
    return tuple(x.size for x in d)


def test_reorder_template_shapes_and_errors():
    t = PreBeamformReorderTemplate(None, n_ants=5, n_channels_per_stream=51, n_samples_per_channel=256, n_batches=3)
    assert (t.n_pols, t.n_samples_per_block, t.n_blocks) == (2, 16, 16)
    assert dims(t.inputDataShape) == (3, 5, 51, 256, 2, 2)
    assert dims(t.outputDataShape) == (3, 2, 51, 16, 16, 5, 2)
    assert t.matrix_size == 5 * 51 * 256 * 2
    with pytest.raises(ValueError):
        PreBeamformReorderTemplate(None, 4, 4, 100, 1)  # T not a multiple of 16
    with pytest.raises(ValueError):
        PreBeamformReorderTemplate(None, 0, 4, 256, 1)


def test_coeff_template_shapes():
    t = CoeffGeneratorTemplate(None, 3, 2, 16, 4096, 16, 16, 64, 2, 0, TS)
    assert dims(t.delay_vals_data_dimensions) == (16, 2, 64, 4)
    assert dims(t.coeff_data_dimensions) == (3, 2, 16, 128, 4)
    with pytest.raises(ValueError):
        CoeffGeneratorTemplate(None, 3, 2, 16, 4096, 16, 16, 64, 2, -1, TS)
    with pytest.raises(ValueError):
        CoeffGeneratorTemplate(None, 3, 2, 16, 4096, 16, 16, 64, 2, 0, 0.0)


def test_matrix_multiply_template_shapes():
    t = MatrixMultiplyTemplate(None, n_ants=19, n_channels_per_stream=13, n_samples_per_channel=256, n_beams=2,
                               n_batches=3)
    assert (t.n_pols, t.complexity, t.n_samples_per_block, t.n_blocks) == (2, 2, 16, 16)
    assert dims(t.input_data_dimensions) == (3, 2, 13, 16, 16, 19, 2)
    assert dims(t.output_data_dimensions) == (3, 2, 13, 16, 16, 4)
    assert dims(t.coeff_data_dimensions) == (3, 2, 13, 38, 4)
    op = t.instantiate(FakeQueue())
    assert op.slots["inData"].dtype == np.uint8 and op.slots["outData"].dtype == np.float32
    assert MatrixMultiplyTemplate(None, 4, 1, 16, 1, 1, sample_signed=True).instantiate(
        FakeQueue()).slots["inData"].dtype == np.int8


def test_fused_template():
    t = FusedBeamformerTemplate(None, 8, 4096, 4096, 256, 64, 16, delay_channels=1, sample_signed=True)
    assert t.input_shape == (8, 64, 4096, 256, 2, 2)
    assert t.output_shape == (8, 2, 4096, 16, 16, 32)
    assert t.flags == 1
    assert FusedBeamformerTemplate(None, 1, 4, 4, 16, 4, 1, out_int8=True, exact_coeffs=True).flags == 6
    with pytest.raises(ValueError):
        FusedBeamformerTemplate(None, 1, 4, 4, 16, 4, 1, delay_channels=3)


def test_op_sequence_compounds_alias_buffers():
    tmpl = OpSequenceTemplate(None, 3, 2, 16, 4096, 16, 16, 64, 2, 0, TS, 256)
    op = tmpl.instantiate(FakeQueue())
    assert set(op.slots) == {"bufin_delay_vals", "bufint_coeff", "bufin_reorder", "bufint_data", "bufout_mult"}
    buf = FakeBuf((3, 2, 16, 128, 4), np.float32)
    op.slots["bufint_coeff"].bind(buf)
    assert op.beamform_coeff.buffer("outCoeffs") is buf
    assert op.beamform_mult.buffer("inCoeffs") is buf
    data = FakeBuf((3, 2, 16, 16, 16, 64, 2), np.uint8)
    op.bind(bufint_data=data)
    assert op.prebeamform_reorder.buffer("outReordered") is data and op.beamform_mult.buffer("inData") is data
    with pytest.raises(ValueError):
        op.slots["bufin_reorder"].bind(FakeBuf((1,), np.uint8))
    with pytest.raises(ValueError):
        op()  # unbound slots


def test_compound_slot_rejects_mismatched_children():
    a = accel.IOSlot((2, 3), np.float32)
    b = accel.IOSlot((2, 4), np.float32)
    with pytest.raises(ValueError):
        accel.CompoundIOSlot([a, b])


def test_dimension_and_slot_sizes():
    s = accel.IOSlot((accel.Dimension(4, exact=True), 5), np.float32)
    assert s.shape == (4, 5) and s.required_bytes() == 80


def test_beam_weights_request_semantics():
    """`?beam-weights <beam> w_0..w_{A-1}` (corr3_servlet.py:140-153): the count must equal n_ants; the table starts
    at ones; updates are per beam; int8 output bounds the magnitude (Q14 limbs, int32 accumulator)."""
    t = FusedBeamformerTemplate(None, 1, 4, 4, 16, 5, 3, delay_channels=1, beam_weights=True)
    op = t.instantiate(FakeQueue())
    assert op.slots["beamWeights"].shape == (3, 5)
    np.testing.assert_array_equal(op.beam_weights(), np.ones((3, 5), np.float32))
    op.set_beam_weights(1, 0.5, 0.25, 1, 2, 3)
    op.set_beam_weights(2, np.arange(5))
    w = op.beam_weights()
    np.testing.assert_array_equal(w[0], 1)
    np.testing.assert_array_equal(w[1], [0.5, 0.25, 1, 2, 3])
    np.testing.assert_array_equal(w[2], np.arange(5))
    with pytest.raises(ValueError, match="4 weights received, expected 5"):
        op.set_beam_weights(0, 1, 1, 1, 1)
    with pytest.raises(ValueError):
        op.set_beam_weights(3, *[1] * 5)
    with pytest.raises(ValueError):
        op.set_beam_weights(0, 1, 1, np.nan, 1, 1)
    i8 = FusedBeamformerTemplate(None, 1, 4, 4, 16, 5, 3, out_int8=True, beam_weights=True).instantiate(FakeQueue())
    i8.set_beam_weights(0, 1.992, -1.992, 0, 0, 0)
    with pytest.raises(ValueError, match="out of range"):
        i8.set_beam_weights(0, 2.0, 0, 0, 0, 0)
    with pytest.raises(ValueError, match="without beam_weights"):
        FusedBeamformerTemplate(None, 1, 4, 4, 16, 5, 3).instantiate(FakeQueue()).set_beam_weights(0, *[1] * 5)


def test_streaming_template():
    from dpdk_dc_sand_amd.beamforming import StreamingBeamformerTemplate
    t = StreamingBeamformerTemplate(None, 2, 8, 64, 32, 4, 3, delay_channels=1, batch_dt=1e-3, out_int8=True, depth=3)
    assert (t.depth, t.frame_dt, t.input_shape, t.flags) == (3, 2e-3, (2, 4, 8, 32, 2, 2), 2)
    with pytest.raises(ValueError):
        StreamingBeamformerTemplate(None, 2, 8, 64, 32, 4, 3, depth=0)

