"""Diagnostic: error of the GPU beamformer and of the f32 CPU oracle against the exact (float64) product."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import oracle as O
from dpdk_dc_sand_amd import accel
from dpdk_dc_sand_amd.beamforming import MatrixMultiplyTemplate

TS = O.TS_MEERKAT
ctx = accel.create_some_context()
q = ctx.create_command_queue()


def delays(C, M, A, kind, seed=0):
    d = np.zeros((C, M, A, 4), np.float32)
    if kind == "uniform":
        d[..., 0] = np.single(5 * TS); d[..., 2] = np.single(np.pi / 2)
    else:
        r = np.random.default_rng(seed)
        d[..., 0] = r.uniform(0, 10 * TS, (C, M, A)); d[..., 2] = r.uniform(-np.pi, np.pi, (C, M, A))
    return d


for (A, M, C, B, kind) in [(5, 2, 1638, 3, "uniform"), (64, 16, 64, 2, "random"), (64, 2, 16, 3, "uniform"),
                           (256, 64, 8, 1, "random"), (19, 2, 431, 3, "uniform")]:
    T = 256
    d = delays(C, M, A, kind, A)
    w = O.coeffs(d, B, 2, C, 4096 * 8, A, M, 0)
    x = O.u8_voltages((B, 2, C, T // 16, 16, A, 2))
    op = MatrixMultiplyTemplate(ctx, A, C, T, M, B).instantiate(q)
    op.ensure_all_bound()
    op.buffer("inData").set(q, x); op.buffer("inCoeffs").set(q, w); op()
    y = op.buffer("outData").get(q)
    y32 = O.complex_mult(x, w)
    X = x.reshape(B, 2, C, T, 2 * A).astype(np.float64)
    ex = np.matmul(X, w.astype(np.float64)).reshape(y.shape)
    mag = np.matmul(np.abs(X), np.abs(w).astype(np.float64)).reshape(y.shape)
    tol = 1e-4 + 1e-4 * np.abs(ex)
    eg, eo = np.abs(y - ex), np.abs(y32 - ex)
    tol_o = 1e-4 + 1e-4 * np.abs(y32)
    print(f"A={A} M={M} C={C} {kind}: n={y.size}")
    print(f"   gpu vs exact : viol {(eg > tol).sum()}  max {eg.max():.2e}  max/mag {(eg / mag).max():.2e}")
    print(f"   f32 oracle vs exact: viol {(eo > tol).sum()}  max {eo.max():.2e}  max/mag {(eo / mag).max():.2e}")
    print(f"   gpu vs oracle: viol {(np.abs(y - y32) > tol_o).sum()}")
