"""MI355X-native (gfx950) beamformer: the hot path of magnate3/dpdk_dc_sand's `beamformer/beamforming` package.

    dpdk_dc_sand_amd.accel        -- HIP-backed stand-in for the katsdpsigproc.accel subset the operators use
    dpdk_dc_sand_amd.beamforming  -- drop-in operators (same class names, constructor signatures, slots)
    dpdk_dc_sand_amd._lib         -- ctypes binding of libbf.so (C ABI: include/bf.h)

All compute runs in hand-written HIP kernels in libbf.so; there is no CPU fallback.
"""
__version__ = "0.1.0"
