"""ctypes binding of libbf.so (the C ABI in include/bf.h).

The library is built in-tree (`make`, or `__graft_entry__.build()`); there is no fallback: if it is missing,
or a call fails, this module raises.  Every wrapper converts a negative status into
`BeamformerError(bf_last_error())` (the reference's errors surface as Python exceptions from PyCUDA/numba and
as GPU_ERRCHK exits in C++: common/Utils.cpp:8-16).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbf.so")

c_int, c_float, c_double, c_size_t, c_void_p, c_char_p = (ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p)
c_longlong = ctypes.c_longlong
P_int, P_float, P_void = ctypes.POINTER(c_int), ctypes.POINTER(c_float), ctypes.POINTER(c_void_p)
P_size_t, P_longlong = ctypes.POINTER(c_size_t), ctypes.POINTER(c_longlong)

# name -> (restype, argtypes); mirrors include/bf.h (tests/test_abi.py checks the two agree).
PROTOTYPES = {
    "bf_last_error": (c_char_p, []),
    "bf_abi_version": (c_int, []),
    "bf_device_count": (c_int, [P_int]),
    "bf_set_device": (c_int, [c_int]),
    "bf_get_device": (c_int, [P_int]),
    "bf_device_name": (c_int, [c_int, c_char_p, c_size_t]),
    "bf_malloc": (c_int, [P_void, c_size_t]),
    "bf_free": (c_int, [c_void_p]),
    "bf_host_alloc": (c_int, [P_void, c_size_t]),
    "bf_host_free": (c_int, [c_void_p]),
    "bf_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bf_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bf_memcpy_d2d": (c_int, [c_void_p, c_void_p, c_size_t, c_void_p]),
    "bf_memset": (c_int, [c_void_p, c_int, c_size_t, c_void_p]),
    "bf_stream_create": (c_int, [P_void]),
    "bf_stream_destroy": (c_int, [c_void_p]),
    "bf_stream_synchronize": (c_int, [c_void_p]),
    "bf_stream_wait_event": (c_int, [c_void_p, c_void_p]),
    "bf_device_synchronize": (c_int, []),
    "bf_event_create": (c_int, [P_void]),
    "bf_event_destroy": (c_int, [c_void_p]),
    "bf_event_record": (c_int, [c_void_p, c_void_p]),
    "bf_event_synchronize": (c_int, [c_void_p]),
    "bf_event_elapsed_ms": (c_int, [P_float, c_void_p, c_void_p]),
    "bf_trace_mark": (c_int, [c_int, c_void_p]),
    "bf_coeff_gen": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_double,
                             c_void_p]),
    "bf_coeff_gen_time": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_double, c_double, c_double, c_void_p]),
    "bf_coeff_gen_time_study": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                                        c_void_p]),
    "bf_beamform_study_single_channel": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                                 c_int, c_void_p]),
    "bf_reorder": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]),
    "bf_beamform": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                            c_void_p]),
    "bf_beamform_fused": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                  c_int, c_double, c_double, c_double, c_int, c_float, c_void_p]),
    "bf_beamform_fused_weighted": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                           c_int, c_int, c_int, c_double, c_double, c_double, c_int, c_float,
                                           c_void_p]),
    "bf_fused_workspace_bytes": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, P_size_t]),
    "bf_beamform_fused_ws": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                     c_int, c_int, c_int, c_double, c_double, c_double, c_int, c_float, c_void_p,
                                     c_size_t, c_void_p]),
    "bf_q14_coeffs": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                              c_double, c_double, c_double, c_void_p]),
    "bf_pipeline_create": (c_int, [P_void, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_double, c_int,
                                   c_float, c_int, c_int]),
    "bf_pipeline_destroy": (c_int, [c_void_p]),
    "bf_pipeline_frame_bytes": (c_int, [c_void_p, P_size_t, P_size_t]),
    "bf_pipeline_set_delays": (c_int, [c_void_p, c_void_p]),
    "bf_pipeline_set_gains": (c_int, [c_void_p, c_void_p]),
    "bf_pipeline_submit": (c_int, [c_void_p, c_void_p, c_void_p, c_double, c_double, P_longlong]),
    "bf_pipeline_wait": (c_int, [c_void_p, c_longlong, c_int]),
    "bf_pipeline_query": (c_int, [c_void_p, c_longlong, c_int, P_int]),
    "bf_pipeline_flush": (c_int, [c_void_p]),
    "bf_pipeline_stage_ms": (c_int, [c_void_p, c_longlong, P_float, P_float, P_float]),
    "bf_requant": (c_int, [c_void_p, c_void_p, c_size_t, c_float, c_void_p]),
    "bf_fused_algorithmic_bytes": (c_double, [c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "bf_comm_unique_id": (c_int, [c_void_p, c_size_t]),
    "bf_comm_create": (c_int, [P_void, c_void_p, c_size_t, c_int, c_int]),
    "bf_comm_destroy": (c_int, [c_void_p]),
    "bf_comm_allreduce_max": (c_int, [c_void_p, ctypes.POINTER(c_double)]),
    "bf_channel_scatter": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p]),
    "bf_comm_stats": (c_int, [c_void_p, ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]),
    "bf_comm_load": (c_int, []),
    "bf_scatter_plan": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_size_t, c_void_p, c_size_t,
                                ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)]),
    "bf_checksum": (c_int, [c_void_p, c_size_t, c_size_t, c_size_t, ctypes.POINTER(ctypes.c_ulonglong), c_void_p]),
    "bf_fill_random": (c_int, [c_void_p, c_size_t, ctypes.c_ulonglong, c_void_p]),
}


# bf_beamform_fused flags (include/bf.h)
FUSED_SIGNED, FUSED_OUT_INT8, FUSED_EXACT_COEFF, FUSED_INT8_VIA_F32 = 1, 2, 4, 8
# kernel-path / workgroup-order overrides (tests and measurement; every path computes the same contract)
FUSED_PATH = {"auto": 0, "item": 0x100, "generic": 0x300, "wide": 0x400}
FUSED_ORDER = {"auto": 0, "channel": 0x1000, "xcd": 0x2000}


class BeamformerError(RuntimeError):
    """A libbf call returned a negative status."""

    def __init__(self, func, status, message):
        super().__init__(f"{func} failed ({status}): {message}")
        self.func, self.status, self.message = func, status, message


_lock = threading.Lock()
_lib = None


def load(path=None):
    """Load libbf.so (once).  Raises OSError with a build hint when it is missing -- no fallback."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise OSError(f"libbf.so not found at {p}: build it with `make` (or __graft_entry__.build()); "
                          "the beamformer has no CPU fallback")
        lib = ctypes.CDLL(p)
        for name, (res, args) in PROTOTYPES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        if path is None:
            _lib = lib
        return lib


def last_error():
    return load().bf_last_error().decode(errors="replace")


def call(name, *args):
    """Call a status-returning entry point; raise BeamformerError on a negative status."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        raise BeamformerError(name, st, lib.bf_last_error().decode(errors="replace"))
    return st


def ptr(x):
    """Device/host pointer of a DeviceArray, HostArray, int or None as a c_void_p-compatible int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    return x.ptr
