"""Minimal HIP-backed stand-in for the `katsdpsigproc.accel` subset the reference operators use.

Reference callers (e.g. beamform_op_sequence_test.py:105-163, beamform_coeff_test.py:129-165) use:
    ctx = accel.create_some_context(device_filter=lambda x: x.is_cuda, interactive=False)
    queue = ctx.create_command_queue()
    op = SomeTemplate(ctx, ...).instantiate(queue); op.ensure_all_bound()
    buf = op.buffer("slot"); host = buf.empty_like(); buf.set(queue, host); op(); buf.get(queue, host)
plus accel.Dimension / IOSlot / Operation / OperationSequence (compound slots alias one buffer across ops,
beamform_op_sequence.py:148-156).  This module provides exactly that surface over libbf's HIP runtime helpers:
a Context is one GPU, a CommandQueue is one HIP stream, a DeviceArray is one hipMalloc allocation.
"""
import ctypes

import numpy as np

from . import _lib


class Device:
    """One HIP device.  `is_cuda` is True so the reference's `device_filter=lambda d: d.is_cuda` selects it
    (katsdpsigproc's flag for its CUDA-class backend; the backend here is HIP on gfx950)."""

    is_cuda = True
    is_hip = True

    def __init__(self, index):
        self.index = index
        buf = ctypes.create_string_buffer(256)
        _lib.call("bf_device_name", index, buf, 256)
        self.name = buf.value.decode()

    def make_context(self):
        return Context(self)

    def __repr__(self):
        return f"Device({self.index}, {self.name!r})"


def device_count():
    n = ctypes.c_int(0)
    st = _lib.load().bf_device_count(ctypes.byref(n))
    return n.value if st == 0 else 0


def candidate_devices():
    return [Device(i) for i in range(device_count())]


def create_some_context(interactive=False, device_filter=None, device=None):
    """katsdpsigproc.accel.create_some_context: the first device passing `device_filter` (or `device`)."""
    devs = candidate_devices()
    if device is not None:
        devs = [d for d in devs if d.index == device]
    if device_filter is not None:
        devs = [d for d in devs if device_filter(d)]
    if not devs:
        raise RuntimeError("no HIP device available: " + _lib.last_error())
    return devs[0].make_context()


class Context:
    """A context owns the allocations of one device (katsdpsigproc AbstractContext)."""

    def __init__(self, device):
        self.device = device
        _lib.call("bf_set_device", device.index)

    def activate(self):
        _lib.call("bf_set_device", self.device.index)

    def __enter__(self):
        self.activate()
        return self

    def __exit__(self, *exc):
        return False

    def create_command_queue(self, profile=False):
        return CommandQueue(self)

    def allocate_raw(self, nbytes):
        self.activate()
        p = ctypes.c_void_p()
        _lib.call("bf_malloc", ctypes.byref(p), nbytes)
        return p.value or 0

    def empty_like(self, shape, dtype):
        return np.empty(shape, dtype)


class CommandQueue:
    """One non-blocking HIP stream (katsdpsigproc AbstractCommandQueue)."""

    def __init__(self, context):
        self.context = context
        context.activate()
        s = ctypes.c_void_p()
        _lib.call("bf_stream_create", ctypes.byref(s))
        self.handle = s.value

    @property
    def ptr(self):
        return self.handle

    def finish(self):
        _lib.call("bf_stream_synchronize", self.handle)

    def enqueue_marker(self):
        return Event(self)

    def trace_mark(self, tag=0):
        """One empty `bf_trace_mark_kernel` dispatch on this stream: delimits a region of a profiler's kernel trace
        (tools/kernel_stats.py)."""
        _lib.call("bf_trace_mark", int(tag), self.handle)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.load().bf_stream_destroy(h)
            except Exception:
                pass
            self.handle = None


class Event:
    """hipEvent recorded on a queue; `time_since(other)` in seconds (katsdpsigproc AbstractEvent)."""

    def __init__(self, queue=None):
        e = ctypes.c_void_p()
        _lib.call("bf_event_create", ctypes.byref(e))
        self.handle = e.value
        if queue is not None:
            self.record(queue)

    def record(self, queue):
        _lib.call("bf_event_record", self.handle, queue.handle if queue is not None else None)

    def wait(self):
        _lib.call("bf_event_synchronize", self.handle)

    def time_since(self, prior):
        ms = ctypes.c_float()
        _lib.call("bf_event_elapsed_ms", ctypes.byref(ms), prior.handle, self.handle)
        return ms.value * 1e-3

    def __del__(self):
        h = getattr(self, "handle", None)
        if h:
            try:
                _lib.load().bf_event_destroy(h)
            except Exception:
                pass
            self.handle = None


class Dimension:
    """One axis of a slot (katsdpsigproc accel.Dimension); only exact sizes are needed here."""

    def __init__(self, size, min_padded_size=None, alignment=1, align_dtype=None, exact=False):
        self.size = int(size)
        self.exact = exact

    def __repr__(self):
        return f"Dimension({self.size})"


class _PinnedAllocation:
    """Owner of one bf_host_alloc (hipHostMalloc) block; freed when the last array view goes away."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ctypes.c_void_p()
        _lib.call("bf_host_alloc", ctypes.byref(p), max(self.nbytes, 1))
        self.ptr = p.value

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                _lib.load().bf_host_free(self.ptr)
            except Exception:
                pass
            self.ptr = None


class HostArray(np.ndarray):
    """Page-locked host array (katsdpsigproc accel.HostArray): the host side of asynchronous copies and of the
    streaming pipeline's frames, so DMA can overlap compute.  A numpy array in every other respect; views keep
    the allocation alive."""

    def __new__(cls, shape, dtype, context=None):
        shape = tuple(int(s) for s in (shape if np.ndim(shape) else (shape,)))
        dtype = np.dtype(dtype)
        count = int(np.prod(shape, dtype=np.int64))
        if context is not None:
            context.activate()
        alloc = _PinnedAllocation(count * dtype.itemsize)
        raw = (ctypes.c_uint8 * max(count * dtype.itemsize, 1)).from_address(alloc.ptr)
        obj = np.frombuffer(raw, dtype=dtype, count=count).reshape(shape).view(cls)
        obj._alloc = alloc
        return obj

    def __array_finalize__(self, obj):
        self._alloc = getattr(obj, "_alloc", None)

    @property
    def ptr(self):
        return self.ctypes.data


class DeviceArray:
    """Device buffer with numpy-like metadata (katsdpsigproc accel.DeviceArray subset)."""

    def __init__(self, context, shape, dtype, ptr=None, owner=True):
        self.context = context
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        self._owner = owner and ptr is None
        self.ptr = ptr if ptr is not None else context.allocate_raw(self.nbytes)

    @property
    def buffer(self):
        # The reference passes `slot.buffer` to its kernels; here the array itself is the handle.
        return self

    @property
    def size(self):
        return self.nbytes // self.dtype.itemsize

    def empty_like(self):
        return np.empty(self.shape, self.dtype)

    def zero(self, queue):
        _lib.call("bf_memset", self.ptr, 0, self.nbytes, queue.handle)

    def _check(self, ary):
        ary = np.asarray(ary)
        if ary.shape != self.shape or ary.dtype != self.dtype:
            raise ValueError(f"host array {ary.shape}/{ary.dtype} does not match device {self.shape}/{self.dtype}")
        return ary

    def set_async(self, queue, ary):
        ary = np.ascontiguousarray(self._check(ary))
        self._keep = ary  # keep alive until the copy retires (the queue is synchronised by set())
        _lib.call("bf_memcpy_h2d", self.ptr, ary.ctypes.data, self.nbytes, queue.handle)

    def set(self, queue, ary):
        """Synchronous host -> device copy (katsdpsigproc DeviceArray.set)."""
        self.set_async(queue, ary)
        queue.finish()
        self._keep = None

    def get_async(self, queue, ary=None):
        if ary is None:
            ary = self.empty_like()
        ary = self._check(ary)
        if not ary.flags.c_contiguous or not ary.flags.writeable:
            raise ValueError("destination must be a writeable C-contiguous array")
        _lib.call("bf_memcpy_d2h", ary.ctypes.data, self.ptr, self.nbytes, queue.handle)
        return ary

    def get(self, queue, ary=None):
        """Synchronous device -> host copy (katsdpsigproc DeviceArray.get)."""
        ary = self.get_async(queue, ary)
        queue.finish()
        return ary

    def copy_region(self, queue, src):
        if src.nbytes != self.nbytes:
            raise ValueError("size mismatch")
        _lib.call("bf_memcpy_d2d", self.ptr, src.ptr, self.nbytes, queue.handle)

    def __del__(self):
        if getattr(self, "_owner", False) and getattr(self, "ptr", None):
            try:
                self.context.activate()
                _lib.load().bf_free(self.ptr)
            except Exception:
                pass
            self.ptr = None


class IOSlot:
    """A named operand of an Operation (katsdpsigproc accel.IOSlot): fixed shape and dtype."""

    def __init__(self, dimensions, dtype):
        self.dimensions = tuple(d if isinstance(d, Dimension) else Dimension(d, exact=True) for d in dimensions)
        self.shape = tuple(d.size for d in self.dimensions)
        self.dtype = np.dtype(dtype)
        self.buffer = None

    def check(self, buf):
        if tuple(buf.shape) != self.shape or np.dtype(buf.dtype) != self.dtype:
            raise ValueError(f"buffer {buf.shape}/{buf.dtype} does not match slot {self.shape}/{self.dtype}")

    def bind(self, buf):
        if buf is not None:
            self.check(buf)
        self.buffer = buf

    def allocate(self, context):
        buf = DeviceArray(context, self.shape, self.dtype)
        self.bind(buf)
        return buf

    def required_bytes(self):
        return int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize


class CompoundIOSlot(IOSlot):
    """Several slots (of several operations) sharing one buffer (katsdpsigproc accel.CompoundIOSlot)."""

    def __init__(self, children):
        first = children[0]
        for c in children[1:]:
            if c.shape != first.shape or c.dtype != first.dtype:
                raise ValueError(f"compound slots disagree: {c.shape}/{c.dtype} vs {first.shape}/{first.dtype}")
        super().__init__(first.dimensions, first.dtype)
        self.children = list(children)

    def bind(self, buf):
        super().bind(buf)
        for c in self.children:
            c.bind(buf)


class Operation:
    """Base class of a device operation with named slots (katsdpsigproc accel.Operation)."""

    def __init__(self, command_queue):
        self.command_queue = command_queue
        self.slots = {}

    def bind(self, **kwargs):
        for name, buf in kwargs.items():
            self.slots[name].bind(buf)

    def ensure_bound(self, name):
        slot = self.slots[name]
        if slot.buffer is None:
            slot.allocate(self.command_queue.context)
        return slot.buffer

    def ensure_all_bound(self):
        for name in self.slots:
            self.ensure_bound(name)

    def buffer(self, name):
        return self.slots[name].buffer

    def required_bytes(self):
        return sum(s.required_bytes() for s in self.slots.values())

    def _run(self):
        raise NotImplementedError

    def __call__(self, **kwargs):
        if kwargs:
            self.bind(**kwargs)
        for name, slot in self.slots.items():
            if slot.buffer is None:
                raise ValueError(f"slot {name!r} is not bound")
        self.command_queue.context.activate()
        self._run()


class OperationSequence(Operation):
    """Runs operations in order; compounds alias a buffer across their slots (katsdpsigproc
    accel.OperationSequence, used at beamform_op_sequence.py:117-157)."""

    def __init__(self, command_queue, operations, compounds=None, aliases=None):
        super().__init__(command_queue)
        self.operations = dict(operations)
        self._order = [name for name, _ in operations]
        claimed = set()
        for cname, members in (compounds or {}).items():
            children = []
            for m in members:
                op_name, slot_name = m.split(":")
                children.append(self.operations[op_name].slots[slot_name])
                claimed.add(m)
            self.slots[cname] = CompoundIOSlot(children)
        # Slots not named by a compound are exposed as "op:slot".
        for op_name, op in self.operations.items():
            for slot_name, slot in op.slots.items():
                key = f"{op_name}:{slot_name}"
                if key not in claimed:
                    self.slots[key] = CompoundIOSlot([slot])

    def _run(self):
        for name in self._order:
            self.operations[name]._run()
