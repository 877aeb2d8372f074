"""Python face of the native HIP runtime layer (csrc/hip/runtime.hip, in libtbhip.so).

Everything the device path needs — HBM and pinned host memory from caching allocators,
non-blocking streams, events, async copies and fills, per-thread current device and stream —
without importing PyTorch. Arrays are 1-D typed views of a cached block:

    a = hiprt.empty(n, np.int64)            # HBM, uninitialised
    z = hiprt.zeros(n, np.int32)            # memset on the current stream
    d = hiprt.to_device(host_array)         # synchronous upload (init-time tables)
    with hiprt.stream(s):                   # launches and fills go to s
        ...
    host = d.to_host()                      # synchronous download
    p = hiprt.pinned(nbytes, np.uint8)      # numpy view of page-locked memory

Lifetime rule (the same one the pipeline follows for every batch): a block returns to its
cache when the last Python reference to it is dropped, so code that queues GPU work on an
array keeps a reference until that work's completion event has been waited on.
"""
from __future__ import annotations

import contextlib
import ctypes
import threading
from typing import Iterator, Optional

import numpy as np

from ..errors import DeviceError

_lib = None
_lock = threading.Lock()
_tls = threading.local()
_default_streams = {}


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                from .. import native

                _lib = native.hip()
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise DeviceError(f"{what} failed with hipError_t {rc}")


# ---------------------------------------------------------------------------------------------
# devices

def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().tbrt_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


def set_device(index: int) -> None:
    check(lib().tbrt_set_device(int(index)), "hipSetDevice")
    _tls.device = int(index)


def current_device() -> int:
    d = getattr(_tls, "device", None)
    if d is None:
        v = ctypes.c_int(0)
        check(lib().tbrt_get_device(ctypes.byref(v)), "hipGetDevice")
        d = _tls.device = v.value
    return d


def parse_device(device) -> int:
    """'cuda', 'cuda:1', 1, or an object with an ``index`` attribute -> device index."""
    if device is None:
        return current_device()
    if isinstance(device, int):
        return device
    if not isinstance(device, str):
        idx = getattr(device, "index", None)   # e.g. torch.device
        if isinstance(idx, int):
            return idx
    s = str(device)
    if s in ("cuda", "hip", "gpu"):
        return current_device()
    for pre in ("cuda:", "hip:", "gpu:"):
        if s.startswith(pre):
            return int(s[len(pre):])
    raise DeviceError(f"unknown device {device!r}")


def synchronize() -> None:
    check(lib().tbrt_device_sync(), "hipDeviceSynchronize")


def mem_info():
    f, t = ctypes.c_size_t(0), ctypes.c_size_t(0)
    check(lib().tbrt_mem_info(ctypes.byref(f), ctypes.byref(t)), "hipMemGetInfo")
    return f.value, t.value


def cache_stats() -> dict:
    a = (ctypes.c_size_t * 6)()
    check(lib().tbrt_cache_stats(a), "tbrt_cache_stats")
    return dict(device_in_use=a[0], device_cached=a[1], device_peak=a[2], host_in_use=a[3], host_cached=a[4],
                host_peak=a[5])


def empty_cache() -> None:
    check(lib().tbrt_empty_cache(), "tbrt_empty_cache")


# ---------------------------------------------------------------------------------------------
# streams and events

class Stream:
    """A non-blocking HIP stream on the current device (lower priority value = higher priority)."""

    def __init__(self, priority: int = 0, handle: Optional[int] = None):
        if handle is not None:
            self.handle = handle
            return
        lo, hi = ctypes.c_int(0), ctypes.c_int(0)
        check(lib().tbrt_stream_priority_range(ctypes.byref(lo), ctypes.byref(hi)), "hipDeviceGetStreamPriorityRange")
        prio = max(min(priority, lo.value), hi.value)  # HIP: lo = least, hi = greatest priority
        h = ctypes.c_void_p()
        check(lib().tbrt_stream_create(ctypes.byref(h), prio), "hipStreamCreate")
        self.handle = h.value or 0

    def synchronize(self) -> None:
        check(lib().tbrt_stream_sync(self.handle), "hipStreamSynchronize")

    def wait_event(self, ev: "Event") -> None:
        check(lib().tbrt_stream_wait_event(self.handle, ev.handle), "hipStreamWaitEvent")

    def record(self, timing: bool = False) -> "Event":
        ev = Event(timing)
        ev.record(self)
        return ev


# host waits on events sleep instead of spinning (TB_TUNE event_blocking=0: spin, HIP's default;
# DeviceRunner sets it from its tuning)
_BLOCKING_EVENTS = True


def set_blocking_events(on: bool) -> None:
    global _BLOCKING_EVENTS
    _BLOCKING_EVENTS = bool(on)


class Event:
    def __init__(self, timing: bool = False, blocking: Optional[bool] = None):
        h = ctypes.c_void_p()
        blocking = _BLOCKING_EVENTS if blocking is None else blocking
        flags = (1 if timing else 0) | (2 if blocking else 0)
        check(lib().tbrt_event_create(ctypes.byref(h), flags), "hipEventCreate")
        self.handle = h.value

    def record(self, s: Optional[Stream] = None) -> "Event":
        s = s or current_stream()
        check(lib().tbrt_event_record(self.handle, s.handle), "hipEventRecord")
        return self

    def synchronize(self) -> None:
        check(lib().tbrt_event_sync(self.handle), "hipEventSynchronize")

    def query(self) -> bool:
        r = lib().tbrt_event_query(self.handle)
        if r >= 2:
            raise DeviceError(f"hipEventQuery failed with hipError_t {r - 2}")
        return r == 0

    def elapsed_time(self, end: "Event") -> float:
        """Milliseconds between this event and ``end`` (both created with timing=True)."""
        ms = ctypes.c_float(0)
        check(lib().tbrt_event_elapsed(ctypes.byref(ms), self.handle, end.handle), "hipEventElapsedTime")
        return ms.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.tbrt_event_destroy(h)


def default_stream(device: Optional[int] = None) -> Stream:
    """Per-device non-blocking stream used when no ``stream(...)`` context is active."""
    d = current_device() if device is None else device
    s = _default_streams.get(d)
    if s is None:
        with _lock:
            s = _default_streams.get(d)
            if s is None:
                s = _default_streams[d] = Stream()
    return s


def current_stream() -> Stream:
    st = getattr(_tls, "stack", None)
    return st[-1] if st else default_stream()


@contextlib.contextmanager
def stream(s: Stream) -> Iterator[Stream]:
    st = getattr(_tls, "stack", None)
    if st is None:
        st = _tls.stack = []
    st.append(s)
    try:
        yield s
    finally:
        st.pop()


# ---------------------------------------------------------------------------------------------
# memory

class _Block:
    __slots__ = ("ptr", "nbytes", "host", "__weakref__")

    def __init__(self, nbytes: int, host: bool = False):
        self.ptr = 0
        p = ctypes.c_void_p()
        n = max(int(nbytes), 1)
        if host:
            check(lib().tbrt_host_alloc(ctypes.byref(p), n), f"pinned alloc of {n} bytes")
        else:
            check(lib().tbrt_malloc(ctypes.byref(p), n), f"device alloc of {n} bytes")
        self.ptr = p.value
        self.nbytes = n
        self.host = host

    def __del__(self):
        if self.ptr and _lib is not None:
            (_lib.tbrt_host_free if self.host else _lib.tbrt_free)(self.ptr)
            self.ptr = 0


class DevArray:
    """1-D typed view of device memory (``data_ptr``/``numel`` like the kernel launchers expect)."""

    __slots__ = ("block", "offset", "n", "dtype")

    def __init__(self, block: _Block, offset: int, n: int, dtype):
        self.block = block
        self.offset = offset
        self.n = n
        self.dtype = np.dtype(dtype)

    # -- introspection
    def data_ptr(self) -> int:
        return self.block.ptr + self.offset

    def numel(self) -> int:
        return self.n

    def __len__(self) -> int:
        return self.n

    @property
    def nbytes(self) -> int:
        return self.n * self.dtype.itemsize

    @property
    def shape(self):
        return (self.n,)

    # -- views
    def __getitem__(self, sl) -> "DevArray":
        if not isinstance(sl, slice) or (sl.step not in (None, 1)):
            raise TypeError("DevArray supports contiguous slices only")
        a, b, _ = sl.indices(self.n)
        b = max(a, b)
        return DevArray(self.block, self.offset + a * self.dtype.itemsize, b - a, self.dtype)

    def view(self, dtype) -> "DevArray":
        dt = np.dtype(dtype)
        if self.nbytes % dt.itemsize:
            raise ValueError("view: size not a multiple of the new item size")
        return DevArray(self.block, self.offset, self.nbytes // dt.itemsize, dt)

    # -- copies
    def copy_from_host(self, a: np.ndarray, s: Optional[Stream] = None) -> None:
        """Async H2D on ``s`` (the source must stay alive and unchanged until the copy is done;
        pageable sources are staged by the runtime before this returns)."""
        if not a.flags.c_contiguous:
            raise ValueError("copy_from_host: the source must be contiguous (an async copy reads it later)")
        if a.nbytes > self.nbytes:
            raise ValueError("copy_from_host: source larger than the destination")
        if a.nbytes:
            check(lib().tbrt_memcpy_h2d(self.data_ptr(), a.ctypes.data, a.nbytes, (s or current_stream()).handle),
                  "hipMemcpyAsync H2D")

    def copy_to_host(self, out: np.ndarray, s: Optional[Stream] = None) -> None:
        """Async D2H into ``out`` (pinned for a truly asynchronous copy)."""
        if not out.flags.c_contiguous or out.nbytes < self.nbytes:
            raise ValueError("copy_to_host: destination too small or not contiguous")
        if self.nbytes:
            check(lib().tbrt_memcpy_d2h(out.ctypes.data, self.data_ptr(), self.nbytes, (s or current_stream()).handle),
                  "hipMemcpyAsync D2H")

    def copy_from(self, src: "DevArray", s: Optional[Stream] = None) -> None:
        if src.nbytes > self.nbytes:
            raise ValueError("copy_from: source larger than the destination")
        if src.nbytes:
            check(lib().tbrt_memcpy_d2d(self.data_ptr(), src.data_ptr(), src.nbytes, (s or current_stream()).handle),
                  "hipMemcpyAsync D2D")

    def to_host(self) -> np.ndarray:
        """Synchronous download (on the current stream) into a new numpy array."""
        out = np.empty(self.n, dtype=self.dtype)
        s = current_stream()
        self.copy_to_host(out, s)
        s.synchronize()
        return out

    def fill_(self, byte: int = 0, s: Optional[Stream] = None) -> "DevArray":
        if self.nbytes:
            check(lib().tbrt_memset(self.data_ptr(), int(byte), self.nbytes, (s or current_stream()).handle),
                  "hipMemsetAsync")
        return self


def empty(n: int, dtype=np.uint8) -> DevArray:
    dt = np.dtype(dtype)
    return DevArray(_Block(int(n) * dt.itemsize), 0, int(n), dt)


def zeros(n: int, dtype=np.uint8, s: Optional[Stream] = None) -> DevArray:
    return empty(n, dtype).fill_(0, s)


def to_device(a, dtype=None) -> DevArray:
    """Synchronous upload of a host array (or bytes) — for tables and small operands."""
    if isinstance(a, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(a), dtype=np.uint8)
    a = np.ascontiguousarray(a, dtype=dtype).reshape(-1)
    d = empty(len(a), a.dtype)
    s = current_stream()
    d.copy_from_host(a, s)
    s.synchronize()
    return d


def pinned(n: int, dtype=np.uint8) -> np.ndarray:
    """numpy array over page-locked host memory; the memory returns to the pinned cache when the
    array (and every view of it) is gone."""
    dt = np.dtype(dtype)
    nbytes = max(int(n) * dt.itemsize, 1)
    blk = _Block(nbytes, host=True)
    raw = (ctypes.c_uint8 * nbytes).from_address(blk.ptr)
    raw._tb_block = blk        # the ctypes buffer owns the block; numpy's base owns the buffer
    return np.frombuffer(raw, dtype=np.uint8)[: int(n) * dt.itemsize].view(dt)


def is_pinned(a: np.ndarray) -> bool:
    """True when ``a`` is a view of memory from :func:`pinned` (page-locked: an async H2D copy
    can DMA straight from it, no staging copy)."""
    obj = a
    for _ in range(8):
        if obj is None:
            return False
        if getattr(obj, "_tb_block", None) is not None:
            return True
        obj = getattr(obj, "base", None) if not isinstance(obj, memoryview) else obj.obj
    return False


def scan_strided_i64(src: DevArray, stride: int, n: int, out: DevArray, s: Optional[Stream] = None) -> None:
    """out[i] = sum(src[j * stride] for j <= i), i < n (k_scan_strided_i64)."""
    if src.dtype != np.int64 or out.dtype != np.int64:
        raise DeviceError("scan_strided_i64 needs int64 operands")
    if n < 0 or out.n < n or (n and (n - 1) * stride >= src.n) or stride < 1:
        raise DeviceError("scan_strided_i64: operand shapes")
    check(lib().tb_scan_strided_i64((s or current_stream()).handle, src.data_ptr(), stride, n, out.data_ptr()),
          "tb_scan_strided_i64")
