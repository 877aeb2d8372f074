"""roctx ranges around the pipeline phases (the reference's tracing spans
``process_task``/``pipeline_step``, worker_logic.rs:44,150, become timeline ranges here).

Enabled with ``TB_ROCTX=1``: ranges are pushed through librocprofiler-sdk-roctx, so a
``rocprofv3 --marker-trace --kernel-trace`` run shows, per thread, the host phases of every
batch (stage_h2d, launch, gpu_wait, resolve, assemble, parquet read/write) next to the kernels
they enqueue. Disabled (the default) the helpers cost one attribute check.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterator, Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("TB_ROCTX", "") not in ("", "0")


def _load() -> Optional[ctypes.CDLL]:
    global _lib, _enabled
    if _lib is not None or not _enabled:
        return _lib
    for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4",
                 "/opt/rocm/lib/libroctx64.so.4"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.argtypes = []
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.restype = None
            _lib = lib
            return lib
        except OSError:
            continue
    _enabled = False  # no roctx library: tracing stays off
    return None


def enabled() -> bool:
    return _enabled and _load() is not None


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    """``with trace_range("resolve"): ...`` -> one roctx range (no-op unless TB_ROCTX=1)."""
    lib = _load() if _enabled else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _load() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())
