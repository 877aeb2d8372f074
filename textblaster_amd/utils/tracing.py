"""roctx ranges around the pipeline phases (the reference's tracing spans
``process_task``/``pipeline_step``, worker_logic.rs:44,150, become timeline ranges here).

Enabled with ``TB_ROCTX=1``: ranges are pushed through librocprofiler-sdk-roctx, so a
``rocprofv3 --marker-trace --kernel-trace`` run shows, per thread, the host phases of every
batch (stage_h2d, launch, gpu_wait, resolve, assemble, parquet read/write) next to the kernels
they enqueue. Disabled (the default) the helpers cost one attribute check.

``TB_TIMELINE=<path>`` (or ``record_timeline(path)``) additionally records every range in
process as ``(thread, name, start, end)`` and ``dump_timeline()`` writes them as JSON: a
profiler-free host timeline of the reader / submit / wait / assemble / writer overlap
(tools/timeline_summary.py turns it into per-thread busy time and the critical path).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from typing import Iterator, List, Optional, Tuple

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("TB_ROCTX", "") not in ("", "0")
_tl_path: Optional[str] = os.environ.get("TB_TIMELINE") or None
_tl_events: List[Tuple[str, str, float, float]] = []
_tl_lock = threading.Lock()
_tl_t0 = time.perf_counter()


def record_timeline(path: Optional[str]) -> None:
    """Start (path) or stop (None) recording host ranges; clears earlier events."""
    global _tl_path, _tl_t0
    with _tl_lock:
        _tl_path = path
        _tl_events.clear()
        _tl_t0 = time.perf_counter()


def timeline_events() -> List[Tuple[str, str, float, float]]:
    with _tl_lock:
        return list(_tl_events)


def dump_timeline(suffix: str = "") -> Optional[str]:
    """Writes the recorded ranges to the timeline path (+suffix); returns the file name."""
    if not _tl_path:
        return None
    path = _tl_path + suffix
    ev = timeline_events()
    with open(path, "w", encoding="utf-8") as f:
        json.dump({"t0": 0.0, "events": [{"thread": t, "name": n, "start": round(a - _tl_t0, 6),
                                          "end": round(b - _tl_t0, 6)} for t, n, a, b in ev]}, f)
    return path


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
    t0 = time.perf_counter() if _tl_path else 0.0
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
        if _tl_path and t0:
            t1 = time.perf_counter()
            with _tl_lock:
                _tl_events.append((threading.current_thread().name, name, t0, t1))


def mark(name: str) -> None:
    lib = _load() if _enabled else None
    if lib is not None:
        lib.roctxMarkA(name.encode())


def name_os_thread(name: str) -> None:
    """Give the calling thread an OS-level name (15 chars, Linux prctl PR_SET_NAME) so per-thread
    CPU profiles (tools/thread_cpu.py) can attribute it; a no-op elsewhere."""
    try:
        import ctypes

        libc = ctypes.CDLL(None)
        libc.prctl(15, name.encode()[:15], 0, 0, 0)  # PR_SET_NAME
    except Exception:  # noqa: BLE001 - best effort
        pass
