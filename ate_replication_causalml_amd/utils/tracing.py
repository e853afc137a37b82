"""Tracing / profiling.

The reference has no instrumentation beyond a "~1min" comment
(ate_functions.R:168,230). Here every estimator, nuisance fit and fold runs inside
``trace(name)``, which

* pushes a roctx range (libroctx64, loaded with ctypes) so ``rocprofv3
  --marker-trace`` / ``--kernel-trace`` timelines group kernels by estimator;
* records host wall time and, on a GPU, device time between two HIP events on the
  current stream;
* appends a span record to the process-wide ``TRACE`` list (exportable as JSONL).

Tracing is on by default and costs two event records per span; ``ATE_TRACE=0``
disables the device events (roctx pushes are free when no profiler is attached).
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from dataclasses import asdict, dataclass, field

_roctx = None
_roctx_tried = False
_lock = threading.Lock()


def _lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


def mark(msg: str):
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


@dataclass
class Span:
    name: str
    depth: int
    wall_ms: float
    device_ms: float | None
    attrs: dict = field(default_factory=dict)


TRACE: list[Span] = []
_depth = threading.local()


def _events_enabled():
    return os.environ.get("ATE_TRACE", "1") != "0"


@contextlib.contextmanager
def trace(name: str, **attrs):
    """Time a region (host wall + device events) and label it for rocprof."""
    import torch
    lib = _lib()
    d = getattr(_depth, "v", 0)
    _depth.v = d + 1
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    ev = None
    if _events_enabled() and torch.cuda.is_available() and torch.cuda.is_initialized():
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dev_ms = None
        if ev is not None:
            ev[1].record()
            ev[1].synchronize()
            dev_ms = ev[0].elapsed_time(ev[1])
        wall = (time.perf_counter() - t0) * 1e3
        if lib is not None:
            lib.roctxRangePop()
        _depth.v = d
        with _lock:
            TRACE.append(Span(name, d, wall, dev_ms, attrs))


def reset():
    with _lock:
        TRACE.clear()


def spans(name_prefix: str = ""):
    return [s for s in TRACE if s.name.startswith(name_prefix)]


def export_jsonl(path):
    with open(path, "a") as f:
        for s in TRACE:
            f.write(json.dumps(asdict(s)) + "\n")


def summary() -> str:
    lines = [f"{'span':50s} {'wall ms':>10s} {'device ms':>10s}"]
    for s in TRACE:
        dm = "" if s.device_ms is None else f"{s.device_ms:10.2f}"
        lines.append(f"{'  ' * s.depth + s.name:50s} {s.wall_ms:10.2f} {dm:>10s}")
    return "\n".join(lines)
