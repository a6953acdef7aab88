"""Optional roctx ranges for rocprofv3 timelines (the reference has no tracing).

Enabled with ``TORCHKAFKA_ROCTX=1``.  Ranges show up under ``--marker-trace`` in
rocprofv3 (never combine marker tracing with ``--pmc`` on this pool).  When
disabled, :func:`trace_range` is a no-op context manager with no per-call cost
beyond the ``with`` statement.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = os.environ.get("TORCHKAFKA_ROCTX") == "1"


def _load():
    global _lib, _enabled
    if _lib is not None or not _enabled:
        return _lib
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            _lib = ctypes.CDLL(name)
            _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            return _lib
        except OSError:
            continue
    _enabled = False
    return None


def enabled() -> bool:
    return _enabled and _load() is not None


@contextlib.contextmanager
def trace_range(name: str):
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
