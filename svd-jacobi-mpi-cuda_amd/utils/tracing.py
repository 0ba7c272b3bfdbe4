"""Tracing and phase timing.

The reference has no instrumentation beyond one omp_get_wtime pair around the
whole solve (reference main.cu:1586, 1610-1611).  Here:

* ROCTX ranges (``libroctx64``) around sweeps / rounds / phases, visible in
  ``rocprofv3 --marker-trace`` timelines; no-ops when the library is absent;
* :class:`PhaseTimer` -- HIP-event based per-phase device time, accumulated
  without host synchronisation until :meth:`PhaseTimer.summary`.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import time
from collections import defaultdict

import torch

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("SVDJ_NO_ROCTX") == "1":
        return None
    for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = C.CDLL(name)
            lib.roctxRangePushA.argtypes = [C.c_char_p]
            lib.roctxRangePushA.restype = C.c_int
            lib.roctxRangePop.restype = C.c_int
            lib.roctxMarkA.argtypes = [C.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


@contextlib.contextmanager
def trace_range(name: str):
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str):
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


class PhaseTimer:
    """Accumulates device time per named phase with HIP events (CPU: wall)."""

    def __init__(self, device, enabled: bool = True):
        self.cuda = torch.device(device).type == "cuda" and enabled
        self.enabled = enabled
        self._pending = defaultdict(list)
        self._cpu = defaultdict(float)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        with trace_range(name):
            if self.cuda:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                yield
                e1.record()
                self._pending[name].append((e0, e1))
            else:
                t0 = time.perf_counter()
                yield
                self._cpu[name] += time.perf_counter() - t0

    def summary(self) -> dict:
        out = dict(self._cpu)
        if self.cuda and self._pending:
            torch.cuda.synchronize()
            for k, evs in self._pending.items():
                out[k] = out.get(k, 0.0) + sum(a.elapsed_time(b) for a, b in evs) / 1e3
        return {k: round(v, 6) for k, v in out.items()}
