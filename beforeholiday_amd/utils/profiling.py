"""Tracing helpers: named ranges visible in rocprofv3 / torch.profiler traces, device-event timers,
profiler start/stop brackets (reference: NVTX ranges in apex/parallel/distributed.py and
examples/imagenet/main_amp.py --prof, hipified to roctx on ROCm).

``range_push`` / ``range_pop`` go through ``torch.cuda.nvtx`` (roctx on ROCm builds) and also
open a ``torch.profiler.record_function`` scope, so the same annotation shows up in both tools.
"""
import contextlib
import functools
import time

import torch

_stack = []


def range_push(name: str) -> None:
    rf = torch.profiler.record_function(name)
    rf.__enter__()
    _stack.append(rf)
    try:
        torch.cuda.nvtx.range_push(name)
    except Exception:  # noqa: BLE001 - no roctx in CPU-only builds
        pass


def range_pop() -> None:
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:  # noqa: BLE001
        pass
    if _stack:
        _stack.pop().__exit__(None, None, None)


@contextlib.contextmanager
def profile_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


def annotate(name=None):
    """Decorator: run the function inside a named range."""
    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            with profile_range(label):
                return fn(*args, **kwargs)
        return wrapper
    return deco


def profiler_start():
    """Start capture for ``rocprofv3 --selected-regions`` style runs (hipProfilerStart)."""
    if torch.cuda.is_available():
        try:
            torch.cuda.cudart().cudaProfilerStart()
        except Exception:  # noqa: BLE001
            pass


def profiler_stop():
    if torch.cuda.is_available():
        try:
            torch.cuda.cudart().cudaProfilerStop()
        except Exception:  # noqa: BLE001
            pass


class EventTimer:
    """Device-side elapsed time between ``start()`` and ``stop()`` (HIP events, no host sync until
    ``elapsed_ms``); falls back to wall clock on CPU."""

    def __init__(self):
        self._gpu = torch.cuda.is_available()
        self._start = self._end = None
        self._t0 = self._t1 = None

    def start(self):
        if self._gpu:
            self._start = torch.cuda.Event(enable_timing=True)
            self._start.record()
        else:
            self._t0 = time.perf_counter()
        return self

    def stop(self):
        if self._gpu:
            self._end = torch.cuda.Event(enable_timing=True)
            self._end.record()
        else:
            self._t1 = time.perf_counter()
        return self

    def elapsed_ms(self) -> float:
        if self._gpu:
            self._end.synchronize()
            return self._start.elapsed_time(self._end)
        return (self._t1 - self._t0) * 1000.0


def report_memory(name: str = "") -> str:
    """Allocated / reserved device memory summary string (MB)."""
    if not torch.cuda.is_available():
        return f"{name} memory: n/a (no GPU)"
    mb = 2.0 ** 20
    return (f"{name} memory (MB) | allocated: {torch.cuda.memory_allocated() / mb:.1f} | max allocated: "
            f"{torch.cuda.max_memory_allocated() / mb:.1f} | reserved: {torch.cuda.memory_reserved() / mb:.1f}")
