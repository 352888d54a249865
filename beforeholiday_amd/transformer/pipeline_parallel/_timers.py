"""Named interval timers for the pipeline schedules (API of apex/transformer/pipeline_parallel/_timers.py:
``timers(name).start() / .stop() / .elapsed(reset)``, ``timers.log(names)``, ``timers.write(...)``).

Device-side design: on a GPU, ``start`` / ``stop`` only RECORD a pair of HIP events on the current stream,
so timing a region never stalls the host or drains the queue (the reference synchronises the whole device
at every start and stop). Intervals pile up as event pairs and are resolved lazily: ``elapsed`` waits for
the last recorded stop event only, then sums ``start.elapsed_time(stop)`` over the pairs. Without a GPU the
same interface runs on ``time.perf_counter``.
"""
from __future__ import annotations

import time
from typing import Dict, Iterable, List, Optional, Tuple

import torch


def _on_device() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_initialized()


class _Interval:
    """One started (and maybe stopped) interval: a pair of HIP events, or two perf_counter stamps."""

    __slots__ = ("dev", "t0", "t1")

    def __init__(self):
        self.dev = _on_device()
        if self.dev:
            self.t0 = torch.cuda.Event(enable_timing=True)
            self.t0.record()
        else:
            self.t0 = time.perf_counter()
        self.t1 = None

    def close(self):
        if self.dev:
            self.t1 = torch.cuda.Event(enable_timing=True)
            self.t1.record()
        else:
            self.t1 = time.perf_counter()

    def seconds(self) -> float:
        if self.dev:
            self.t1.synchronize()
            return self.t0.elapsed_time(self.t1) / 1000.0
        return self.t1 - self.t0


class _Timer:
    def __init__(self, name: str):
        self.name = name
        self._done: List[_Interval] = []  # closed intervals not yet folded into _total
        self._open: Optional[_Interval] = None
        self._total = 0.0  # seconds of resolved intervals

    @property
    def running(self) -> bool:
        return self._open is not None

    def start(self):
        if self._open is not None:
            raise RuntimeError(f"timer {self.name!r} is already running")
        self._open = _Interval()

    def stop(self):
        if self._open is None:
            raise RuntimeError(f"timer {self.name!r} was not started")
        self._open.close()
        self._done.append(self._open)
        self._open = None

    def reset(self):
        self._done.clear()
        self._open = None
        self._total = 0.0

    def _resolve(self) -> float:
        # the events complete in record order on one stream: the waits after the first return at once
        self._total += sum(iv.seconds() for iv in self._done)
        self._done.clear()
        return self._total

    def elapsed(self, reset: bool = True) -> float:
        """Seconds accumulated so far. A running interval is cut here and continues in a new one."""
        running = self._open is not None
        if running:
            self.stop()
        value = self._resolve()
        if reset:
            self.reset()
        if running:
            self.start()
        return value


class _Timers:
    """``timers(name)`` returns (creating on first use) the named :class:`_Timer`."""

    def __init__(self):
        self.timers: Dict[str, _Timer] = {}

    def __call__(self, name: str) -> _Timer:
        t = self.timers.get(name)
        if t is None:
            t = self.timers[name] = _Timer(name)
        return t

    def _values(self, names: Iterable[str], normalizer: float, reset: bool) -> List[Tuple[str, float]]:
        if not normalizer > 0.0:
            raise ValueError("normalizer must be positive")
        return [(n, self.timers[n].elapsed(reset=reset) / normalizer) for n in names]

    def write(self, names, writer, iteration, normalizer=1.0, reset=False):
        """``writer.add_scalar(f"{name}-time", seconds / normalizer, iteration)`` per timer (TensorBoard)."""
        for n, v in self._values(names, normalizer, reset):
            writer.add_scalar(f"{n}-time", v, iteration)

    def log(self, names, normalizer=1.0, reset=True):
        """Print one line of per-timer milliseconds; on the last rank only when distributed."""
        parts = [f"{n}: {v * 1e3:.2f}" for n, v in self._values(names, normalizer, reset)]
        line = "time (ms) | " + " | ".join(parts)
        dist = torch.distributed
        if dist.is_available() and dist.is_initialized() and dist.get_rank() != dist.get_world_size() - 1:
            return
        print(line, flush=True)
