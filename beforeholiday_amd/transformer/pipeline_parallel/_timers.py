"""Named interval timers for the pipeline schedules (API of apex/transformer/pipeline_parallel/_timers.py:
``timers(name).start() / .stop() / .elapsed(reset)``, ``timers.log(names)``, ``timers.write(...)``).

Device-side design: on a GPU, ``start`` / ``stop`` only RECORD a pair of HIP events on the current stream,
so timing a region never stalls the host or drains the queue (the reference synchronises the whole device
at every start and stop). Intervals pile up as event pairs and are resolved lazily: ``elapsed`` waits for
the last recorded stop event only, then sums ``start.elapsed_time(stop)`` over the pairs. Without a GPU the
same interface runs on ``time.perf_counter``.

An interval is tied to the stream it started on: stopping it from another stream raises (the event pair
would measure nothing meaningful), and work on streams the timed stream does not wait on is not counted.
``_Timers(sync=True)`` (or ``BH_TIMERS_SYNC=1``) restores the reference's device-synchronised wall-clock
timing for regions that include host or side-stream work. Closed intervals are folded into the total
whenever more than ``_FOLD_AT`` are pending, for the ones whose stop event has already completed.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Iterable, List, Optional, Tuple

import torch


def _on_device() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_initialized()


_FOLD_AT = 64  # closed intervals pending before the completed ones are folded into the total


class _Interval:
    """One started (and maybe stopped) interval: a pair of HIP events on one stream, or two perf_counter
    stamps (no GPU, or sync mode: the device is synchronised at both ends, as the reference does)."""

    __slots__ = ("dev", "sync", "stream", "t0", "t1")

    def __init__(self, sync: bool = False):
        on = _on_device()
        self.sync = sync and on
        self.dev = on and not sync
        self.stream = None
        if self.dev:
            self.stream = torch.cuda.current_stream()
            self.t0 = torch.cuda.Event(enable_timing=True)
            self.t0.record(self.stream)
        else:
            if self.sync:
                torch.cuda.synchronize()
            self.t0 = time.perf_counter()
        self.t1 = None

    def close(self, name: str = "?"):
        if self.dev:
            cur = torch.cuda.current_stream()
            if cur != self.stream:
                raise RuntimeError(f"timer {name!r} started on {self.stream} and stopped on {cur}: an event pair "
                                   "across streams measures nothing (time each stream separately, or sync mode)")
            self.t1 = torch.cuda.Event(enable_timing=True)
            self.t1.record(self.stream)
        else:
            if self.sync:
                torch.cuda.synchronize()
            self.t1 = time.perf_counter()

    def done(self) -> bool:
        return not self.dev or self.t1.query()

    def seconds(self) -> float:
        if self.dev:
            self.t1.synchronize()
            return self.t0.elapsed_time(self.t1) / 1000.0
        return self.t1 - self.t0


class _Timer:
    def __init__(self, name: str, sync: bool = False):
        self.name = name
        self.sync = sync
        self._done: List[_Interval] = []  # closed intervals not yet folded into _total
        self._open: Optional[_Interval] = None
        self._total = 0.0  # seconds of resolved intervals

    @property
    def running(self) -> bool:
        return self._open is not None

    def start(self):
        if self._open is not None:
            raise RuntimeError(f"timer {self.name!r} is already running")
        self._open = _Interval(self.sync)

    def stop(self):
        if self._open is None:
            raise RuntimeError(f"timer {self.name!r} was not started")
        self._open.close(self.name)
        self._done.append(self._open)
        self._open = None
        if len(self._done) > _FOLD_AT:  # fold the finished pairs (no wait) so they do not pile up
            keep = []
            for iv in self._done:
                if iv.done():
                    self._total += iv.seconds()
                else:
                    keep.append(iv)
            self._done = keep

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

    def __init__(self, sync: Optional[bool] = None):
        self.timers: Dict[str, _Timer] = {}
        self.sync = os.environ.get("BH_TIMERS_SYNC", "0") == "1" if sync is None else sync

    def __call__(self, name: str) -> _Timer:
        t = self.timers.get(name)
        if t is None:
            t = self.timers[name] = _Timer(name, self.sync)
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
