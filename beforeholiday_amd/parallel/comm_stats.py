"""Opt-in timing of the collectives on the training hot path (DDP bucket waits, SyncBN all-reduces).

Off by default (zero cost: one module-level bool test per call site). Inside
``with comm_stats.collect():`` every instrumented call site records a pair of HIP events on the
compute stream around the point where the compute stream depends on the collective:

* ``ddp_wait``   -- end-of-backward wait on each gradient bucket's all-reduce (the part of the
  bucketed all-reduce that did NOT overlap with backward);
* ``syncbn_fwd`` / ``syncbn_bwd`` -- the blocking SyncBatchNorm statistics collectives.

``summary()`` synchronises once and returns ``{name: {"ms": total, "calls": n}}``. CPU tensors
(gloo) are timed with the host clock instead. The reference has only NVTX ranges for this
(``apex/parallel/distributed.py:360-361,517-518``); this is the counter we report in
the benchmark line.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Tuple

import torch

_enabled = False
_events: Dict[str, List[Tuple[object, object]]] = defaultdict(list)
_host: Dict[str, List[float]] = defaultdict(list)


def enabled() -> bool:
    return _enabled


def reset() -> None:
    _events.clear()
    _host.clear()


@contextlib.contextmanager
def collect():
    global _enabled
    prev = _enabled
    _enabled = True
    try:
        yield
    finally:
        _enabled = prev


@contextlib.contextmanager
def timed(name: str, ref: torch.Tensor):
    """Time the enclosed region on ``ref``'s device stream (no-op unless collecting)."""
    if not _enabled:
        yield
        return
    if ref.is_cuda:
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        yield
        b.record()
        _events[name].append((a, b))
    else:
        t0 = time.perf_counter()
        yield
        _host[name].append((time.perf_counter() - t0) * 1e3)


def summary() -> Dict[str, Dict[str, float]]:
    out: Dict[str, Dict[str, float]] = {}
    if _events:
        torch.cuda.synchronize()
    for name, pairs in _events.items():
        out[name] = {"ms": sum(a.elapsed_time(b) for a, b in pairs), "calls": len(pairs)}
    for name, vals in _host.items():
        d = out.setdefault(name, {"ms": 0.0, "calls": 0})
        d["ms"] += sum(vals)
        d["calls"] += len(vals)
    return out
