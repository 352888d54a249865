"""Whole-step HIP graph capture: one training step (forward, backward, loss scaling, optimizer) recorded
once as a hipGraph and replayed, so a step costs one graph launch instead of ~650 kernel launches from
Python.

This is the MI355X replacement for a tracing compiler: the step is still ordinary eager code (the
fused HIP kernels, hipBLASLt, RCCL), captured by ``torch.cuda.CUDAGraph`` (hipStreamBeginCapture).
What a captured step requires of the code inside it:

* no host synchronisation -- amp's device-resident loss scaler (``BH_AMP_DEVICE_SCALER=1``,
  amp/scaler.py) and the optimizers' device step counters (``_device_step``) keep the whole step on
  the device;
* static tensors: the step reads its inputs from tensors the caller refills in place
  (``static_x.copy_(batch)``) and its outputs stay in graph-owned memory (copy them out before the
  next replay if they must be kept);
* host scalars frozen at capture time (learning rate, weight decay) stay frozen: re-capture after
  changing them, or keep them in device tensors.

Kernels launch on the current stream (bindings/common.h ``stream_for``), so the capture stream picks
them up; the multi-tensor plan cache (bindings/mta.cpp) pins plans created while capturing.
"""
from __future__ import annotations

import time
from typing import Any, Callable, Optional

import torch


class GraphedStep:
    """``step = GraphedStep(fn); out = step()`` -- ``fn()`` runs ``warmup`` times eagerly on a side
    stream (so lazy initialisation, bucket building and plan caches reach steady state), then once
    under capture; each call replays the graph and returns the tensors ``fn`` returned during capture
    (refreshed in place by the replay)."""

    def __init__(self, fn: Callable[[], Any], warmup: int = 3, pool=None):
        self.fn = fn
        self.warmup = warmup
        self.pool = pool
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.capture_ms = 0.0

    def capture(self) -> "GraphedStep":
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(self.warmup):
                self.fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            self.out = self.fn()
        torch.cuda.synchronize()
        self.capture_ms = (time.perf_counter() - t0) * 1e3
        self.graph = g
        return self

    def __call__(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()
        return self.out

    def reset(self):
        """Drop the graph (and its memory pool); the next call captures again."""
        self.graph = None
        self.out = None
