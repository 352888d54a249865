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

    def __init__(self, fn: Callable[[], Any], warmup: int = 3, pool=None, before: Optional[Callable[[], Any]] = None):
        self.fn = fn
        self.warmup = warmup
        self.pool = pool
        self.before = before
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.capture_ms = 0.0

    def capture(self) -> "GraphedStep":
        # warm-up and capture run on ONE side stream; ``before`` runs there first (DDP re-registers its
        # gradient hooks there: autograd runs a hooked parameter's AccumulateGrad node on the stream the
        # node was created on, and a node created on the default stream is not part of a capture on
        # another one -- the replay then misses those accumulations)
        # A caller already on a side stream (bench.py builds DDP and trains on one) captures right there.
        cur = torch.cuda.current_stream()
        side = cur if cur != torch.cuda.default_stream() else torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            if self.before is not None:
                self.before()
            for _ in range(self.warmup):
                self.fn()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool, stream=side):
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


def training_state(*roots, model=None, optimizer=None):
    """Every device tensor a training step mutates, for :func:`capture_checked`'s save / restore:
    the model's parameters and buffers, the optimizer's parameters (amp's fp32 masters), their group's
    device hyper-parameters and state,
    and the tensor attributes (one level deep) of the optimizer, its amp stash and every extra root
    (loss scalers: device scale / counters / flags; device step counters). Deduplicated by storage
    pointer + shape."""
    out, seen = [], set()

    def add(t):
        if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() > 0:
            key = (t.data_ptr(), tuple(t.shape), t.dtype)
            if key not in seen:
                seen.add(key)
                out.append(t)

    if model is not None:
        for t in list(model.parameters()) + list(model.buffers()):
            add(t)
    if optimizer is not None:
        for g in optimizer.param_groups:
            for p in g["params"]:
                add(p)
            for k, v in g.items():  # device hyper-parameters (capturable FusedAdam: lr and step tensors)
                if k != "params":
                    add(v)
        for st in optimizer.state.values():
            for v in (st.values() if isinstance(st, dict) else ()):
                add(v)
        roots = roots + (optimizer, getattr(optimizer, "_amp_stash", None))
    for r in roots:
        if r is None:
            continue
        for v in vars(r).values():
            if isinstance(v, (list, tuple)):
                for x in v:
                    add(x)
            else:
                add(v)
    return out


def _rehook_ddp(model):
    """Re-register the gradient hooks of every beforeholiday_amd DDP module in ``model`` on the current
    stream (see GraphedStep.capture)."""
    from ..parallel.distributed import DistributedDataParallel

    if model is None:
        return
    for m in model.modules():
        if isinstance(m, DistributedDataParallel) and m._collectives:
            m._refresh_params()


def capture_checked(fn: Callable[[], torch.Tensor], state, watch=(), warmup: int = 2, group=None, model=None):
    """Capture ``fn`` (a training step returning its loss) and PROVE the replay before using it.

    1. capture (a failure on any rank is agreed on by all ranks before anyone replays a collective);
    2. save ``state`` (:func:`training_state`), replay once, record the loss and ``watch``; restore the
       saved state, run ``fn`` eagerly, compare loss and ``watch`` BITWISE;
    3. one MIN all-reduce of the verdict: every rank keeps the graph, or every rank runs eager in this
       same process (collectives stay matched: the agreement is an eager collective on all ranks).

    Returns ``(runner, report)``: the :class:`GraphedStep` or ``fn`` itself, and a dict for logs. The
    check costs two steps and one copy of the state; it runs at every world size (world 1 included)."""
    import torch.distributed as dist

    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1

    def agree(ok: bool) -> bool:
        if not multi:
            return ok
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        return bool(int(t.item()))

    g = GraphedStep(fn, warmup=warmup, before=lambda: _rehook_ddp(model))
    err = None
    try:
        g.capture()
        ok = True
    except Exception as e:  # noqa: BLE001 - any capture failure means: run eager
        ok, err = False, f"{type(e).__name__}: {e}"
        g.reset()
        torch.cuda.synchronize()
    if not agree(ok):
        return fn, {"graph": "eager (capture failed on some rank)", "error": err}
    saved = [t.detach().clone() for t in state]
    # torch's own dropout draws from the device generator, whose (seed, offset) the replay advances on the
    # host: the eager step restarts from the same generator state as the replay
    rng = torch.cuda.get_rng_state() if torch.cuda.is_available() else None
    torch.cuda.synchronize()
    loss_g = g().detach().clone()
    got = [loss_g] + [w.detach().clone() for w in watch]
    with torch.no_grad():
        for t, s in zip(state, saved):
            t.copy_(s)
    if rng is not None:
        torch.cuda.set_rng_state(rng)
    loss_e = fn().detach().clone()
    want = [loss_e] + [w.detach().clone() for w in watch]
    torch.cuda.synchronize()
    diffs = [i for i, (a, b) in enumerate(zip(got, want)) if not (a.shape == b.shape and torch.equal(a, b))]
    same = not diffs
    rep = {}
    if diffs:
        # diagnosis: is the eager step itself bitwise repeatable from the same state? (a non-deterministic
        # kernel -- float atomics, a timed algorithm pick -- makes any replay check fail)
        with torch.no_grad():
            for t, s_ in zip(state, saved):
                t.copy_(s_)
        if rng is not None:
            torch.cuda.set_rng_state(rng)
        fn()
        again = [w.detach().clone() for w in watch]
        rep["eager_repeatable"] = all(torch.equal(a, b) for a, b in zip(again, want[1:]))
        rep["mismatch"] = [(i, tuple(got[i].shape), float((got[i].float() - want[i].float()).abs().max()))
                           for i in diffs[:6]]
        rep["n_mismatch"] = len(diffs)
    del saved
    if not agree(same):
        g.reset()
        rep.update({"graph": "eager (replay != eager step on some rank)", "capture_ms": round(g.capture_ms, 1),
                    "loss_graph": float(loss_g), "loss_eager": float(loss_e)})
        return fn, rep
    return g, {"graph": "captured (replay == eager step, bitwise, every rank)", "capture_ms": round(g.capture_ms, 1),
               "state_tensors": len(state)}
