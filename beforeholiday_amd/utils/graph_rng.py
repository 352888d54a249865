"""Dropout seeds a captured training step can replay (utils/graphs.py).

The fused dropout kernels (the flash attention kernels of kernels/attn.hip, the bias-dropout-add of
kernels/dense.hip) take their seed as a host integer, drawn per call from a CPU generator
(transformer/tensor_parallel/random.py ``dropout_seed``, contrib/multihead_attn/_core.py ``_seed``). A
HIP graph freezes kernel arguments, so a replayed step would draw the SAME masks every step. In device
mode the seed has two parts:

* a per-call salt, fixed by the call's position in the step (the n-th dropout call of every step gets
  the same salt, so capture and replay agree on it), passed as the host integer;
* the step seed, an int64 [1] device tensor that :func:`new_step` advances ON THE DEVICE at the start of
  each step (inside the captured region), which the kernels read and mix into the salt.

Forward and backward of one step see the same step seed, so the attention backward regenerates the
forward's mask. The step seed is an ordinary device tensor: ``utils.training_state`` picks it up through
``state_tensors()`` for capture_checked's save / restore.

    graph_rng.enable()          # once, before warm-up / capture
    def step():
        graph_rng.new_step()    # first thing in the step
        ...
"""
from __future__ import annotations

from typing import Optional

import torch

_step_seed: Optional[torch.Tensor] = None
_calls = 0


def enable(seed: int = 0, device=None) -> torch.Tensor:
    """Switch the fused dropout kernels to device step seeds (returns the int64 [1] step-seed tensor)."""
    global _step_seed, _calls
    _step_seed = torch.full((1,), int(seed), dtype=torch.int64,
                            device=device if device is not None else torch.device("cuda", torch.cuda.current_device()))
    _calls = 0
    return _step_seed


def disable() -> None:
    global _step_seed, _calls
    _step_seed, _calls = None, 0


def active() -> bool:
    return _step_seed is not None


def step_seed() -> Optional[torch.Tensor]:
    return _step_seed


def state_tensors():
    """The device state a captured step mutates here (for utils.training_state roots)."""
    return [_step_seed] if _step_seed is not None else []


def new_step() -> None:
    """Start a step: advance the step seed on the device and restart the per-call salts."""
    global _calls
    if _step_seed is not None:
        _step_seed.add_(1)
        _calls = 0


def _mix64(x: int) -> int:
    x &= (1 << 64) - 1
    x ^= x >> 33
    x = (x * 0xFF51AFD7ED558CCD) & ((1 << 64) - 1)
    x ^= x >> 33
    x = (x * 0xC4CEB9FE1A85EC53) & ((1 << 64) - 1)
    return x ^ (x >> 33)


def next_salt(stream: int = 0) -> int:
    """The host part of the next dropout call's seed: a hash of (stream, call index within the step).
    ``stream`` separates seed streams that must differ (tensor-parallel ranks)."""
    global _calls
    _calls += 1
    return _mix64(stream * 0x9E3779B97F4A7C15 + _calls) & ((1 << 62) - 1)
