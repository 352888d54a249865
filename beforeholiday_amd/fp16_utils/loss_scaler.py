"""Loss scalers of the legacy ``FP16_Optimizer`` (reference: apex/fp16_utils/loss_scaler.py:10-133).

Both classes share one base: the scale itself, ``backward`` (scaled loss) and ``scale_gradient``
(a module backward hook that scales ``grad_in``). The static one never overflows; the dynamic one
halves (``/ scale_factor``, floor 1) on an overflowing step and doubles after ``scale_window`` clean
steps since the last overflow. The overflow test is one device-side reduction over all gradients
(one host sync per step) instead of one ``float(sum)`` round trip per tensor.
"""
from __future__ import annotations

import torch


def to_python_float(t):
    return t.item() if hasattr(t, "item") else t[0]


def _nonfinite(x: torch.Tensor) -> torch.Tensor:
    """0-dim bool device tensor: x holds an Inf or NaN."""
    return torch.logical_not(torch.isfinite(x)).any()


class _ScaleBase:
    def __init__(self, scale):
        self.cur_scale = scale

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.cur_scale * g for g in grad_in)

    def backward(self, loss, retain_graph=False):
        (loss * self.cur_scale).backward(retain_graph=retain_graph)


class LossScaler(_ScaleBase):
    """A fixed loss scale: never reports an overflow, never changes."""

    def __init__(self, scale=1):
        super().__init__(scale)

    def has_overflow(self, params):
        return False

    @staticmethod
    def _has_inf_or_nan(x):
        return False

    def update_scale(self, overflow):
        return None


class DynamicLossScaler(_ScaleBase):
    """Loss scale that backs off on Inf / NaN gradients and grows again after a clean window."""

    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000):
        super().__init__(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window

    @staticmethod
    def _has_inf_or_nan(x):
        return bool(_nonfinite(x.float()).item())

    def has_overflow_serial(self, params):
        return any(p.grad is not None and self._has_inf_or_nan(p.grad) for p in params)

    def has_overflow(self, params):
        flags = [_nonfinite(p.grad) for p in params if p.grad is not None]
        return bool(torch.stack(flags).any().item()) if flags else False

    def update_scale(self, overflow):
        since = self.cur_iter - self.last_overflow_iter
        if overflow:
            self.cur_scale = max(self.cur_scale / self.scale_factor, 1)
            self.last_overflow_iter = self.cur_iter
        elif since % self.scale_window == 0:
            self.cur_scale *= self.scale_factor
        self.cur_iter += 1
