"""Legacy loss scalers for FP16_Optimizer (reference: apex/fp16_utils/loss_scaler.py:10-133)."""
from __future__ import annotations

import torch


def to_python_float(t):
    return t.item() if hasattr(t, "item") else t[0]


class LossScaler:
    """Static loss scale."""

    def __init__(self, scale=1):
        self.cur_scale = scale

    def has_overflow(self, params):
        return False

    def _has_inf_or_nan(x):
        return False

    def update_scale(self, overflow):
        pass

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)


class DynamicLossScaler:
    """Dynamic loss scale: /factor on overflow, x factor after ``scale_window`` clean steps."""

    def __init__(self, init_scale=2 ** 32, scale_factor=2.0, scale_window=1000):
        self.cur_scale = init_scale
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window

    def has_overflow_serial(self, params):
        for p in params:
            if p.grad is not None and DynamicLossScaler._has_inf_or_nan(p.grad.data):
                return True
        return False

    def has_overflow(self, params):
        # one device reduction over every gradient instead of a host sync per tensor
        grads = [p.grad.data for p in params if p.grad is not None]
        if not grads:
            return False
        flags = torch.stack([(~torch.isfinite(g.float())).any() for g in grads])
        return bool(flags.any().item())

    @staticmethod
    def _has_inf_or_nan(x):
        try:
            cpu_sum = float(x.float().sum())
        except RuntimeError as instance:
            if "value cannot be converted" not in instance.args[0]:
                raise
            return True
        return cpu_sum in (float("inf"), -float("inf")) or cpu_sum != cpu_sum

    def update_scale(self, overflow):
        if overflow:
            self.cur_scale = max(self.cur_scale / self.scale_factor, 1)
            self.last_overflow_iter = self.cur_iter
        elif (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
            self.cur_scale *= self.scale_factor
        self.cur_iter += 1

    @property
    def loss_scale(self):
        return self.cur_scale

    def scale_gradient(self, module, grad_in, grad_out):
        return tuple(self.loss_scale * g for g in grad_in)

    def backward(self, loss, retain_graph=False):
        (loss * self.loss_scale).backward(retain_graph=retain_graph)
