"""FusedAdagrad (reference: apex/optimizers/fused_adagrad.py:5-121)."""
from __future__ import annotations

import torch

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._common import first_device, grad_like_param, noop_buffer, zero_grad


class FusedAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-2, eps=1e-10, weight_decay=0.0, set_grad_none=True,
                 adagrad_w_mode=False):
        defaults = dict(lr=lr, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adagrad_w_mode = 1 if adagrad_w_mode else 0
        self.set_grad_none = set_grad_none
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.multi_tensor_adagrad = amp_C.multi_tensor_adagrad

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdagrad does not support sparse gradients")
                if p.dtype not in (torch.float16, torch.bfloat16, torch.float32):
                    raise RuntimeError("FusedAdagrad only support fp16, bfloat16 and fp32.")
                state = self.state[p]
                if len(state) == 0:
                    state["sum"] = torch.zeros_like(p)
                lists = buckets.setdefault(p.dtype, [[], [], []])
                lists[0].append(grad_like_param(p)), lists[1].append(p), lists[2].append(state["sum"])
            for lists in buckets.values():
                multi_tensor_applier(self.multi_tensor_adagrad, self._dummy_overflow_buf, lists, group["lr"],
                                     group["eps"], self.adagrad_w_mode, group["weight_decay"])
        return loss
