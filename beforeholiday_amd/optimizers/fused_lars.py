"""FusedLARS (reference: apex/optimizers/fused_lars.py:7-224).

Per-tensor trust ratio ``tc * ||w|| / (||g|| + wd * ||w|| + eps)`` from deterministic per-tensor
norms, then momentum SGD, one launch per dtype bucket. Groups may set ``is_skipped=True`` to use
the plain learning rate (e.g. for BN/bias params). bf16 params are supported.
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import required

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._common import first_device, grad_like_param, noop_buffer, zero_grad


class FusedLARS(torch.optim.Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0,
                 trust_coefficient=0.001, eps=0.0, nesterov=False, wd_after_momentum=False,
                 materialize_master_grads=True, set_grad_none=False):
        if lr is not required and lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if momentum < 0.0:
            raise ValueError("Invalid momentum value: {}".format(momentum))
        if weight_decay < 0.0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, trust_coefficient=trust_coefficient, eps=eps, is_skipped=False)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults)
        self.wd_after_momentum = wd_after_momentum
        self.materialize_master_grads = materialize_master_grads
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        self.set_grad_none = set_grad_none
        self.trust_coefficient = trust_coefficient
        self.eps = eps
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
        self.multi_tensor_lars = amp_C.multi_tensor_lars

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    def get_momentums(self, params):
        momentums, first_run = [], True
        for p in params:
            st = self.state[p]
            if "momentum_buffer" not in st:
                first_run = True
                st["momentum_buffer"] = torch.zeros_like(p)
            else:
                first_run = False
            momentums.append(st["momentum_buffer"])
        return momentums, first_run

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            for dt in (torch.float16, torch.bfloat16, torch.float32):
                ps = [p for p in group["params"] if p.dtype == dt and p.grad is not None]
                if not ps:
                    continue
                gs = [grad_like_param(p) for p in ps]
                moms, first_run = self.get_momentums(ps)
                w_norms = multi_tensor_applier(self.multi_tensor_l2norm, self._dummy_overflow_buf, [ps], True)[1]
                g_norms = multi_tensor_applier(self.multi_tensor_l2norm, self._dummy_overflow_buf, [gs], True)[1]
                multi_tensor_applier(self.multi_tensor_lars, self._dummy_overflow_buf, [gs, ps, moms], g_norms,
                                     w_norms, group["lr"], group["trust_coefficient"], self.eps,
                                     group["weight_decay"], group["momentum"], group["dampening"],
                                     group["nesterov"], first_run, self.wd_after_momentum,
                                     1.0 / self.most_recent_scale, group["is_skipped"])
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        return loss
