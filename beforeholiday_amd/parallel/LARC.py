"""LARC: layer-wise adaptive rate clipping/scaling wrapper (reference: apex/parallel/LARC.py).

Per-parameter trust ratio ``tc * ||p|| / (||g|| + wd * ||p|| + eps)`` (clipped to lr when
``clip=True``) applied to the gradients before the wrapped optimizer's step. All parameter and
gradient norms come from two multi-tensor norm launches and the ratios stay on the device (the
reference issues two norm kernels and a host-synchronising comparison per parameter).
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from ..multi_tensor_apply import multi_tensor_applier_l2norm
from ..ops import amp_C


class LARC(object):
    def __init__(self, optimizer, trust_coefficient=0.02, clip=True, eps=1e-8):
        self.optim = optimizer
        self.trust_coefficient = trust_coefficient
        self.eps = eps
        self.clip = clip

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    @property
    def state(self):
        return self.optim.state

    def __repr__(self):
        return self.optim.__repr__()

    @property
    def param_groups(self):
        return self.optim.param_groups

    @param_groups.setter
    def param_groups(self, value):
        self.optim.param_groups = value

    def state_dict(self):
        return self.optim.state_dict()

    def load_state_dict(self, state_dict):
        self.optim.load_state_dict(state_dict)

    def zero_grad(self, *args, **kwargs):
        self.optim.zero_grad(*args, **kwargs)

    def add_param_group(self, param_group):
        self.optim.add_param_group(param_group)

    def _norms(self, tensors):
        by = {}
        for i, t in enumerate(tensors):
            by.setdefault(t.dtype, []).append(i)
        out = torch.empty(len(tensors), device=tensors[0].device)
        noop = torch.zeros(1, dtype=torch.int, device=tensors[0].device)
        for idx in by.values():
            per = multi_tensor_applier_l2norm(amp_C.multi_tensor_l2norm, noop, [[tensors[i] for i in idx]], True)[1]
            out[idx] = per
        return out

    def step(self, closure=None):
        with torch.no_grad():
            weight_decays = []
            for group in self.optim.param_groups:
                weight_decay = group.get("weight_decay", 0)
                weight_decays.append(weight_decay)
                group["weight_decay"] = 0
                params = [p for p in group["params"] if p.grad is not None]
                if not params:
                    continue
                pn = self._norms([p.data for p in params])
                gn = self._norms([p.grad.data for p in params])
                ok = (pn != 0) & (gn != 0)
                adaptive = self.trust_coefficient * pn / (gn + pn * weight_decay + self.eps)
                if self.clip:
                    adaptive = torch.clamp(adaptive / group["lr"], max=1.0)
                factor = torch.where(ok, adaptive, torch.ones_like(adaptive))
                wd = torch.where(ok, torch.full_like(pn, float(weight_decay)), torch.zeros_like(pn))
                for i, p in enumerate(params):
                    p.grad.data.add_(p.data * wd[i].to(p.dtype)).mul_(factor[i].to(p.grad.dtype))
        self.optim.step(closure) if closure is not None else self.optim.step()
        for i, group in enumerate(self.optim.param_groups):
            group["weight_decay"] = weight_decays[i]
