"""FusedSGD (reference: apex/optimizers/fused_sgd.py:6-264).

Includes the amp master-weight integration (``_amp_stash``: fp32 master params updated and the
16-bit model params written in the same kernel, ``materialize_master_grads``) and channels_last
gradients. bf16 model params are handled like fp16 (the reference ignores them).
"""
from __future__ import annotations

import torch
from torch.optim.optimizer import required

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._common import first_device, grad_like_param, noop_buffer, zero_grad

_LOW = (torch.float16, torch.bfloat16)


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True, set_grad_none=False):
        if lr is not required and lr < 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if momentum < 0.0:
            raise ValueError("Invalid momentum value: {}".format(momentum))
        if weight_decay < 0.0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults)
        self.wd_after_momentum = wd_after_momentum
        self.materialize_master_grads = materialize_master_grads
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        self.set_grad_none = set_grad_none
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.multi_tensor_sgd = amp_C.multi_tensor_sgd

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    def get_momentums(self, params):
        momentums = []
        first_run = True
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
        explicit_master_params = hasattr(self, "_amp_stash") and hasattr(self._amp_stash, "fp32_from_fp16_groups")
        for gid, group in enumerate(self.param_groups):
            wd, momentum, dampening, nesterov = (group["weight_decay"], group["momentum"],
                                                 group["dampening"], group["nesterov"])
            launch_sets = []
            if explicit_master_params:
                stash = self._amp_stash
                fp32_params = [p for p in stash.fp32_from_fp32_groups[gid] if p.grad is not None]
                fp32_grads = [grad_like_param(p) for p in fp32_params]
                fp32_moms, fr32 = self.get_momentums(fp32_params)
                if self.materialize_master_grads:
                    pairs = [(m, h) for m, h in zip(stash.fp32_from_fp16_groups[gid], stash.fp16_groups[gid])
                             if m.grad is not None]
                    masters = [m for m, _ in pairs]
                    models = [h for _, h in pairs]
                    grads = [grad_like_param(m) for m in masters]
                else:
                    pairs = [(m, h) for m, h in zip(stash.fp32_from_fp16_groups[gid], stash.fp16_groups[gid])
                             if h.grad is not None]
                    masters = [m for m, _ in pairs]
                    models = [h for _, h in pairs]
                    grads = [grad_like_param(h) for h in models]
                moms, fr16 = self.get_momentums(masters)
                # split the 16-bit copy-out by model dtype (fp16 / bf16)
                for dt in _LOW:
                    idx = [i for i, h in enumerate(models) if h.dtype == dt]
                    if idx:
                        launch_sets.append(([[grads[i] for i in idx], [masters[i] for i in idx],
                                             [moms[i] for i in idx], [models[i] for i in idx]], fr16))
                launch_sets.append(([fp32_grads, fp32_params, fp32_moms], fr32))
            else:
                for dt in (torch.float16, torch.bfloat16, torch.float32, torch.float64):
                    ps = [p for p in group["params"] if p.dtype == dt and p.grad is not None]
                    if not ps:
                        continue
                    moms, fr = self.get_momentums(ps)
                    launch_sets.append(([[grad_like_param(p) for p in ps], ps, moms], fr))
            for lists, first_run in launch_sets:
                if len(lists[0]) == 0:
                    continue
                multi_tensor_applier(self.multi_tensor_sgd, self._dummy_overflow_buf, lists, wd, momentum,
                                     dampening, group["lr"], nesterov, first_run, self.wd_after_momentum,
                                     1.0 / self.most_recent_scale)
        self.most_recent_scale = 1.0
        self.scale_set_by_backward = False
        return loss
