"""Legacy FusedSGD driven by ``contrib.optimizers.FP16_Optimizer`` (explicit grads / output params /
scale) (reference: apex/contrib/optimizers/fused_sgd.py:7-240): one multi-tensor SGD launch per
(fp16 model, fp32 master) set, writing the fp16 model copy in the same pass."""
import torch
from torch.optim.optimizer import Optimizer, required

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C
from ._legacy import group_lists


class FusedSGD(Optimizer):
    def __init__(self, params, lr=required, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 wd_after_momentum=False, materialize_master_grads=True):
        if lr is not required and lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay, nesterov=nesterov)
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, defaults)
        self.wd_after_momentum = wd_after_momentum

    def __setstate__(self, state):
        super().__setstate__(state)
        for group in self.param_groups:
            group.setdefault("nesterov", False)

    def get_momentums(self, params):
        momentums, first_run = [], True
        for p in params:
            st = self.state[p]
            if "momentum_buffer" not in st:
                st["momentum_buffer"] = torch.zeros_like(p)
            else:
                first_run = False
            momentums.append(st["momentum_buffer"])
        return momentums, first_run

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=1.0, grad_norms=None):
        if hasattr(self, "_amp_stash"):
            raise RuntimeError("apex.contrib.optimizers.FusedSGD should not be used with AMP.")
        loss = closure() if closure is not None else None
        if grads is None:
            raise RuntimeError("apex.contrib.optimizers.FusedSGD must be wrapped with "
                               "apex.contrib.optimizers.FP16_Optimizer which provides grads.")
        if output_params is None:
            raise RuntimeError("apex.contrib.optimizers.FusedSGD must be wrapped with "
                               "apex.contrib.optimizers.FP16_Optimizer which provides output_params.")
        n = len(self.param_groups)
        for group, g_this, o_this in zip(self.param_groups, group_lists(grads, n), group_lists(output_params, n)):
            if g_this is None or o_this is None:
                raise RuntimeError("apex.contrib.optimizers.FusedSGD only works when all parameters require grad.")
            # (the reference leaves fp32 model params un-updated here; they get the copy-out like fp16 ones)
            fp32 = [(g, p2, p1) for (p1, g, p2) in zip(o_this, g_this, group["params"]) if p1.dtype == torch.float32]
            fp16 = [(g, p2, p1) for (p1, g, p2) in zip(o_this, g_this, group["params"]) if p1.dtype != torch.float32]
            sets = []
            if fp16:
                m, first = self.get_momentums([x[1] for x in fp16])
                sets.append(([x[0] for x in fp16], [x[1] for x in fp16], m, [x[2] for x in fp16], first))
            if fp32:
                m, first = self.get_momentums([x[1] for x in fp32])
                sets.append(([x[0] for x in fp32], [x[1] for x in fp32], m, [x[2] for x in fp32], first))
            for g, p, m, copy, first in sets:
                lists = [g, p, m] + ([copy] if copy is not None else [])
                flag = torch.zeros(1, dtype=torch.int, device=p[0].device)
                multi_tensor_applier(amp_C.multi_tensor_sgd, flag, lists, group["weight_decay"], group["momentum"],
                                     group["dampening"], group["lr"], group["nesterov"], first,
                                     self.wd_after_momentum, 1.0 / scale)
        return loss
