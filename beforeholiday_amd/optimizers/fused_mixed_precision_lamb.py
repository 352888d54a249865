"""FusedMixedPrecisionLamb (reference: apex/optimizers/fused_mixed_precision_lamb.py:8-256).

Sync-free LAMB: lr and step are device tensors, ``torch.amp.GradScaler`` integration through
``found_inf``/``inv_scale`` (step skipped on the device, no ``.item()``), and optional
reduced-precision params (``reduced_precision_dtype``) with fp32 master copies; the 16-bit
params are re-written by the same apply kernel (5-list launch).
"""
from __future__ import annotations

from collections import abc as container_abcs
from collections import defaultdict
from copy import deepcopy
from itertools import chain

import torch

from ..multi_tensor_apply import multi_tensor_applier, multi_tensor_applier_l2norm
from ..ops import amp_C
from ._common import first_device, grad_like_param, noop_buffer


class FusedMixedPrecisionLamb(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, step=0, bias_correction=True, betas=(0.9, 0.999), eps=1e-6,
                 weight_decay=0.01, amsgrad=False, adam_w_mode=True, grad_averaging=True,
                 max_grad_norm=1.0, use_nvlamb=False, reduced_precision_dtype=None):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=torch.tensor(lr, dtype=torch.float32), step=torch.tensor([step], dtype=torch.int),
                        bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        device = first_device(self.param_groups)
        for group in self.param_groups:
            for item in ("lr", "step"):
                group[item] = group[item].to(device=device)
        self.multi_tensor_l2norm = amp_C.multi_tensor_l2norm_mp
        self.multi_tensor_lamb = amp_C.multi_tensor_lamb_mp
        self._dummy_overflow_buf = noop_buffer(device)
        self.reduced_precision_dtype = reduced_precision_dtype
        self.param_groups_full_precision = []
        self._step_supports_amp_scaling = True
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.use_nvlamb = use_nvlamb

    def load_state_dict(self, state_dict):
        state_dict = deepcopy(state_dict)
        groups = self.param_groups
        saved_groups = state_dict["param_groups"]
        if len(groups) != len(saved_groups):
            raise ValueError("loaded state dict has a different number of parameter groups")
        if any(len(g["params"]) != len(s["params"]) for g, s in zip(groups, saved_groups)):
            raise ValueError("loaded state dict contains a parameter group that doesn't match the size of optimizer's group")
        id_map = {old: p for old, p in zip(chain.from_iterable(g["params"] for g in saved_groups),
                                           chain.from_iterable(g["params"] for g in groups))}

        def cast(param, value):
            # keep fp32 state fp32 even for reduced-precision params; move to the param's device
            if isinstance(value, torch.Tensor):
                return value.to(param.device)
            if isinstance(value, dict):
                return {k: cast(param, v) for k, v in value.items()}
            if isinstance(value, container_abcs.Iterable) and not isinstance(value, str):
                return type(value)(cast(param, v) for v in value)
            return value

        state = defaultdict(dict)
        for k, v in state_dict["state"].items():
            if k in id_map:
                state[id_map[k]] = cast(id_map[k], v)
            else:
                state[k] = v
        dev = first_device(groups)
        new_groups = []
        for g, ng in zip(groups, saved_groups):
            ng["params"] = g["params"]
            for item in ("lr", "step"):
                if isinstance(ng.get(item), torch.Tensor):
                    ng[item] = ng[item].to(dev)
            new_groups.append(ng)
        self.__setstate__({"state": state, "param_groups": new_groups})

    def _setup_full_precision_params(self):
        for pg in self.param_groups:
            self.param_groups_full_precision.append({
                "params": [p.clone().detach().float()
                           if self.reduced_precision_dtype is not None and p.dtype == self.reduced_precision_dtype
                           else None for p in pg["params"]]
            })

    def add_param_group(self, param_group):
        super().add_param_group(param_group)
        for name, default in self.defaults.items():
            if isinstance(default, torch.Tensor):
                self.param_groups[-1][name] = default.clone().to(first_device(self.param_groups))

    @torch.no_grad()
    def step(self, closure=None, grad_scaler=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups_full_precision) == 0:
            self._setup_full_precision_params()
        grad_list = []
        for group in self.param_groups:
            for p in group["params"]:
                assert group["params"][0].dtype == p.dtype, "Error: Parameters are not of the identical type"
                if p.grad is not None:
                    grad_list.append(p.grad)
        device = first_device(self.param_groups)
        found_inf = (grad_scaler._check_inf_per_device(self)[device] if grad_scaler is not None
                     else torch.zeros((1,), device=device))
        self._dummy_overflow_buf.copy_(found_inf)
        if grad_scaler is not None:
            scale = grad_scaler._get_scale_async()
            inv_scale = scale.double().reciprocal().float()
        else:
            scale = torch.ones((1,), device=device)
            inv_scale = torch.ones((1,), device=device)
        max_grad_norm = self.defaults["max_grad_norm"] * scale
        by_dtype = {}
        for g in grad_list:
            by_dtype.setdefault(g.dtype, []).append(g)
        norms = [multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [gl], False)[0]
                 for gl in by_dtype.values()]
        if len(norms) > 1:
            grad_norm = multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [norms], False)[0]
        else:
            grad_norm = norms[0] if norms else torch.zeros(1, device=device)

        for group, group_full in zip(self.param_groups, self.param_groups_full_precision):
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] += (self._dummy_overflow_buf != 1).to(torch.int)
            lists = [[], [], [], []]
            if self.reduced_precision_dtype is not None:
                lists.append([])
            for p, p_full in zip(group["params"], group_full["params"]):
                if p.grad is None:
                    continue
                assert not p.grad.is_sparse
                state = self.state[p]
                if len(state) == 0:
                    dtype = p.dtype
                    if self.reduced_precision_dtype is not None and p.dtype == self.reduced_precision_dtype:
                        dtype = torch.float32
                    state["exp_avg"] = torch.zeros_like(p, dtype=dtype)
                    state["exp_avg_sq"] = torch.zeros_like(p, dtype=dtype)
                lists[0].append(grad_like_param(p))
                if self.reduced_precision_dtype is not None:
                    lists[1].append(p_full if p_full is not None else p)
                    lists[4].append(p)
                else:
                    lists[1].append(p)
                lists[2].append(state["exp_avg"])
                lists[3].append(state["exp_avg_sq"])
            if not lists[0]:
                continue
            multi_tensor_applier(self.multi_tensor_lamb, self._dummy_overflow_buf, lists, group["lr"], beta1,
                                 beta2, group["eps"], group["step"], bias_correction, group["weight_decay"],
                                 grad_averaging, self.adam_w_mode, grad_norm, max_grad_norm, self.use_nvlamb,
                                 found_inf, inv_scale)
        return loss
