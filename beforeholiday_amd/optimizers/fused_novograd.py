"""FusedNovoGrad (reference: apex/optimizers/fused_novograd.py:4-214).

Per-tensor second-moment *norms* (L2 or L-inf) live in ``group['exp_avg_sq']`` (one fp32 vector
per dtype bucket) and are blended on the device by the norm_out stage of the native op.
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._common import first_device, grad_like_param, noop_buffer, zero_grad


class FusedNovoGrad(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.0, amsgrad=False, reg_inside_moment=False, grad_averaging=True,
                 norm_type=2, init_zero=False, set_grad_none=True):
        if amsgrad:
            raise RuntimeError("FusedNovoGrad does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, grad_averaging=grad_averaging, norm_type=norm_type,
                        init_zero=init_zero)
        super().__init__(params, defaults)
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.multi_tensor_novograd = amp_C.multi_tensor_novograd
        self.moment_mode = 0 if reg_inside_moment else 1
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for group in self.param_groups:
            if len(group["params"]) > 0 and "exp_avg_sq" in group:
                dev = group["params"][0].device
                group["exp_avg_sq"] = [t.to(dev) if t is not None else None for t in group["exp_avg_sq"]]

    @staticmethod
    def _init_norms(gs, norm_type, dev):
        if norm_type == 0:
            v = [g.float().abs().max() for g in gs]
        elif norm_type == 2:
            v = [g.float().pow(2).sum().sqrt() for g in gs]
        else:
            raise RuntimeError("FusedNovoGrad only support l2/inf norm now.")
        return torch.stack(v).to(dev) if v else torch.zeros(0, device=dev)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        dev = first_device(self.param_groups)
        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] = group.get("step", 0) + 1
            g_16, p_16, m_16, g_32, p_32, m_32 = [], [], [], [], [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedNovoGrad does not support sparse gradients, please consider SparseAdam instead")
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p)
                if p.dtype in (torch.float16, torch.bfloat16):
                    g_16.append(grad_like_param(p)), p_16.append(p), m_16.append(state["exp_avg"])
                elif p.dtype == torch.float32:
                    g_32.append(grad_like_param(p)), p_32.append(p), m_32.append(state["exp_avg"])
                else:
                    raise RuntimeError("FusedNovoGrad only support fp16, bfloat16 and fp32.")
            if "exp_avg_sq" not in group:
                if group["init_zero"]:
                    group["exp_avg_sq"] = [torch.zeros(len(g_16), device=dev), torch.zeros(len(g_32), device=dev)]
                else:  # init with the first step's norm so the first blend is a no-op
                    group["exp_avg_sq"] = [self._init_norms(g_16, group["norm_type"], dev),
                                           self._init_norms(g_32, group["norm_type"], dev)]
            else:
                assert len(g_16) == group["exp_avg_sq"][0].numel()
                assert len(g_32) == group["exp_avg_sq"][1].numel()
            for lists, norms in (([g_16, p_16, m_16], group["exp_avg_sq"][0]),
                                 ([g_32, p_32, m_32], group["exp_avg_sq"][1])):
                if not lists[0]:
                    continue
                if lists[1][0].dtype != lists[1][-1].dtype or any(x.dtype != lists[1][0].dtype for x in lists[1]):
                    raise RuntimeError("FusedNovoGrad: mixed fp16/bf16 params in one group are not supported")
                multi_tensor_applier(self.multi_tensor_novograd, self._dummy_overflow_buf, lists, norms,
                                     group["lr"], beta1, beta2, group["eps"], group["step"], bias_correction,
                                     group["weight_decay"], grad_averaging, self.moment_mode,
                                     group["norm_type"])
        return loss
