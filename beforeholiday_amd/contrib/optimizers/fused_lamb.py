"""contrib FusedLAMB: the deprecated contrib optimizer (reference: apex/contrib/optimizers/fused_lamb.py:6-208)
with its own semantics, which differ from :class:`beforeholiday_amd.optimizers.FusedLAMB` in three ways the
reference's users can observe:

* only fp32 and fp16 parameters (bf16 raises, as the reference's ``fused_lamb_cuda`` extension does);
* one ``max_grad_norm`` for the whole optimizer, read from ``defaults`` (not per group), and the global
  gradient norm blended from ONE fp32 and ONE fp16 list norm, sqrt(n32^2 + n16^2);
* the fp16 and fp32 parameters of a group update in separate launches (two lists, as the reference).

The reference reads both list norms to the host (``.item()``) and blends them there; here the blend stays on
the device and the fused LAMB kernels (kernels/multi_tensor.hip stage 1 / stage 2) read the norm from device
memory, so a step never synchronises the host."""
from __future__ import annotations

import torch

from ...multi_tensor_apply import multi_tensor_applier, multi_tensor_applier_l2norm
from ...ops import amp_C
from ...optimizers._common import first_device, noop_buffer, zero_grad

__all__ = ["FusedLAMB"]


class FusedLAMB(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01,
                 amsgrad=False, adam_w_mode=True, grad_averaging=True, set_grad_none=True, max_grad_norm=1.0):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps, weight_decay=weight_decay,
                        grad_averaging=grad_averaging, max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
        self.multi_tensor_lamb = amp_C.multi_tensor_lamb
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    @staticmethod
    def _check_dtype(p):
        if p.dtype not in (torch.float32, torch.float16):
            raise RuntimeError("FusedLAMB only support fp16 and fp32.")

    def _global_grad_norm(self, device):
        g32, g16 = [], []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                self._check_dtype(p)
                (g32 if p.dtype == torch.float32 else g16).append(p.grad)
        zero = torch.zeros(1, device=device, dtype=torch.float32)
        n32 = multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [g32], False)[0] \
            if g32 else zero
        n16 = multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [g16], False)[0] \
            if g16 else zero
        return torch.sqrt(n32.float() * n32.float() + n16.float() * n16.float()).reshape(1)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        device = first_device(self.param_groups)
        global_grad_norm = self._global_grad_norm(device)
        max_grad_norm = self.defaults["max_grad_norm"]
        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] = group.get("step", 0) + 1  # one step count per group, as the reference
            lists = {torch.float16: ([], [], [], []), torch.float32: ([], [], [], [])}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedLAMB does not support sparse gradients, please consider SparseAdam instead")
                self._check_dtype(p)
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                g, w, m, v = lists[p.dtype]
                g.append(p.grad)
                w.append(p)
                m.append(state["exp_avg"])
                v.append(state["exp_avg_sq"])
            for dt in (torch.float16, torch.float32):  # the reference's launch order
                if lists[dt][0]:
                    multi_tensor_applier(self.multi_tensor_lamb, self._dummy_overflow_buf, list(lists[dt]),
                                         group["lr"], beta1, beta2, group["eps"], group["step"], bias_correction,
                                         group["weight_decay"], grad_averaging, self.adam_w_mode, global_grad_norm,
                                         max_grad_norm)
        return loss
