"""FusedLAMB (reference: apex/optimizers/fused_lamb.py:4-215).

Global gradient norm over fp32 and 16-bit gradients (one deterministic multi-tensor norm per
dtype, blended on the device -- no host sync), then the LAMB update as two streaming kernels
(``multi_tensor_lamb``: moments + fused param/update norms, then the trust-ratio apply). bf16
gradients are accepted (the reference raises).
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import multi_tensor_applier, multi_tensor_applier_l2norm
from ..ops import amp_C
from ._common import ParamTableMixin, first_device, grad_like_param, noop_buffer, zero_grad


class FusedLAMB(ParamTableMixin, torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-6,
                 weight_decay=0.01, amsgrad=False, adam_w_mode=True, grad_averaging=True,
                 set_grad_none=True, max_grad_norm=1.0, use_nvlamb=False):
        if amsgrad:
            raise RuntimeError("FusedLAMB does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay, grad_averaging=grad_averaging,
                        max_grad_norm=max_grad_norm)
        super().__init__(params, defaults)
        self.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
        self.multi_tensor_lamb = amp_C.multi_tensor_lamb
        self._dummy_overflow_buf = noop_buffer(first_device(self.param_groups))
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self.use_nvlamb = use_nvlamb

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    def _global_grad_norm(self, device):
        by_dtype = {}
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.dtype not in (torch.float32, torch.float16, torch.bfloat16):
                    raise RuntimeError("FusedLAMB only support fp16, bfloat16 and fp32.")
                by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
        norms = [multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [gl], False)[0]
                 for gl in by_dtype.values()]
        if not norms:
            return torch.zeros(1, device=device)
        if len(norms) == 1:
            return norms[0]
        return multi_tensor_applier_l2norm(self.multi_tensor_l2norm, self._dummy_overflow_buf, [norms], False)[0]

    def _native_step(self, amp_models=None, inv_scale=None, scaled_norm=None):
        """GPU step through the native parameter table: one host call for the global norm and every
        group's LAMB launches (same kernels and semantics as the list path below).

        ``amp_models`` ({id(master): 16-bit model param}) is amp O2's fused mixed-precision step: the
        gradients are read from the model parameters, unscaled by the device ``inv_scale`` inside the
        kernels, and stage 2 writes the model parameters (reference: csrc/multi_tensor_lamb_mp.cu:41,
        248,367). ``scaled_norm`` is the norm of those scaled gradients if amp already computed it."""
        hyper = []
        for group in self.param_groups:
            group["step"] = group.get("step", 0) + 1
            beta1, beta2 = group["betas"]
            hyper.append([float(group["lr"]), beta1, beta2, group["eps"], group["step"],
                          1 if group["bias_correction"] else 0, group["weight_decay"],
                          1 if group["grad_averaging"] else 0])
        steps = self._device_step_counters()
        keys = ("exp_avg", "exp_avg_sq")
        args = (self._dummy_overflow_buf, hyper, self.adam_w_mode, self.defaults["max_grad_norm"], self.use_nvlamb,
                steps, inv_scale, scaled_norm)

        def table():
            return self._native_table(keys) if amp_models is None else self._amp_native_table(keys, amp_models)

        if not table().lamb_step(*args):
            for group in self.param_groups:
                for p in group["params"]:
                    src = p if amp_models is None else amp_models.get(id(p), p)
                    if src.grad is not None and "exp_avg" not in self.state[p]:
                        self.state[p]["exp_avg"] = torch.zeros_like(p)
                        self.state[p]["exp_avg_sq"] = torch.zeros_like(p)
            self._reset_tables()
            if not table().lamb_step(*args):
                raise RuntimeError("FusedLAMB: optimizer state missing after initialisation")

    def _amp_fused_ok(self):
        return self._fast_path_ok()

    def _amp_fused_step(self, models, inv_scale, scaled_norm):
        self._native_step(models, inv_scale, scaled_norm)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self._fast_path_ok():
            self._native_step()
            return loss
        if getattr(self, "_device_step", False) and bool(self._dummy_overflow_buf.item()):
            # device-scaled amp on the list path (no parameter table): the kernels would no-op on the
            # flag, but the host step counters below must not advance for a skipped step either
            return loss
        device = first_device(self.param_groups)
        global_grad_norm = self._global_grad_norm(device)
        max_grad_norm = self.defaults["max_grad_norm"]

        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            grad_averaging = 1 if group["grad_averaging"] else 0
            group["step"] = group.get("step", 0) + 1
            buckets = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedLAMB does not support sparse gradients, please consider SparseAdam instead")
                state = self.state[p]
                if len(state) == 0:
                    state["exp_avg"] = torch.zeros_like(p)
                    state["exp_avg_sq"] = torch.zeros_like(p)
                lists = buckets.setdefault((p.dtype, p.grad.dtype), [[], [], [], []])
                lists[0].append(grad_like_param(p))
                lists[1].append(p)
                lists[2].append(state["exp_avg"])
                lists[3].append(state["exp_avg_sq"])
            for lists in buckets.values():
                multi_tensor_applier(self.multi_tensor_lamb, self._dummy_overflow_buf, lists, group["lr"],
                                     beta1, beta2, group["eps"], group["step"], bias_correction,
                                     group["weight_decay"], grad_averaging, self.adam_w_mode,
                                     global_grad_norm, max_grad_norm, self.use_nvlamb)
        return loss
