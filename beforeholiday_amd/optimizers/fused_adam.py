"""FusedAdam (reference: apex/optimizers/fused_adam.py:4-193).

Same constructor and semantics as the reference; differences by design:
* bf16 parameters get their own launch (the reference's bf16 branch is unreachable);
* ``capturable=True`` keeps lr/step on the device (no host scalars in the launch, so the whole
  optimizer step can be captured in a HIP graph), and accepts a ``grad_scaler`` for a fused,
  sync-free unscale + inf-skip;
* ``master_weights=True`` keeps fp32 master copies of 16-bit params and writes the 16-bit params
  back inside the same kernel (5-list launch) instead of a separate copy pass.
"""
from __future__ import annotations

import torch

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C
from ._common import ParamTableMixin, first_device, grad_like_param, noop_buffer, zero_grad


class FusedAdam(ParamTableMixin, torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, bias_correction=True, betas=(0.9, 0.999), eps=1e-8,
                 adam_w_mode=True, weight_decay=0.0, amsgrad=False, set_grad_none=True,
                 capturable=False, master_weights=False):
        if amsgrad:
            raise RuntimeError("FusedAdam does not support the AMSGrad variant.")
        defaults = dict(lr=lr, bias_correction=bias_correction, betas=betas, eps=eps,
                        weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.adam_w_mode = 1 if adam_w_mode else 0
        self.set_grad_none = set_grad_none
        self.capturable = capturable
        self.master_weights = master_weights
        dev = first_device(self.param_groups)
        self._dummy_overflow_buf = noop_buffer(dev)
        self.multi_tensor_adam = amp_C.multi_tensor_adam
        if capturable:
            for group in self.param_groups:
                group["lr"] = torch.tensor(float(group["lr"]), dtype=torch.float32, device=dev)
                group["step"] = torch.zeros(1, dtype=torch.int, device=dev)

    def zero_grad(self, set_to_none=None):
        zero_grad(self, self.set_grad_none, set_to_none)

    def _master(self, p):
        st = self.state[p]
        if "master_param" not in st:
            st["master_param"] = p.detach().float().clone()
        return st["master_param"]

    def _init_state(self, p):
        state = self.state[p]
        use_master = self.master_weights and p.dtype in (torch.float16, torch.bfloat16)
        target = self._master(p) if use_master else p
        if "exp_avg" not in state:
            # 16-bit params keep fp32 moments: an fp16 exp_avg_sq underflows to 0 for
            # |g| < 8e-3 and the update then blows up to inf (the reference stores them in
            # the param dtype); the kernel reads/writes fp32 state natively.
            sdt = torch.float32 if target.dtype in (torch.float16, torch.bfloat16) else target.dtype
            state["exp_avg"] = torch.zeros_like(target, dtype=sdt)
            state["exp_avg_sq"] = torch.zeros_like(target, dtype=sdt)
        return state, use_master, target

    def _native_step(self, amp_models=None, inv_scale=None):
        """GPU step through the native parameter table (one host call for every group's launches).
        ``amp_models`` ({id(master): 16-bit model param}): amp O2 / O5's fused step -- the fp32
        masters (this optimizer's parameters) are updated from the model parameters' 16-bit
        gradients times the device ``inv_scale`` and the model parameters are written in the same
        launch (no fp32 master gradient, no separate master-to-model copy)."""
        hyper = []
        for group in self.param_groups:
            group["step"] = group.get("step", 0) + 1
            beta1, beta2 = group["betas"]
            hyper.append([float(group["lr"]), beta1, beta2, group["eps"], group["step"],
                          1 if group["bias_correction"] else 0, group["weight_decay"]])
        master = "master_param" if self.master_weights else None
        keys = ("exp_avg", "exp_avg_sq")
        args = (self._dummy_overflow_buf, hyper, self.adam_w_mode, self._device_step_counters(), inv_scale)

        def table():
            if amp_models is None:
                return self._native_table(keys, master)
            return self._amp_native_table(keys, amp_models)

        if not table().adam_step(*args):
            for group in self.param_groups:
                for p in group["params"]:
                    src = p if amp_models is None else amp_models.get(id(p), p)
                    if src.grad is not None:
                        self._init_state(p)
            self._reset_tables()
            if not table().adam_step(*args):
                raise RuntimeError("FusedAdam: optimizer state missing after initialisation")

    def _amp_fused_ok(self):
        return not self.capturable and not self.master_weights and self._fast_path_ok()

    def _amp_fused_step(self, models, inv_scale, scaled_norm):
        self._native_step(models, inv_scale)

    @torch.no_grad()
    def step(self, closure=None, grads=None, output_params=None, scale=None, grad_norms=None,
             grad_scaler=None):
        if any(x is not None for x in (grads, output_params, scale, grad_norms)):
            raise RuntimeError("FusedAdam has been updated. Simply initialize it identically to "
                               "torch.optim.Adam, and call step() with no arguments.")
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self.capturable and grad_scaler is None and self._fast_path_ok():
            self._native_step()
            return loss
        if getattr(self, "_device_step", False) and bool(self._dummy_overflow_buf.item()):
            # device-scaled amp on the list path: the list kernels do not read the flag, and the host
            # step counters must not advance for a skipped step either
            return loss
        inv_scale = found_inf = None
        if grad_scaler is not None:
            if not self.capturable:
                raise RuntimeError("grad_scaler integration requires capturable=True")
            dev = first_device(self.param_groups)
            found_inf = grad_scaler._check_inf_per_device(self)[dev]
            inv_scale = grad_scaler._get_scale_async().double().reciprocal().float()

        for group in self.param_groups:
            bias_correction = 1 if group["bias_correction"] else 0
            beta1, beta2 = group["betas"]
            if self.capturable:
                if found_inf is not None:
                    group["step"] += (found_inf == 0).to(torch.int)
                else:
                    group["step"] += 1
            else:
                group["step"] = group.get("step", 0) + 1

            buckets = {}  # (param dtype, state dtype, copy) -> lists
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients, please consider SparseAdam instead")
                if p.dtype not in (torch.float16, torch.bfloat16, torch.float32, torch.float64):
                    raise RuntimeError("FusedAdam only support fp16, bfloat16, fp32 and fp64.")
                state, use_master, target = self._init_state(p)
                g = grad_like_param(p)
                key = (target.dtype, state["exp_avg"].dtype, use_master)
                lists = buckets.setdefault(key, [[], [], [], [], []])
                lists[0].append(g)
                lists[1].append(target)
                lists[2].append(state["exp_avg"])
                lists[3].append(state["exp_avg_sq"])
                lists[4].append(p)
            for (dt, sdt, use_master), lists in buckets.items():
                if not use_master:
                    lists = lists[:4]
                if self.capturable:
                    amp_C.multi_tensor_adam_capturable(
                        multi_tensor_applier.chunk_size, self._dummy_overflow_buf, lists, group["lr"],
                        beta1, beta2, group["eps"], group["step"], self.adam_w_mode, bias_correction,
                        group["weight_decay"], inv_scale, found_inf)
                else:
                    multi_tensor_applier(self.multi_tensor_adam, self._dummy_overflow_buf, lists,
                                         group["lr"], beta1, beta2, group["eps"], group["step"],
                                         self.adam_w_mode, bias_correction, group["weight_decay"])
        return loss
