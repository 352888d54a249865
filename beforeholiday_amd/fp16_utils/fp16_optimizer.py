"""FP16_Optimizer: legacy master-weight wrapper (reference: apex/fp16_utils/fp16_optimizer.py:13-554).

Wraps any optimizer over 16-bit params: fp32 masters are what the inner optimizer updates,
``backward(loss)`` scales the loss, ``update_master_grads`` unscales fp16 grads into the fp32
master grads (one multi-tensor launch with an overflow flag) and ``step`` copies masters back.
State dict keys match the reference checkpoint format.
"""
from __future__ import annotations

import torch

from ..amp._amp_state import maybe_print
from ..amp.scaler import LossScaler
from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C

_LOW = (torch.float16, torch.bfloat16)


class FP16_Optimizer(object):
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 verbose=True):
        self.verbose = verbose
        self.optimizer = init_optimizer
        self.fp16_groups, self.fp32_from_fp16_groups, self.fp32_from_fp32_groups = [], [], []
        for param_group in self.optimizer.param_groups:
            fp16_this, fp32_from_fp16_this, fp32_this = [], [], []
            for i, param in enumerate(param_group["params"]):
                if not param.requires_grad:
                    continue
                if param.dtype in _LOW:
                    fp16_this.append(param)
                    master = param.detach().clone().float()
                    master.requires_grad = True
                    param_group["params"][i] = master
                    fp32_from_fp16_this.append(master)
                    if param in self.optimizer.state:
                        self.optimizer.state[master] = self.optimizer.state.pop(param)
                elif param.dtype == torch.float32:
                    fp32_this.append(param)
                    param_group["params"][i] = param
                else:
                    raise TypeError("Wrapped parameters must be float32, float16 or bfloat16. Received {}"
                                    .format(param.type()))
            self.fp16_groups.append(fp16_this)
            self.fp32_from_fp16_groups.append(fp32_from_fp16_this)
            self.fp32_from_fp32_groups.append(fp32_this)
        self.all_fp16_params = [p for g in self.fp16_groups for p in g]
        self.all_fp32_from_fp16_params = [p for g in self.fp32_from_fp16_groups for p in g]
        self.all_fp32_from_fp32_params = [p for g in self.fp32_from_fp32_groups for p in g]
        self.optimizer.load_state_dict(self.optimizer.state_dict())
        dev = (self.all_fp16_params + self.all_fp32_from_fp32_params)[0].device if \
            (self.all_fp16_params or self.all_fp32_from_fp32_params) else torch.device("cpu")
        if dynamic_loss_scale:
            self.dynamic_loss_scale = True
            self.loss_scaler = LossScaler("dynamic", device=dev, **(dynamic_loss_args or {}))
        else:
            self.dynamic_loss_scale = False
            self.loss_scaler = LossScaler(static_loss_scale, device=dev)
        self.overflow = False
        self.first_closure_call_this_step = True
        self.clip_grad_norm = torch.nn.utils.clip_grad_norm_
        self.multi_tensor_scale = amp_C.multi_tensor_scale
        self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int, device=dev)

    def maybe_print(self, msg):
        if self.verbose:
            print(msg)

    def __getstate__(self):
        raise RuntimeError("FP16_Optimizer should be serialized using state_dict().")

    def __setstate__(self, state):
        raise RuntimeError("FP16_Optimizer should be deserialized using load_state_dict().")

    def zero_grad(self, set_grads_to_None=False):
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                if set_grads_to_None:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.detach_()
                    p.grad.zero_()
        for fp16_group in self.fp16_groups:
            for param in fp16_group:
                if set_grads_to_None:
                    param.grad = None
                elif param.grad is not None:
                    param.grad.detach_()
                    param.grad.zero_()

    def _master_params_to_model_params(self):
        groups = {}
        for master, model in zip(self.all_fp32_from_fp16_params, self.all_fp16_params):
            groups.setdefault(model.dtype, ([], []))
            groups[model.dtype][0].append(master.data)
            groups[model.dtype][1].append(model.data)
        for masters, models in groups.values():
            multi_tensor_applier(self.multi_tensor_scale, self._dummy_overflow_buf, [masters, models], 1.0)

    def clip_master_grads(self, max_norm, norm_type=2):
        if not self.overflow:
            fp32_params = [p for g in self.optimizer.param_groups for p in g["params"]]
            return self.clip_grad_norm(fp32_params, max_norm, norm_type)
        return -1

    def state_dict(self):
        return {
            "loss_scaler": self.loss_scaler,
            "dynamic_loss_scale": self.dynamic_loss_scale,
            "overflow": self.overflow,
            "first_closure_call_this_step": self.first_closure_call_this_step,
            "optimizer_state_dict": self.optimizer.state_dict(),
            "fp32_from_fp16": self.fp32_from_fp16_groups,
        }

    def load_state_dict(self, state_dict):
        self.loss_scaler = state_dict["loss_scaler"]
        self.dynamic_loss_scale = state_dict["dynamic_loss_scale"]
        self.overflow = state_dict["overflow"]
        self.first_closure_call_this_step = state_dict["first_closure_call_this_step"]
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        for current_group, saved_group in zip(self.fp32_from_fp16_groups, state_dict["fp32_from_fp16"]):
            for current, saved in zip(current_group, saved_group):
                current.data.copy_(saved.data)

    def step(self, closure=None):
        if self.overflow:
            maybe_print("Gradient overflow.  Skipping step, reducing loss scale to {}".format(
                self.loss_scaler.loss_scale()))
            return
        if closure is not None:
            retval = self._step_with_closure(closure)
        else:
            retval = self.optimizer.step()
        self._master_params_to_model_params()
        return retval

    def _step_with_closure(self, closure):
        def wrapped_closure():
            if self.first_closure_call_this_step:
                self.first_closure_call_this_step = False
            else:
                self._master_params_to_model_params()
            temp_loss = closure()
            while self.overflow:
                scale = self.loss_scaler.loss_scale()
                self.maybe_print("OVERFLOW within closure! Skipping step, reducing loss scale to {}".format(scale))
                temp_loss = closure()
            return temp_loss

        retval = self.optimizer.step(wrapped_closure)
        self.first_closure_call_this_step = True
        return retval

    def backward(self, loss, update_master_grads=True, retain_graph=False):
        scaled_loss = loss.float() * self.loss_scaler.loss_scale()
        scaled_loss.backward(retain_graph=retain_graph)
        if update_master_grads:
            self.update_master_grads()

    def update_master_grads(self):
        self.loss_scaler.clear_overflow_state()
        if self.all_fp16_params:
            model_grads, master_grads = [], []
            for model_param, master_param in zip(self.all_fp16_params, self.all_fp32_from_fp16_params):
                if model_param.grad is not None:
                    model_grads.append(model_param.grad)
                    if master_param.grad is None:
                        master_param.grad = torch.empty_like(master_param)
                    master_grads.append(master_param.grad)
            self.loss_scaler.unscale(model_grads, master_grads, self.loss_scaler.loss_scale())
        if self.all_fp32_from_fp32_params:
            grads = [p.grad for p in self.all_fp32_from_fp32_params if p.grad is not None]
            self.loss_scaler.unscale(grads, grads, self.loss_scaler.loss_scale())
        self.overflow = self.loss_scaler.update_scale()

    def inspect_master_grad_data(self):
        if self.overflow:
            print("Warning:  calling FP16_Optimizer.inspect_master_grad_data while in an overflow state.  "
                  "Gradients are currently invalid (may be inf, nan, or stale).  Returning None.")
            return None
        return [[p.grad.data if p.grad is not None else None for p in g["params"]]
                for g in self.optimizer.param_groups]

    def _get_loss_scale(self):
        return self.loss_scaler.loss_scale()

    def _set_loss_scale(self, value):
        self.loss_scaler._loss_scale = value

    loss_scale = property(_get_loss_scale, _set_loss_scale)

    def _get_state(self):
        return self.optimizer.state

    def _set_state(self, value):
        self.optimizer.state = value

    state = property(_get_state, _set_state)

    def _get_param_groups(self):
        return self.optimizer.param_groups

    def _set_param_groups(self, value):
        self.optimizer.param_groups = value

    param_groups = property(_get_param_groups, _set_param_groups)
