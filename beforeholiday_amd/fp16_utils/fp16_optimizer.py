"""FP16_Optimizer: the legacy master-weight wrapper (API of /root/reference/apex/fp16_utils/fp16_optimizer.py).

Any optimizer over 16-bit parameters: the wrapped optimizer sees fp32 master copies, ``backward(loss)``
scales the loss, ``update_master_grads`` unscales the 16-bit gradients into the master gradients (one
multi-tensor launch per dtype with an overflow flag, amp/scaler.py) and ``step`` writes the masters
back into the model. ``state_dict`` keeps the reference checkpoint keys.

Layout here: each param group is split once into a :class:`_Split` (16-bit model params, their
masters, plain fp32 params), and every later operation walks those splits.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List

import torch

from ..amp._amp_state import maybe_print
from ..amp.scaler import LossScaler
from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C

_LOW = (torch.float16, torch.bfloat16)


@dataclass
class _Split:
    model: List[torch.Tensor] = field(default_factory=list)    # 16-bit params the model computes with
    master: List[torch.Tensor] = field(default_factory=list)   # their fp32 masters (what the optimizer updates)
    fp32: List[torch.Tensor] = field(default_factory=list)     # fp32 params, updated in place


def _split_group(group, opt_state) -> _Split:
    """Replace the group's 16-bit params by fp32 masters (moving any optimizer state over)."""
    s = _Split()
    params = group["params"]
    for i, p in enumerate(params):
        if not p.requires_grad:
            continue
        if p.dtype in _LOW:
            m = p.detach().clone().float().requires_grad_(True)
            params[i] = m
            if p in opt_state:
                opt_state[m] = opt_state.pop(p)
            s.model.append(p)
            s.master.append(m)
        elif p.dtype == torch.float32:
            s.fp32.append(p)
        else:
            raise TypeError(f"FP16_Optimizer wraps float32 / float16 / bfloat16 parameters, got {p.type()}")
    return s


class _Inner:
    """Attribute of the wrapped optimizer exposed (read / write) on the wrapper."""

    def __init__(self, name):
        self.name = name

    def __get__(self, obj, cls=None):
        return self if obj is None else getattr(obj.optimizer, self.name)

    def __set__(self, obj, value):
        setattr(obj.optimizer, self.name, value)


class FP16_Optimizer(object):
    state = _Inner("state")
    param_groups = _Inner("param_groups")

    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False, dynamic_loss_args=None,
                 verbose=True):
        self.verbose = verbose
        self.optimizer = init_optimizer
        self._splits = [_split_group(g, init_optimizer.state) for g in init_optimizer.param_groups]
        # re-key the optimizer's per-param state structures on the new master tensors
        init_optimizer.load_state_dict(init_optimizer.state_dict())
        any_p = [p for s in self._splits for p in s.model + s.fp32]
        dev = any_p[0].device if any_p else torch.device("cpu")
        self.dynamic_loss_scale = bool(dynamic_loss_scale)
        self.loss_scaler = (LossScaler("dynamic", device=dev, **(dynamic_loss_args or {})) if dynamic_loss_scale
                            else LossScaler(static_loss_scale, device=dev))
        self.overflow = False
        self.first_closure_call_this_step = True
        self.clip_grad_norm = torch.nn.utils.clip_grad_norm_
        self.multi_tensor_scale = amp_C.multi_tensor_scale
        self._dummy_overflow_buf = torch.zeros(1, dtype=torch.int, device=dev)

    # reference attribute names (read by user code and by the checkpoint format)
    fp16_groups = property(lambda self: [s.model for s in self._splits])
    fp32_from_fp16_groups = property(lambda self: [s.master for s in self._splits])
    fp32_from_fp32_groups = property(lambda self: [s.fp32 for s in self._splits])
    all_fp16_params = property(lambda self: [p for s in self._splits for p in s.model])
    all_fp32_from_fp16_params = property(lambda self: [p for s in self._splits for p in s.master])
    all_fp32_from_fp32_params = property(lambda self: [p for s in self._splits for p in s.fp32])

    def maybe_print(self, msg):
        if self.verbose:
            print(msg)

    def __getstate__(self):
        raise RuntimeError("pickling FP16_Optimizer is not supported: save state_dict() instead")

    def __setstate__(self, state):
        raise RuntimeError("unpickling FP16_Optimizer is not supported: use load_state_dict()")

    # ---- gradients -------------------------------------------------------------------------------

    def zero_grad(self, set_grads_to_None=False):
        from ..optimizers._common import zero_param_grads

        zero_param_grads([p for g in self.optimizer.param_groups for p in g["params"]] + self.all_fp16_params,
                         set_grads_to_None)

    def backward(self, loss, update_master_grads=True, retain_graph=False):
        (loss.float() * self.loss_scaler.loss_scale()).backward(retain_graph=retain_graph)
        if update_master_grads:
            self.update_master_grads()

    def update_master_grads(self):
        """Unscale into the masters' gradients and update the loss scale; sets ``self.overflow``."""
        sc = self.loss_scaler
        sc.clear_overflow_state()
        src, dst = [], []
        for s in self._splits:
            for p, m in zip(s.model, s.master):
                if p.grad is None:
                    continue
                if m.grad is None:
                    m.grad = torch.empty_like(m)
                src.append(p.grad)
                dst.append(m.grad)
        if src:
            sc.unscale(src, dst, sc.loss_scale())
        own = [p.grad for s in self._splits for p in s.fp32 if p.grad is not None]
        if own:
            sc.unscale(own, own, sc.loss_scale())
        self.overflow = sc.update_scale()

    def clip_master_grads(self, max_norm, norm_type=2):
        """Clip the fp32 gradients the optimizer will use; -1 (and nothing clipped) after an overflow."""
        if self.overflow:
            return -1
        return self.clip_grad_norm([p for g in self.optimizer.param_groups for p in g["params"]], max_norm, norm_type)

    def inspect_master_grad_data(self):
        if self.overflow:
            print("FP16_Optimizer.inspect_master_grad_data: the last backward overflowed, master gradients are not "
                  "valid; returning None")
            return None
        return [[p.grad.data if p.grad is not None else None for p in g["params"]]
                for g in self.optimizer.param_groups]

    # ---- step ------------------------------------------------------------------------------------

    def _master_params_to_model_params(self):
        by_dtype = {}
        for s in self._splits:
            for p, m in zip(s.model, s.master):
                src, dst = by_dtype.setdefault(p.dtype, ([], []))
                src.append(m.data)
                dst.append(p.data)
        for src, dst in by_dtype.values():
            multi_tensor_applier(self.multi_tensor_scale, self._dummy_overflow_buf, [src, dst], 1.0)

    def step(self, closure=None):
        if self.overflow:
            maybe_print(f"FP16_Optimizer: gradient overflow, step skipped; loss scale is now "
                        f"{self.loss_scaler.loss_scale()}")
            return None
        out = self.optimizer.step() if closure is None else self._closure_step(closure)
        self._master_params_to_model_params()
        return out

    def _closure_step(self, closure):
        """The wrapped optimizer may call the closure several times (e.g. LBFGS): every call after the
        first re-publishes the masters first, and a call whose backward overflowed is repeated at the
        reduced scale."""

        def evaluate():
            if self.first_closure_call_this_step:
                self.first_closure_call_this_step = False
            else:
                self._master_params_to_model_params()
            loss = closure()
            while self.overflow:
                self.maybe_print(f"FP16_Optimizer: overflow inside the closure, re-evaluating at loss scale "
                                 f"{self.loss_scaler.loss_scale()}")
                loss = closure()
            return loss

        try:
            return self.optimizer.step(evaluate)
        finally:
            self.first_closure_call_this_step = True

    # ---- checkpointing ---------------------------------------------------------------------------

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
        for k in ("loss_scaler", "dynamic_loss_scale", "overflow", "first_closure_call_this_step"):
            setattr(self, k, state_dict[k])
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        # the masters are restored from the saved fp32 copies (exact), not re-derived from 16-bit params
        for s, saved in zip(self._splits, state_dict["fp32_from_fp16"]):
            for m, v in zip(s.master, saved):
                m.data.copy_(v.data)

    @property
    def loss_scale(self):
        return self.loss_scaler.loss_scale()

    @loss_scale.setter
    def loss_scale(self, value):
        self.loss_scaler._loss_scale = value
