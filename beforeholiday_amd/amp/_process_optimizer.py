"""Optimizer patching for amp (reference: apex/amp/_process_optimizer.py:28-489).

Master weights (O2/O5): 16-bit params are replaced in the optimizer by fp32 masters; after
backward the 16-bit grads are unscaled into fp32 master grads with one multi-tensor launch per
dtype pair, and after ``step`` the masters are copied back into the 16-bit model params (again one
launch). Gradient stashing supports accumulation across several ``scale_loss`` contexts.
"""
from __future__ import annotations

import types

import torch

from ..multi_tensor_apply import multi_tensor_applier
from ..ops import amp_C

_LOW = (torch.float16, torch.bfloat16)


class AmpOptimizerState(object):
    pass


def _check_param_type(param):
    if param.dtype in _LOW or param.dtype == torch.float32:
        return
    raise TypeError("Optimizer's parameters must be one of float32, float16, bfloat16. Received {}"
                    .format(param.type()))


def _master_params_to_model_params(self):
    stash = self._amp_stash
    if len(stash.all_fp16_params) == 0:
        return
    groups = {}
    for master, model in zip(stash.all_fp32_from_fp16_params, stash.all_fp16_params):
        groups.setdefault(model.dtype, ([], []))
        groups[model.dtype][0].append(master.data)
        groups[model.dtype][1].append(model.data)
    for masters, models in groups.values():
        multi_tensor_applier(stash.multi_tensor_scale, stash.dummy_overflow_buf, [masters, models], 1.0)


def lazy_init_with_master_weights(self):
    stash = self._amp_stash
    stash.fp16_groups, stash.fp32_from_fp16_groups, stash.fp32_from_fp32_groups = [], [], []
    for param_group in self.param_groups:
        fp16_this, fp32_this, fp32_from_fp16_this = [], [], []
        for i, param in enumerate(param_group["params"]):
            if not param.requires_grad:
                continue
            _check_param_type(param)
            if param.dtype in _LOW:
                fp16_this.append(param)
                master = param.detach().clone().float()
                master.requires_grad = True
                param_group["params"][i] = master
                fp32_from_fp16_this.append(master)
                if param in self.state:
                    self.state[master] = self.state.pop(param)
            else:
                fp32_this.append(param)
                param_group["params"][i] = param
        stash.fp16_groups.append(fp16_this)
        stash.fp32_from_fp16_groups.append(fp32_from_fp16_this)
        stash.fp32_from_fp32_groups.append(fp32_this)
    stash.all_fp16_params = [p for g in stash.fp16_groups for p in g]
    stash.all_fp32_from_fp16_params = [p for g in stash.fp32_from_fp16_groups for p in g]
    stash.all_fp32_from_fp32_params = [p for g in stash.fp32_from_fp32_groups for p in g]
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_from_fp32_grad_stash = [None for _ in stash.all_fp32_from_fp32_params]
    for param in stash.all_fp32_from_fp16_params:
        param.grad = None
    for param in stash.all_fp32_from_fp32_params:
        param.grad = None
    # re-create optimizer state (e.g. torch.optim momentum) against the new master params
    self.load_state_dict(self.state_dict())


def post_backward_models_are_masters(scaler, params, stashed_grads, scale_override=None):
    if getattr(scaler, "device_mode", False) and scale_override is None:
        # device-resident scale (LossScaler.enable_device_mode): plain unscale without reading it
        need_unscale, keep = [], False
        for i, (param, stashed_grad) in enumerate(zip(params, stashed_grads)):
            if param.grad is None and stashed_grad is not None:
                param.grad = stashed_grad
            elif param.grad is not None and stashed_grad is None:
                need_unscale.append(param.grad)
            elif param.grad is not None and stashed_grad is not None:
                keep = True  # accumulation into stashed grads: the host-scale path below
        if not keep:
            if need_unscale:
                scaler.unscale(need_unscale, need_unscale, None, models_are_masters=True)
            for i in range(len(stashed_grads)):
                stashed_grads[i] = None
            return
    grads_have_scale, stashed_have_scale, out_scale = scaler.loss_scale(), 1.0, 1.0
    # not much to do if scale == 1.0 and static scaling
    if scaler.loss_scale() == 1.0 and not scaler.dynamic:
        for i in range(len(stashed_grads)):
            stashed_grads[i] = None
        return
    if scale_override is not None:
        grads_have_scale, stashed_have_scale, out_scale = scale_override
    need_unscale, need_stash, stashed = [], [], []
    for param, stashed_grad in zip(params, stashed_grads):
        if param.grad is None and stashed_grad is not None:
            param.grad = stashed_grad
        elif param.grad is not None and stashed_grad is None:
            need_unscale.append(param.grad)
        elif param.grad is not None and stashed_grad is not None:
            need_stash.append(param.grad)
            stashed.append(stashed_grad)
    if need_unscale:
        scaler.unscale(need_unscale, need_unscale, None, models_are_masters=True,
                       scale_override=grads_have_scale / out_scale)
    if need_stash:
        scaler.unscale_with_stashed(need_stash, stashed, need_stash,
                                    scale_override=(grads_have_scale, stashed_have_scale, out_scale))
    for i in range(len(stashed_grads)):
        stashed_grads[i] = None


def prepare_backward_with_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    for param in stash.all_fp16_params:
        # fp16 grads never need stashing: they are folded into the fp32 master grads
        param.grad = None
    for i, param in enumerate(stash.all_fp32_from_fp32_params):
        stash.all_fp32_from_fp32_grad_stash[i] = param.grad
        param.grad = None


def post_backward_with_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()
    fp16_unscale, new_fp32, fp16_unscale_stash, preexisting = [], [], [], []
    for fp16_param, fp32_param in zip(stash.all_fp16_params, stash.all_fp32_from_fp16_params):
        if fp16_param.grad is None and fp32_param.grad is not None:
            continue
        elif fp16_param.grad is not None and fp32_param.grad is None:
            fp32_param.grad = torch.empty_like(fp32_param)
            fp16_unscale.append(fp16_param.grad)
            new_fp32.append(fp32_param.grad)
        elif fp16_param.grad is not None and fp32_param.grad is not None:
            fp16_unscale_stash.append(fp16_param.grad)
            preexisting.append(fp32_param.grad)
    if fp16_unscale:
        scaler.unscale(fp16_unscale, new_fp32, None, models_are_masters=False)
    if fp16_unscale_stash:
        scaler.unscale_with_stashed(fp16_unscale_stash, preexisting, preexisting)
    post_backward_models_are_masters(scaler, stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)


def lazy_init_no_master_weights(self):
    stash = self._amp_stash
    stash.all_fp16_params, stash.all_fp32_params = [], []
    for param_group in self.param_groups:
        for param in param_group["params"]:
            _check_param_type(param)
            (stash.all_fp16_params if param.dtype in _LOW else stash.all_fp32_params).append(param)
    stash.all_fp16_grad_stash = [None for _ in stash.all_fp16_params]
    stash.all_fp32_grad_stash = [None for _ in stash.all_fp32_params]


def prepare_backward_no_master_weights(self):
    stash = self._amp_stash
    self._amp_lazy_init()
    for i, param in enumerate(stash.all_fp16_params):
        stash.all_fp16_grad_stash[i] = param.grad
        param.grad = None
    for i, param in enumerate(stash.all_fp32_params):
        stash.all_fp32_grad_stash[i] = param.grad
        param.grad = None


def post_backward_no_master_weights(self, scaler):
    stash = self._amp_stash
    self._amp_lazy_init()
    for params, stashed in ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                            (stash.all_fp32_params, stash.all_fp32_grad_stash)):
        post_backward_models_are_masters(scaler, params, stashed)


# FusedSGD can fold the unscale into its own kernel (materialize_master_grads=False)
def prepare_backward_with_master_weights_FusedSGD(self):
    if self.materialize_master_grads:
        prepare_backward_with_master_weights(self)
    else:
        stash = self._amp_stash
        self._amp_lazy_init()
        for i, param in enumerate(stash.all_fp16_params):
            stash.all_fp16_grad_stash[i] = param.grad
            param.grad = None
        for i, param in enumerate(stash.all_fp32_from_fp32_params):
            stash.all_fp32_from_fp32_grad_stash[i] = param.grad
            param.grad = None


def post_backward_with_master_weights_FusedSGD(self, scaler):
    if self.materialize_master_grads:
        post_backward_with_master_weights(self, scaler)
    else:
        stash = self._amp_stash
        self._amp_lazy_init()
        grads_have_scale = scaler.loss_scale()
        stashed_have_scale = self.most_recent_scale
        out_scale = grads_have_scale
        if self.scale_set_by_backward:
            out_scale = min(grads_have_scale, self.most_recent_scale)
        for params, stashed in ((stash.all_fp16_params, stash.all_fp16_grad_stash),
                                (stash.all_fp32_from_fp32_params, stash.all_fp32_from_fp32_grad_stash)):
            post_backward_models_are_masters(scaler, params, stashed,
                                             (grads_have_scale, stashed_have_scale, out_scale))
        self.most_recent_scale = out_scale
        self.scale_set_by_backward = True


def _amp_lazy_init(self):
    stash = self._amp_stash
    if not stash.lazy_init_called:
        self._lazy_init_maybe_master_weights()
        stash.lazy_init_called = True


def _process_optimizer(optimizer, properties):
    from ..optimizers import FusedSGD

    if hasattr(optimizer, "_amp_stash"):
        raise RuntimeError("A given optimizer should only be passed through amp.initialize once.")
    optimizer._amp_stash = AmpOptimizerState()
    optimizer._amp_stash.lazy_init_called = False
    optimizer._amp_stash.already_patched = False
    optimizer._amp_stash.params_have_scaled_gradients = False
    for name in ("_lazy_init_maybe_master_weights", "_master_params_to_model_params", "_prepare_amp_backward",
                 "_post_amp_backward", "_amp_lazy_init"):
        if hasattr(optimizer, name):
            raise RuntimeError("Incoming optimizer already has {} defined.".format(name))

    dev = None
    for g in optimizer.param_groups:
        for p in g["params"]:
            dev = p.device
            break
        if dev is not None:
            break
    optimizer._amp_stash.multi_tensor_scale = amp_C.multi_tensor_scale
    optimizer._amp_stash.multi_tensor_l2norm = amp_C.multi_tensor_l2norm
    optimizer._amp_stash.dummy_overflow_buf = torch.zeros(1, dtype=torch.int, device=dev or "cpu")

    is_fused_sgd = isinstance(optimizer, FusedSGD)
    if properties.master_weights:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(lazy_init_with_master_weights, optimizer)
        optimizer._master_params_to_model_params = types.MethodType(_master_params_to_model_params, optimizer)
        old_step = optimizer.step

        def new_step(self, closure=None):
            if closure is not None:
                raise RuntimeError("Currently, Amp does not support closure use with optimizers.")
            retval = old_step()
            if not isinstance(self, FusedSGD):  # FusedSGD writes the 16-bit params in its kernel
                self._master_params_to_model_params()
            for param in self._amp_stash.all_fp32_from_fp16_params:
                param.grad = None
            return retval

        optimizer.step = types.MethodType(new_step, optimizer)

        def new_zero_grad(self, set_to_none=True):
            # Default set_to_none=True (PyTorch >= 2.0 semantics): the next _prepare_amp_backward
            # stashes / drops these grads anyway, so zero-filling them only adds one fill kernel per
            # parameter plus a stashed-gradient axpby pass after backward. set_to_none=False keeps
            # the reference's zeroing behaviour.
            stash = self._amp_stash
            self._amp_lazy_init()
            grads = []
            for param in stash.all_fp16_params + stash.all_fp32_from_fp32_params:
                if param.grad is not None:
                    if set_to_none:
                        param.grad = None
                    else:
                        param.grad.detach_()
                        grads.append(param.grad)
            if grads:
                torch._foreach_zero_(grads)
            for param in stash.all_fp32_from_fp16_params:
                param.grad = None

        optimizer.zero_grad = types.MethodType(new_zero_grad, optimizer)
        prep = prepare_backward_with_master_weights_FusedSGD if is_fused_sgd else prepare_backward_with_master_weights
        post = post_backward_with_master_weights_FusedSGD if is_fused_sgd else post_backward_with_master_weights
    else:
        optimizer._lazy_init_maybe_master_weights = types.MethodType(lazy_init_no_master_weights, optimizer)
        prep = prepare_backward_no_master_weights
        post = post_backward_no_master_weights
    optimizer._prepare_amp_backward = types.MethodType(prep, optimizer)
    optimizer._post_amp_backward = types.MethodType(post, optimizer)
    optimizer._amp_lazy_init = types.MethodType(_amp_lazy_init, optimizer)

    old_add_param_group = optimizer.add_param_group

    def new_add_param_group(self, new_group):
        stash = self._amp_stash
        if not stash.lazy_init_called:
            self._lazy_init_maybe_master_weights()
            stash.lazy_init_called = True
        assert isinstance(new_group, dict), "param group must be a dict"
        new_params = new_group["params"]
        if isinstance(new_params, torch.Tensor):
            new_group["params"] = [new_params]
        elif isinstance(new_params, set):
            raise TypeError("optimizer parameters need to be organized in ordered collections, but the ordering "
                            "of tensors in sets will change between runs. Please use a list instead.")
        else:
            new_group["params"] = list(new_params)
        if properties.master_weights:
            fp16_this, fp32_this, fp32_from_fp16_this = [], [], []
            for i, param in enumerate(new_group["params"]):
                if not param.requires_grad:
                    continue
                _check_param_type(param)
                if param.dtype in _LOW:
                    fp16_this.append(param)
                    master = param.detach().clone().float()
                    master.requires_grad = True
                    new_group["params"][i] = master
                    fp32_from_fp16_this.append(master)
                else:
                    fp32_this.append(param)
            stash.fp16_groups.append(fp16_this)
            stash.fp32_from_fp16_groups.append(fp32_from_fp16_this)
            stash.fp32_from_fp32_groups.append(fp32_this)
            stash.all_fp16_params += fp16_this
            stash.all_fp32_from_fp16_params += fp32_from_fp16_this
            stash.all_fp32_from_fp32_params += fp32_this
            stash.all_fp32_from_fp32_grad_stash += [None for _ in fp32_this]
        else:
            for param in new_group["params"]:
                _check_param_type(param)
                if param.dtype in _LOW:
                    stash.all_fp16_params.append(param)
                    stash.all_fp16_grad_stash.append(None)
                else:
                    stash.all_fp32_params.append(param)
                    stash.all_fp32_grad_stash.append(None)
        old_add_param_group(new_group)

    optimizer.add_param_group = types.MethodType(new_add_param_group, optimizer)
    return optimizer
