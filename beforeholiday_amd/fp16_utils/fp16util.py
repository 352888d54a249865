"""Legacy fp16 helpers (reference: apex/fp16_utils/fp16util.py:22-187)."""
from __future__ import annotations

import torch
import torch.nn as nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors


class tofp16(nn.Module):
    """``forward(x) = x.half()``."""

    def forward(self, input):
        return input.half()


def BN_convert_float(module):
    """Recursively keep affine BatchNorm layers in fp32."""
    if isinstance(module, torch.nn.modules.batchnorm._BatchNorm) and module.affine is True:
        module.float()
    for child in module.children():
        BN_convert_float(child)
    return module


def network_to_half(network):
    """Batchnorm-safe conversion to half (legacy; prefer :class:`FP16Model`)."""
    return nn.Sequential(tofp16(), BN_convert_float(network.half()))


def convert_module(module, dtype):
    """Convert a module's immediate floating-point parameters (and grads) and buffers to ``dtype``."""
    for param in module.parameters(recurse=False):
        if param is not None:
            if param.data.dtype.is_floating_point:
                param.data = param.data.to(dtype=dtype)
            if param._grad is not None and param._grad.data.dtype.is_floating_point:
                param._grad.data = param._grad.data.to(dtype=dtype)
    for buf in module.buffers(recurse=False):
        if buf is not None and buf.data.dtype.is_floating_point:
            buf.data = buf.data.to(dtype=dtype)


def convert_network(network, dtype):
    """Convert every module except affine BatchNorms (kept fp32 for stable statistics)."""
    for module in network.modules():
        if isinstance(module, torch.nn.modules.batchnorm._BatchNorm) and module.affine is True:
            continue
        convert_module(module, dtype)
        if isinstance(module, torch.nn.RNNBase):
            module.flatten_parameters()
    return network


class FP16Model(nn.Module):
    """Batchnorm-safe half-precision model wrapper; casts inputs to half."""

    def __init__(self, network):
        super().__init__()
        self.network = convert_network(network, dtype=torch.half)

    def forward(self, *inputs):
        return self.network(*tuple(t.half() for t in inputs))


def backwards_debug_hook(grad):
    raise RuntimeError("master_params recieved a gradient in the backward pass!")


def prep_param_lists(model, flat_master=False):
    """Returns (model_params, fp32 master_params) -- master_params is a 1-element list if flat."""
    model_params = [p for p in model.parameters() if p.requires_grad]
    if flat_master:
        try:
            master = _flatten_dense_tensors([p.data for p in model_params]).float()
        except Exception:
            print("Error in prep_param_lists:  model may contain a mixture of parameters of different types.  "
                  "Use flat_master=False, or use F16_Optimizer.")
            raise
        master = torch.nn.Parameter(master)
        master.requires_grad = True
        if master.grad is None:
            master.grad = master.new(*master.size())
        return model_params, [master]
    master_params = [p.clone().float().detach() for p in model_params]
    for p in master_params:
        p.requires_grad = True
    return model_params, master_params


def model_grads_to_master_grads(model_params, master_params, flat_master=False):
    if flat_master:
        master_params[0].grad.data.copy_(_flatten_dense_tensors([p.grad.data for p in model_params]))
        return
    for model, master in zip(model_params, master_params):
        if model.grad is not None:
            if master.grad is None:
                master.grad = torch.empty_like(master.data)
            master.grad.data.copy_(model.grad.data)
        else:
            master.grad = None


def master_params_to_model_params(model_params, master_params, flat_master=False):
    if flat_master:
        for model, master in zip(model_params, _unflatten_dense_tensors(master_params[0].data, model_params)):
            model.data.copy_(master)
        return
    for model, master in zip(model_params, master_params):
        model.data.copy_(master.data)


def to_python_float(t):
    if hasattr(t, "item"):
        return t.item()
    return t[0]


clip_grad_norm = torch.nn.utils.clip_grad_norm_
