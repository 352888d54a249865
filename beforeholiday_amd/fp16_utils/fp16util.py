"""Half-precision model helpers of the legacy fp16 API (reference: apex/fp16_utils/fp16util.py:22-187).

The conversion helpers keep affine BatchNorms in fp32 (their running statistics and affine
parameters lose too much in 16 bits); the master-weight helpers implement the manual
"fp16 model, fp32 master copy" loop either per tensor or as one flat fp32 master.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from .loss_scaler import to_python_float  # noqa: F401  (re-exported, as in the reference)


def _is_affine_bn(m):
    return isinstance(m, nn.modules.batchnorm._BatchNorm) and m.affine


class tofp16(nn.Module):
    """Input-casting layer: ``forward(x) = x.half()``."""

    def forward(self, input):
        return input.half()


def BN_convert_float(module):
    """Put every affine BatchNorm of ``module`` (recursively) back to fp32; returns ``module``."""
    for m in module.modules():
        if _is_affine_bn(m):
            m.float()
    return module


def network_to_half(network):
    """``Sequential(tofp16(), network.half())`` with the affine BatchNorms kept fp32 (legacy; prefer
    :class:`FP16Model`)."""
    return nn.Sequential(tofp16(), BN_convert_float(network.half()))


def _cast_(t, dtype):
    if t is not None and t.dtype.is_floating_point and t.dtype != dtype:
        t.data = t.data.to(dtype)


def convert_module(module, dtype):
    """Cast the floating-point tensors OWNED by ``module`` (not its children): parameters, their
    gradients, buffers."""
    for p in module.parameters(recurse=False):
        _cast_(p, dtype)
        _cast_(p.grad, dtype)
    for b in module.buffers(recurse=False):
        _cast_(b, dtype)


def convert_network(network, dtype):
    """``convert_module`` on every module except the affine BatchNorms; RNN weights re-flattened."""
    for m in network.modules():
        if _is_affine_bn(m):
            continue
        convert_module(m, dtype)
        if isinstance(m, nn.RNNBase):
            m.flatten_parameters()
    return network


class FP16Model(nn.Module):
    """Half-precision copy of ``network`` (affine BatchNorms fp32) whose inputs are cast to half."""

    def __init__(self, network):
        super().__init__()
        self.network = convert_network(network, dtype=torch.half)

    def forward(self, *inputs):
        return self.network(*(t.half() for t in inputs))


def backwards_debug_hook(grad):
    raise RuntimeError("master_params recieved a gradient in the backward pass!")


def prep_param_lists(model, flat_master=False):
    """(model_params, master_params): the trainable parameters and fp32 master copies of them --
    one flat fp32 Parameter (with a gradient buffer) when ``flat_master``."""
    model_params = [p for p in model.parameters() if p.requires_grad]
    if not flat_master:
        masters = []
        for p in model_params:
            m = p.detach().clone().float()
            m.requires_grad = True
            masters.append(m)
        return model_params, masters
    if len({p.dtype for p in model_params}) > 1:
        raise TypeError("prep_param_lists(flat_master=True): the model mixes parameter dtypes; use "
                        "flat_master=False or FP16_Optimizer")
    flat = nn.Parameter(_flatten_dense_tensors([p.detach() for p in model_params]).float())
    flat.grad = torch.empty_like(flat)
    return model_params, [flat]


def model_grads_to_master_grads(model_params, master_params, flat_master=False):
    """Copy the model's (16-bit) gradients into the fp32 masters' gradients."""
    if flat_master:
        master_params[0].grad.data.copy_(_flatten_dense_tensors([p.grad.data for p in model_params]))
        return
    for p, m in zip(model_params, master_params):
        if p.grad is None:
            m.grad = None
            continue
        if m.grad is None:
            m.grad = torch.empty_like(m)
        m.grad.data.copy_(p.grad.data)


def master_params_to_model_params(model_params, master_params, flat_master=False):
    """Copy the fp32 masters back into the (16-bit) model parameters."""
    sources = (_unflatten_dense_tensors(master_params[0].data, model_params) if flat_master
               else [m.data for m in master_params])
    for p, src in zip(model_params, sources):
        p.data.copy_(src)


clip_grad_norm = torch.nn.utils.clip_grad_norm_
