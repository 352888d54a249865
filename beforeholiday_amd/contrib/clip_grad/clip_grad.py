"""Fused gradient-norm clipping (reference: apex/contrib/clip_grad/clip_grad.py:14-129).

GPU path: one multi-tensor L2-norm launch per dtype group, the clip coefficient computed on the
device and applied by one multi-tensor scale launch per group that reads it from device memory —
no host synchronisation (the reference passes the coefficient tensor through a float argument,
which syncs). Other norms / CPU tensors use torch.nn.utils.clip_grad_norm_.
"""
from typing import Iterable, Union

import torch

from ...multi_tensor_apply import multi_tensor_applier
from ...ops import amp_C

_tensor_or_tensors = Union[torch.Tensor, Iterable[torch.Tensor]]


def clip_grad_norm_(parameters: _tensor_or_tensors, max_norm: float, norm_type: float = 2.0,
                    error_if_nonfinite: bool = False) -> torch.Tensor:
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    parameters = [p for p in parameters if p.grad is not None]
    max_norm = float(max_norm)
    norm_type = float(norm_type)
    if len(parameters) == 0:
        return torch.tensor(0.0)
    if not (norm_type == 2.0 and any(p.is_cuda for p in parameters)):
        return torch.nn.utils.clip_grad_norm_(parameters, max_norm, norm_type=norm_type,
                                              error_if_nonfinite=error_if_nonfinite)
    device = next(p.device for p in parameters if p.is_cuda)
    groups = {}
    misc = []
    for p in parameters:
        g = p.grad.detach()
        if p.device == device and g.dtype in (torch.float32, torch.float16, torch.bfloat16):
            groups.setdefault(g.dtype, []).append(g)
        else:
            misc.append(g)
    flag = torch.zeros([1], dtype=torch.int32, device=device)
    norms = [multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [gs], False)[0].reshape(1)
             for gs in groups.values()]
    norms += [torch.linalg.norm(g.float()).reshape(1).to(device) for g in misc]
    total_norm = torch.linalg.norm(torch.cat(norms))
    if error_if_nonfinite and torch.logical_or(total_norm.isnan(), total_norm.isinf()):
        raise RuntimeError(f"The total norm of order {norm_type} for gradients from `parameters` is non-finite, so "
                           "it cannot be clipped. To disable this error and scale the gradients by the non-finite "
                           "norm anyway, set `error_if_nonfinite=False`")
    coef = torch.clamp(max_norm / (total_norm + 1e-6), max=1.0)
    for gs in groups.values():
        multi_tensor_applier(amp_C.multi_tensor_scale, flag, [gs, gs], coef)
    for g in misc:
        g.mul_(coef.to(g.device))
    return total_norm
