"""Shared plumbing for the fused optimizers."""
from __future__ import annotations

import torch


def noop_buffer(device) -> torch.Tensor:
    return torch.zeros(1, dtype=torch.int, device=device)


def first_device(param_groups):
    for g in param_groups:
        for p in g["params"]:
            return p.device
    return torch.device("cpu")


def grad_like_param(p: torch.Tensor) -> torch.Tensor:
    """The gradient laid out exactly like its parameter (the kernels walk raw memory).

    Reference: the channels_last handling in apex/optimizers/fused_sgd.py:166-199.
    """
    g = p.grad
    if g.stride() == p.stride() or p.numel() <= 1:
        return g
    for fmt in (torch.contiguous_format, torch.channels_last, torch.channels_last_3d):
        try:
            if p.is_contiguous(memory_format=fmt):
                return g.contiguous(memory_format=fmt)
        except RuntimeError:
            continue
    raise RuntimeError("fused optimizers support contiguous / channels_last parameters only")


def zero_grad(opt, set_grad_none: bool, set_to_none=None):
    none = set_grad_none if set_to_none is None else set_to_none
    grads = []
    for group in opt.param_groups:
        for p in group["params"]:
            if p.grad is None:
                continue
            if none:
                p.grad = None
            else:
                if p.grad.grad_fn is not None:
                    p.grad.detach_()
                else:
                    p.grad.requires_grad_(False)
                grads.append(p.grad)
    if grads:
        torch._foreach_zero_(grads)
