"""Attention softmax ops (reference modules scaled_upper_triang_masked_softmax_cuda,
scaled_masked_softmax_cuda, scaled_softmax_cuda, generic_scaled_masked_softmax_cuda).
GPU: kernels/softmax.hip; CPU: fp32 PyTorch reference with the same masking conventions
(padding-masked elements -> -10000, fully masked rows -> 0, causal columns > row -> 0)."""
from __future__ import annotations

import torch

from .._native import submodule


def _ref_masked_fwd(x, mask, scale):
    xf = x.float() * scale
    if mask is not None:
        xf = xf.masked_fill(mask.bool(), -10000.0)
    y = torch.softmax(xf, dim=-1)
    if mask is not None:
        dead = (xf.amax(-1, keepdim=True) == -10000.0)
        y = torch.where(dead, torch.zeros_like(y), y)
    return y.to(x.dtype)


def _ref_causal_fwd(x, scale):
    sq, sk = x.shape[-2], x.shape[-1]
    m = torch.triu(torch.ones(sq, sk, dtype=torch.bool, device=x.device), diagonal=1)
    y = torch.softmax((x.float() * scale).masked_fill(m, float("-inf")), dim=-1)
    return y.to(x.dtype)


def _ref_bwd(dy, y, scale):
    yf, gf = y.float(), dy.float()
    return (scale * yf * (gf - (gf * yf).sum(-1, keepdim=True))).to(y.dtype)


def scaled_masked_softmax_forward(x, mask, scale):
    if x.is_cuda:
        return submodule("scaled_masked_softmax_cuda").forward(x, mask, scale)
    return _ref_masked_fwd(x, mask, scale)


def scaled_masked_softmax_backward(dy, y, scale):
    if y.is_cuda:
        return submodule("scaled_masked_softmax_cuda").backward(dy, y, scale)
    return _ref_bwd(dy, y, scale)


def scaled_softmax_forward(x, scale):
    if x.is_cuda:
        return submodule("scaled_softmax_cuda").forward(x, scale)
    return _ref_masked_fwd(x, None, scale)


def scaled_softmax_backward(dy, y, scale):
    if y.is_cuda:
        return submodule("scaled_softmax_cuda").backward(dy, y, scale)
    return _ref_bwd(dy, y, scale)


def scaled_upper_triang_masked_softmax_forward(x, scale):
    if x.is_cuda:
        return submodule("scaled_upper_triang_masked_softmax_cuda").forward(x, scale)
    return _ref_causal_fwd(x, scale)


def scaled_upper_triang_masked_softmax_backward(dy, y, scale):
    if y.is_cuda:
        return submodule("scaled_upper_triang_masked_softmax_cuda").backward(dy, y, scale)
    return _ref_bwd(dy, y, scale)


def generic_scaled_masked_softmax_forward(x, mask, scale):
    if x.is_cuda:
        return submodule("generic_scaled_masked_softmax_cuda").forward(x, mask, scale)
    return _ref_masked_fwd(x, mask, scale)


def generic_scaled_masked_softmax_backward(dy, y, scale):
    if y.is_cuda:
        return submodule("generic_scaled_masked_softmax_cuda").backward(dy, y, scale)
    return _ref_bwd(dy, y, scale)


def get_batch_per_block(sq, sk, b, np):
    return 1


def xentropy_forward(logits, labels, smoothing, half_to_float):
    if logits.is_cuda:
        return submodule("xentropy_cuda").forward(logits, labels, smoothing, half_to_float)
    xf = logits.float()
    lse = torch.logsumexp(xf, dim=-1)
    xy = xf.gather(1, labels.long().clamp(0, xf.size(1) - 1).unsqueeze(1)).squeeze(1)
    loss = lse - (1 - smoothing) * xy - smoothing * xf.mean(-1)
    return loss.to(torch.float32 if half_to_float else logits.dtype), lse


def xentropy_backward(grad_loss, logits, lse, labels, smoothing):
    if logits.is_cuda:
        return submodule("xentropy_cuda").backward(grad_loss, logits, lse, labels, smoothing)
    xf = logits.float()
    p = torch.exp(xf - lse.float().unsqueeze(1))
    tgt = torch.zeros_like(p).scatter_(1, labels.long().unsqueeze(1), 1.0 - smoothing)
    return (grad_loss.float().unsqueeze(1) * (p - tgt - smoothing / xf.size(1))).to(logits.dtype)
