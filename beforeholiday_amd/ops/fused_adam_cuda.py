"""``fused_adam_cuda``: the deprecated contrib Adam extension (reference:
``apex/contrib/csrc/optimizers/fused_adam_cuda.cpp:79-85``).

GPU tensors run ``beforeholiday_amd._C.fused_adam_cuda`` (kernels/legacy_optim.hip); CPU tensors run
the PyTorch references below with the same semantics (they are also the test oracle).

* ``adam(p, p_copy, m, v, g, ...)`` / ``adam_mt(chunk, flag, [p, m, v, g(, p_copy)], ...)``: legacy Adam, ``step_size = lr*sqrt(1-b2^t)/(1-b1^t)``,
  ``p -= step_size*(m/denom + decay*p)``, denom ``sqrt(v+eps)`` (mode 0) or ``sqrt(v)+eps`` (mode 1);
  optional reduced-precision copy ``p_copy`` (fp16 / bf16 / fp32 or uint8 e5m2).
* ``reversible_adam`` skips elements whose scaled gradient is not finite and then stores ``+inf``
  in ``p_copy[0]``; ``maybe_adam_undo`` reverts one step when ``overflow_flag`` is set.
* ``strided_check_finite``, ``maybe_cast`` / ``maybe_cast_mt``: overflow probing and the e5m2
  (de)compression of the distributed optimizers' parameter all-gather.

e5m2 bytes are the upper byte of an fp16 rounded to nearest.
"""
from __future__ import annotations

import math
from typing import List

import torch

from .._native import submodule


def _native():
    return submodule("fused_adam_cuda")


# ------------------------------------------------------------------------------- e5m2 helpers
def to_e5m2(x: torch.Tensor) -> torch.Tensor:
    """float tensor -> uint8 e5m2 (round to nearest, ties away; inf / nan preserved)."""
    xf = x.float()
    bits = xf.view(torch.int32) & torch.tensor(-8388608, dtype=torch.int32)  # 0xFF800000: sign+exponent
    half_ulp = bits.view(torch.float32) * 0.125
    h = (xf + torch.where(torch.isfinite(xf), half_ulp, torch.zeros_like(xf))).to(torch.float16)
    return (h.view(torch.int16) >> 8).to(torch.uint8)


def from_e5m2(b: torch.Tensor) -> torch.Tensor:
    return (b.to(torch.int16) << 8).view(torch.float16).float()


def _load(t: torch.Tensor) -> torch.Tensor:
    return from_e5m2(t) if t.dtype == torch.uint8 else t.float() if t.dtype != torch.float64 else t


def _store(dst: torch.Tensor, val: torch.Tensor):
    dst.copy_(to_e5m2(val) if dst.dtype == torch.uint8 else val.to(dst.dtype))


def _step_size(lr, beta1, beta2, step, bias_correction):
    if bias_correction == 1:
        return lr * math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step)
    return lr


def _ref_adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay,
              skip_nonfinite=False):
    acc = torch.float64 if p.dtype == torch.float64 else torch.float32
    ss = _step_size(lr, beta1, beta2, step, bias_correction)
    sg = g.to(acc) / grad_scale
    ok = torch.isfinite(sg) if skip_nonfinite else torch.ones_like(sg, dtype=torch.bool)
    sg0 = torch.where(ok, sg, torch.zeros_like(sg))
    m_new = beta1 * m.to(acc) + (1 - beta1) * sg0
    v_new = beta2 * v.to(acc) + (1 - beta2) * sg0 * sg0
    denom = torch.sqrt(v_new + eps) if mode == 0 else torch.sqrt(v_new) + eps
    p_new = p.to(acc) - ss * (m_new / denom + decay * p.to(acc))
    p.copy_(torch.where(ok, p_new, p.to(acc)).to(p.dtype))
    m.copy_(torch.where(ok, m_new, m.to(acc)).to(m.dtype))
    v.copy_(torch.where(ok, v_new, v.to(acc)).to(v.dtype))
    if p_copy is not None and p_copy.numel() > 0:
        _store(p_copy, p.to(acc))
        if skip_nonfinite and not bool(ok.all()):
            _store(p_copy.view(-1)[:1], torch.tensor([math.inf]))
    return bool(ok.all())


def adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay):
    if p.is_cuda:
        return _native().adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction,
                              decay)
    _ref_adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay)


def reversible_adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay):
    if p.is_cuda:
        return _native().reversible_adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode,
                                         bias_correction, decay)
    _ref_adam(p, p_copy, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay, True)


def maybe_adam_undo(overflow_flag, p, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay):
    if p.is_cuda:
        return _native().maybe_adam_undo(overflow_flag, p, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode,
                                         bias_correction, decay)
    if int(overflow_flag.reshape(-1)[0]) == 0:
        return
    acc = torch.float64 if p.dtype == torch.float64 else torch.float32
    ss = _step_size(lr, beta1, beta2, step, bias_correction)
    sg = g.to(acc) / grad_scale
    ok = torch.isfinite(sg)
    sg = torch.where(ok, sg, torch.zeros_like(sg))
    pa, ma, va = p.to(acc), m.to(acc), v.to(acc)
    denom = torch.sqrt(va + eps) if mode == 0 else torch.sqrt(va) + eps
    p_old = (pa + ss * (ma / denom)) / (1.0 - ss * decay)
    m_old = (ma - (1 - beta1) * sg) / beta1
    v_old = torch.clamp((va - (1 - beta2) * sg * sg) / beta2, min=0)
    p.copy_(torch.where(ok, p_old, pa).to(p.dtype))
    m.copy_(torch.where(ok, m_old, ma).to(m.dtype))
    v.copy_(torch.where(ok, v_old, va).to(v.dtype))


def adam_mt(chunk_size, overflow_flag, tensor_lists: List[List[torch.Tensor]], lr, beta1, beta2, eps, grad_scale,
            step, mode, bias_correction, decay):
    if tensor_lists and tensor_lists[0] and tensor_lists[0][0].is_cuda:
        return _native().adam_mt(chunk_size, overflow_flag, tensor_lists, lr, beta1, beta2, eps, grad_scale, step,
                                 mode, bias_correction, decay)
    copies = tensor_lists[4] if len(tensor_lists) > 4 else [None] * len(tensor_lists[0])
    for p, m, v, g, c in zip(tensor_lists[0], tensor_lists[1], tensor_lists[2], tensor_lists[3], copies):
        _ref_adam(p, c, m, v, g, lr, beta1, beta2, eps, grad_scale, step, mode, bias_correction, decay)


def strided_check_finite(overflow_flag, p_copy, stride, clear_overflow_first):
    if p_copy.is_cuda:
        return _native().strided_check_finite(overflow_flag, p_copy, stride, clear_overflow_first)
    if clear_overflow_first:
        overflow_flag.zero_()
    if not bool(torch.isfinite(_load(p_copy.reshape(-1)[::stride])).all()):
        overflow_flag.fill_(1)


def maybe_cast(overflow_flag, p_in, p_out):
    if p_in.is_cuda:
        return _native().maybe_cast(overflow_flag, p_in, p_out)
    if overflow_flag is not None and overflow_flag.numel() and int(overflow_flag.reshape(-1)[0]) != 0:
        return
    _store(p_out, _load(p_in))


def maybe_cast_mt(chunk_size, overflow_flag, tensor_lists):
    if tensor_lists and tensor_lists[0] and tensor_lists[0][0].is_cuda:
        return _native().maybe_cast_mt(chunk_size, overflow_flag, tensor_lists)
    for a, b in zip(tensor_lists[0], tensor_lists[1]):
        maybe_cast(overflow_flag, a, b)
