"""``distributed_adam_cuda``: multi-tensor Adam with per-tensor hyper-parameters (reference:
``apex/contrib/csrc/optimizers/multi_tensor_distopt_adam.cpp``, kernel ``:32-228``).

``multi_tensor_fused_adam(chunk, noop, [p, m, v, g(, p_copy)], beta1, beta2, bias_correction, eps,
weight_decay, lr, grad_scale, step, mode)``: ``g/grad_scale``, Adam moments, denom from the
bias-corrected v (``sqrt(v_hat + eps)`` for mode 0, ``sqrt(v_hat) + eps`` for mode 1),
``p -= lr * (m_hat/denom + wd*p)``, optional copy in the gradient dtype. GPU lists run
``beforeholiday_amd._C.distributed_adam_cuda``; CPU lists the reference below.
"""
from __future__ import annotations

import torch

from .._native import submodule


def multi_tensor_fused_adam(chunk_size, noop_flag, tensor_lists, per_tensor_beta1, per_tensor_beta2,
                            per_tensor_bias_correction, per_tensor_eps, per_tensor_weight_decay, lr, grad_scale, step,
                            mode):
    if tensor_lists[0] and tensor_lists[0][0].is_cuda:
        return submodule("distributed_adam_cuda").multi_tensor_fused_adam(
            chunk_size, noop_flag, tensor_lists, per_tensor_beta1, per_tensor_beta2, per_tensor_bias_correction,
            per_tensor_eps, per_tensor_weight_decay, lr, grad_scale, step, mode)
    copies = tensor_lists[4] if len(tensor_lists) > 4 else [None] * len(tensor_lists[0])
    for t, (p, m, v, g, c) in enumerate(zip(*tensor_lists[:4], copies)):
        b1, b2 = float(per_tensor_beta1[t]), float(per_tensor_beta2[t])
        eps, wd = float(per_tensor_eps[t]), float(per_tensor_weight_decay[t])
        c1 = 1 - b1 ** step if int(per_tensor_bias_correction[t]) == 1 else 1.0
        c2 = 1 - b2 ** step if int(per_tensor_bias_correction[t]) == 1 else 1.0
        sg = g.float() / grad_scale
        mv = b1 * m.float() + (1 - b1) * sg
        vv = b2 * v.float() + (1 - b2) * sg * sg
        vh = vv / c2
        denom = torch.sqrt(vh + eps) if mode == 0 else torch.sqrt(vh) + eps
        pv = p.float() - lr * ((mv / c1) / denom + wd * p.float())
        m.copy_(mv)
        v.copy_(vv)
        p.copy_(pv)
        if c is not None:
            c.copy_(pv)
