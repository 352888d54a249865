"""``distributed_lamb_cuda``: the two ZeRO-LAMB stages with device-resident scalars (reference:
``apex/contrib/csrc/optimizers/multi_tensor_distopt_lamb.cpp`` / ``_kernel.cu:109-506``).

GPU lists run ``beforeholiday_amd._C.distributed_lamb_cuda`` (kernels/legacy_optim.hip); CPU lists
run the references below (same math, also the test oracle). Both stages return immediately when
``noop_flag`` is set, so an overflowing step is skipped without a host synchronisation.

* ``multi_tensor_lamb_compute_update_term(chunk, noop, [g, p, m, v, u], beta1, beta2, beta3,
  bias_correction, step, eps, mode, decay, global_scale, global_grad_norm, max_grad_norm)``:
  ``g / combined_scale`` with ``combined_scale = global_scale / min(1, max_norm / (norm/global_scale + 1e-6))``,
  Adam moments, ``u = m_hat / (sqrt(v_hat) + eps) (+ decay * p)`` (mode 1) or L2 folded into g (mode 0).
* ``multi_tensor_lamb_update_weights(chunk, noop, [p, u(, p_copy)], param_norm, update_norm,
  update_norm_offset, lr, decay, global_grad_norm, use_nvlamb)``: trust ratio ``||p|| / ||u||``
  (when ``decay != 0`` or nvlamb), ``p -= lr * ratio * u`` and the optional fp16 / bf16 / e5m2 copy.
"""
from __future__ import annotations

import torch

from .._native import submodule
from .fused_adam_cuda import _store


def _native():
    return submodule("distributed_lamb_cuda")


def multi_tensor_lamb_compute_update_term(chunk_size, noop_flag, tensor_lists, per_tensor_beta1, per_tensor_beta2,
                                          per_tensor_beta3, per_tensor_bias_correction, step, per_tensor_epsilon,
                                          mode, per_tensor_decay, global_scale, global_grad_norm, max_grad_norm):
    if tensor_lists[0] and tensor_lists[0][0].is_cuda:
        return _native().multi_tensor_lamb_compute_update_term(
            chunk_size, noop_flag, tensor_lists, per_tensor_beta1, per_tensor_beta2, per_tensor_beta3,
            per_tensor_bias_correction, step, per_tensor_epsilon, mode, per_tensor_decay, global_scale,
            global_grad_norm, max_grad_norm)
    if int(noop_flag.reshape(-1)[0]) != 0:
        return
    gs = float(global_scale.reshape(-1)[0])
    combined = gs
    if max_grad_norm > 0:
        clip = max_grad_norm / (float(global_grad_norm.reshape(-1)[0]) / gs + 1e-6)
        combined = gs / min(1.0, clip)
    t_step = int(step.reshape(-1)[0])
    for t, (g, p, m, v, u) in enumerate(zip(*tensor_lists)):
        b1, b2, b3 = float(per_tensor_beta1[t]), float(per_tensor_beta2[t]), float(per_tensor_beta3[t])
        eps, decay = float(per_tensor_epsilon[t]), float(per_tensor_decay[t])
        c1 = 1 - b1 ** t_step if int(per_tensor_bias_correction[t]) == 1 else 1.0
        c2 = 1 - b2 ** t_step if int(per_tensor_bias_correction[t]) == 1 else 1.0
        sg = g.float() / combined
        pv = p.float() if decay != 0 else torch.zeros_like(sg)
        if mode == 0:
            sg = sg + decay * pv
        mv = m.float() * b1 + b3 * sg
        vv = v.float() * b2 + (1 - b2) * sg * sg
        upd = (mv / c1) / (torch.sqrt(vv / c2) + eps)
        if mode != 0:
            upd = upd + decay * pv
        m.copy_(mv)
        v.copy_(vv)
        u.copy_(upd)


def multi_tensor_lamb_update_weights(chunk_size, noop_flag, tensor_lists, per_tensor_param_norm,
                                     per_tensor_update_norm, update_norm_offset, learning_rate, per_tensor_decay,
                                     global_grad_norm, use_nvlamb):
    if tensor_lists[0] and tensor_lists[0][0].is_cuda:
        return _native().multi_tensor_lamb_update_weights(
            chunk_size, noop_flag, tensor_lists, per_tensor_param_norm, per_tensor_update_norm, update_norm_offset,
            learning_rate, per_tensor_decay, global_grad_norm, use_nvlamb)
    if int(noop_flag.reshape(-1)[0]) != 0:
        return
    lr = float(learning_rate.reshape(-1)[0])
    copies = tensor_lists[2] if len(tensor_lists) > 2 else [None] * len(tensor_lists[0])
    for t, (p, u, c) in enumerate(zip(tensor_lists[0], tensor_lists[1], copies)):
        ratio = lr
        if use_nvlamb or float(per_tensor_decay[t]) != 0.0:
            pn = float(per_tensor_param_norm[t])
            un = float(per_tensor_update_norm[int(update_norm_offset[t])])
            ratio = lr * (pn / un) if (un != 0.0 and pn != 0.0) else lr
        pv = p.float() - ratio * u.float()
        p.copy_(pv)
        if c is not None:
            _store(c, pv)
