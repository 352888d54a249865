"""Pure-PyTorch reference implementations of the multi-tensor ops (fp32 math).

These define the semantics the HIP kernels in ``csrc/kernels/multi_tensor.hip`` must match and
serve CPU tensors (python-only path, CPU unit tests, gloo plumbing runs). Argument order is the
reference amp_C ABI (``csrc/amp_C_frontend.cpp:3-163``): ``(chunk_size, noop_flag, lists, ...)``.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

Lists = List[List[torch.Tensor]]


def _f(t: torch.Tensor) -> torch.Tensor:
    return t.detach().float()


def _set_flag(noop: torch.Tensor):
    noop.fill_(1)


def multi_tensor_scale(chunk_size, noop, lists: Lists, scale):
    ins, outs = lists
    bad = False
    for i, o in zip(ins, outs):
        x = _f(i)
        if not torch.isfinite(x).all():
            bad = True
        o.copy_((x * scale).to(o.dtype))
    if bad:
        _set_flag(noop)


def multi_tensor_axpby(chunk_size, noop, lists: Lists, a, b, arg_to_check):
    xs, ys, outs = lists
    bad = False
    for x, y, o in zip(xs, ys, outs):
        xf, yf = _f(x), _f(y)
        if arg_to_check == -1:
            bad |= not bool(torch.isfinite(xf).all() and torch.isfinite(yf).all())
        elif arg_to_check == 0:
            bad |= not bool(torch.isfinite(xf).all())
        elif arg_to_check == 1:
            bad |= not bool(torch.isfinite(yf).all())
        o.copy_((a * xf + b * yf).to(o.dtype))
    if bad:
        _set_flag(noop)


def _norms(lst, norm_type=2):
    vals = []
    for t in lst:
        x = _f(t).reshape(-1)
        if norm_type == 0:
            vals.append(x.abs().max() if x.numel() else torch.zeros((), device=x.device))
        else:
            vals.append((x * x).sum())
    return vals


def multi_tensor_l2norm(chunk_size, noop, lists: Lists, per_tensor=False, _mp=False):
    dev = noop.device
    if _mp and int(noop.item()) != 0:
        n = len(lists[0]) if lists and lists[0] else 0
        return torch.zeros(1, device=dev), (torch.zeros(n, device=dev) if per_tensor else torch.empty(0, device=dev))
    if not lists or not lists[0]:
        return torch.zeros(1, device=dev), torch.zeros(0, device=dev)
    sq = _norms(lists[0])
    tot = torch.stack(sq).sum() if sq else torch.zeros((), device=dev)
    if not torch.isfinite(tot):
        _set_flag(noop)
    total = tot.sqrt().reshape(1).to(dev)
    per = torch.stack([s.sqrt() for s in sq]).to(dev) if per_tensor else torch.empty(0, device=dev)
    return total, per


def multi_tensor_l2norm_mp(chunk_size, noop, lists: Lists, per_tensor=False):
    return multi_tensor_l2norm(chunk_size, noop, lists, per_tensor, _mp=True)


def multi_tensor_l2norm_scale(chunk_size, noop, lists: Lists, scale, per_tensor=False):
    total, per = multi_tensor_l2norm(chunk_size, noop, [lists[0]], per_tensor)
    for i, o in zip(lists[0], lists[1]):
        o.copy_((_f(i) * scale).to(o.dtype))
    return total, per


def multi_tensor_norm_out(chunk_size, noop, lists: Lists, out, alpha, beta, norm_type):
    vals = _norms(lists[0], 0 if norm_type == 0 else 2)
    for k, v in enumerate(vals):
        old = out[k].float()
        if norm_type == 0:
            out[k] = alpha * old + beta * v
        else:
            out[k] = torch.sqrt(alpha * old * old + beta * v)


def multi_tensor_adam(chunk_size, noop, lists: Lists, lr, beta1, beta2, eps, step, mode,
                      bias_correction, weight_decay):
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    copies = lists[4] if len(lists) > 4 else [None] * len(lists[0])
    for g, p, m, v, c in zip(lists[0], lists[1], lists[2], lists[3], copies):
        gf, pf, mf, vf = _f(g), _f(p), _f(m), _f(v)
        if mode == 0:
            gf = gf + weight_decay * pf
        mf = beta1 * mf + (1 - beta1) * gf
        vf = beta2 * vf + (1 - beta2) * gf * gf
        upd = (mf / bc1) / (torch.sqrt(vf / bc2) + eps)
        if mode == 1:
            upd = upd + weight_decay * pf
        pf = pf - lr * upd
        p.copy_(pf.to(p.dtype)), m.copy_(mf.to(m.dtype)), v.copy_(vf.to(v.dtype))
        if c is not None:
            c.copy_(pf.to(c.dtype))


def multi_tensor_adam_capturable(chunk_size, noop, lists, lr, beta1, beta2, eps, step, mode,
                                 bias_correction, weight_decay, inv_scale=None, found_inf=None):
    if found_inf is not None and float(found_inf.item()) != 0.0:
        return
    if inv_scale is not None:
        s = float(inv_scale.item())
        lists = [[g.float() * s for g in lists[0]]] + list(lists[1:])
    multi_tensor_adam(chunk_size, noop, lists, float(lr.item()), beta1, beta2, eps, int(step.item()),
                      mode, bias_correction, weight_decay)


def multi_tensor_sgd(chunk_size, noop, lists: Lists, wd, momentum, dampening, lr, nesterov,
                     first_run, wd_after_momentum, scale):
    if int(noop.item()) != 0:
        return
    copies = lists[3] if len(lists) > 3 else [None] * len(lists[0])
    for g, p, mom, c in zip(lists[0], lists[1], lists[2], copies):
        gf, pf = _f(g) * scale, _f(p)
        if wd != 0 and not wd_after_momentum:
            gf = gf + wd * pf
        if momentum != 0:
            mf = gf.clone() if first_run else _f(mom) * momentum + (1 - dampening) * gf
            gf = gf + momentum * mf if nesterov else mf
            mom.copy_(mf.to(mom.dtype))
        if wd != 0 and wd_after_momentum:
            gf = gf + wd * pf
        pf = pf - lr * gf
        p.copy_(pf.to(p.dtype))
        if c is not None:
            c.copy_(pf.to(c.dtype))


def _lamb(lists, lr, beta1, beta2, beta3, bc1, bc2, eps, decay, mode, nvlamb, clip, inv):
    copies = lists[4] if len(lists) > 4 else [None] * len(lists[0])
    for g, p, m, v, c in zip(lists[0], lists[1], lists[2], lists[3], copies):
        gf, pf, mf, vf = _f(g) * (inv / clip), _f(p), _f(m), _f(v)
        if mode == 0:
            gf = gf + decay * pf
        mf = mf * beta1 + beta3 * gf
        vf = vf * beta2 + (1 - beta2) * gf * gf
        u = (mf / bc1) / (torch.sqrt(vf / bc2) + eps)
        if mode == 1:
            u = u + decay * pf
        ratio = lr
        if nvlamb or decay != 0:
            pn, un = pf.norm(), u.norm()
            if pn != 0 and un != 0:
                ratio = lr * float(pn / un)
        pf = pf - ratio * u
        p.copy_(pf.to(p.dtype)), m.copy_(mf.to(m.dtype)), v.copy_(vf.to(v.dtype))
        if c is not None:
            c.copy_(pf.to(c.dtype))


def multi_tensor_lamb(chunk_size, noop, lists: Lists, lr, beta1, beta2, eps, step, bias_correction,
                      weight_decay, grad_averaging, mode, global_grad_norm, max_grad_norm,
                      use_nvlamb_python=False):
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    beta3 = 1 - beta1 if grad_averaging else 1.0
    gn = float(global_grad_norm.reshape(-1)[0])
    clip = gn / max_grad_norm if (max_grad_norm > 0 and gn > max_grad_norm) else 1.0
    _lamb(lists, lr, beta1, beta2, beta3, bc1, bc2, eps, weight_decay, mode, bool(use_nvlamb_python), clip, 1.0)


def multi_tensor_lamb_mp(chunk_size, noop, lists: Lists, lr, beta1, beta2, eps, step, bias_correction,
                         weight_decay, grad_averaging, mode, global_grad_norm, max_grad_norm,
                         use_nvlamb_python, found_inf, inv_scale):
    if int(noop.item()) != 0 or float(found_inf.item()) != 0.0:
        return
    st = int(step.reshape(-1)[0])
    bc1 = 1 - beta1 ** st if bias_correction else 1.0
    bc2 = 1 - beta2 ** st if bias_correction else 1.0
    beta3 = 1 - beta1 if grad_averaging else 1.0
    gn, mx = float(global_grad_norm.reshape(-1)[0]), float(max_grad_norm.reshape(-1)[0])
    clip = gn / mx if (mx > 0 and gn > mx) else 1.0
    _lamb(lists, float(lr.reshape(-1)[0]), beta1, beta2, beta3, bc1, bc2, eps, weight_decay, mode,
          bool(use_nvlamb_python), clip, float(inv_scale.reshape(-1)[0]))


def multi_tensor_lamb_stage1_cuda(chunk_size, noop, lists, per_tensor_decay, step, beta1, beta2, eps,
                                  global_grad_norm, max_global_grad_norm):
    gn = float(global_grad_norm.reshape(-1)[0])
    clipped = gn / max_global_grad_norm if gn > max_global_grad_norm else 1.0
    bc1, bc2 = 1 - beta1 ** step, 1 - beta2 ** step
    for k, (g, p, m, v, u) in enumerate(zip(*lists)):
        sg = _f(g) / clipped
        mf = _f(m) * beta1 + (1 - beta1) * sg
        vf = _f(v) * beta2 + (1 - beta2) * sg * sg
        uf = (mf / bc1) / (torch.sqrt(vf / bc2) + eps) + float(per_tensor_decay[k]) * _f(p)
        u.copy_(uf.to(u.dtype)), m.copy_(mf.to(m.dtype)), v.copy_(vf.to(v.dtype))


def multi_tensor_lamb_stage2_cuda(chunk_size, noop, lists, pnorm, unorm, lr, weight_decay, use_nvlamb=False):
    for k, (p, u) in enumerate(zip(*lists)):
        ratio = lr
        if use_nvlamb or weight_decay != 0:
            pn, un = float(pnorm[k]), float(unorm[k])
            ratio = lr * (pn / un) if (pn != 0 and un != 0) else lr
        p.copy_((_f(p) - ratio * _f(u)).to(p.dtype))


def multi_tensor_novograd(chunk_size, noop, lists, grad_norms, lr, beta1, beta2, eps, step,
                          bias_correction, weight_decay, grad_averaging, mode, norm_type):
    bc1, bc2 = 1.0, 1.0
    if bias_correction:
        bc1 = 1 - beta1 ** step
        bc2 = math.sqrt(1 - beta2 ** step)
    beta3 = 1 - beta1 if grad_averaging else 1.0
    multi_tensor_norm_out(chunk_size, noop, [lists[0]], grad_norms, beta2, 1 - beta2, norm_type)
    for k, (g, p, m) in enumerate(zip(*lists)):
        denom = float(grad_norms[k]) / bc2 + eps
        gf, pf, mf = _f(g), _f(p), _f(m)
        if mode == 0:
            gf = gf / denom + weight_decay * pf
            mf = beta1 * mf + beta3 * gf
            pf = pf - lr * (mf / bc1)
        else:
            mf = beta1 * mf + beta3 * gf
            pf = pf - lr * ((mf / bc1) / denom + weight_decay * pf)
        p.copy_(pf.to(p.dtype)), m.copy_(mf.to(m.dtype))


def multi_tensor_adagrad(chunk_size, noop, lists, lr, eps, mode, weight_decay):
    for g, p, h in zip(*lists):
        gf, pf, hf = _f(g), _f(p), _f(h)
        if mode == 0:
            gf = gf + weight_decay * pf
            hf = hf + gf * gf
            pf = pf - lr * (gf / (torch.sqrt(hf) + eps))
        else:
            hf = hf + gf * gf
            pf = pf - lr * (gf / (torch.sqrt(hf) + eps) + weight_decay * pf)
        p.copy_(pf.to(p.dtype)), h.copy_(hf.to(h.dtype))


def multi_tensor_lars(chunk_size, noop, lists, grad_norms, param_norms, lr, trust_coefficient, eps,
                      weight_decay, momentum, dampening, nesterov, first_run, wd_after_momentum, scale,
                      is_skipped):
    if int(noop.item()) != 0:
        return
    copies = lists[3] if len(lists) > 3 else [None] * len(lists[0])
    for k, (g, p, mom, c) in enumerate(zip(lists[0], lists[1], lists[2], copies)):
        slr = lr
        if not is_skipped:
            pn, gn = float(param_norms[k]), float(grad_norms[k])
            trust = trust_coefficient * pn / (gn + pn * weight_decay + eps) if (gn > 0 and pn > 0) else 1.0
            slr = lr * trust
        gf = _f(g) * scale + weight_decay * _f(p)
        mf = _f(mom) * momentum - slr * gf
        pf = _f(p) + (mf * momentum - slr * gf if nesterov else mf)
        p.copy_(pf.to(p.dtype)), mom.copy_(mf.to(mom.dtype))
        if c is not None:
            c.copy_(pf.to(c.dtype))
