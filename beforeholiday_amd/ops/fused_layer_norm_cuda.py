"""``fused_layer_norm_cuda``: LayerNorm / RMSNorm ops with the reference extension's function names
(csrc/layer_norm_cuda.cpp:428-441). GPU: kernels/layer_norm.hip; CPU: fp32 PyTorch reference."""
from __future__ import annotations

import torch

from .._native import submodule


def _n():
    return submodule("fused_layer_norm_cuda")


def _dims(shape):
    return tuple(range(-len(shape), 0))


def _ref_fwd(x, shape, gamma, beta, eps, rms, out_dtype):
    xf = x.float()
    d = _dims(shape)
    if rms:
        mean = None
        var = xf.pow(2).mean(d, keepdim=True)
        xh = xf * torch.rsqrt(var + eps)
    else:
        mean = xf.mean(d, keepdim=True)
        var = (xf - mean).pow(2).mean(d, keepdim=True)
        xh = (xf - mean) * torch.rsqrt(var + eps)
    y = xh
    if gamma is not None:
        y = y * gamma.float()
    if beta is not None and not rms:
        y = y + beta.float()
    invvar = torch.rsqrt(var + eps).reshape(x.shape[:x.dim() - len(shape)])
    out = [y.to(out_dtype), invvar]
    if not rms:
        out.insert(1, mean.reshape(x.shape[:x.dim() - len(shape)]))
    return out


def _ref_bwd(dout, mean, invvar, xin, shape, gamma, beta, eps, rms, memory_efficient):
    d = _dims(shape)
    bshape = list(invvar.shape) + [1] * len(shape)
    iv = invvar.reshape(bshape)
    xf = xin.float()
    if memory_efficient:
        yv = xf - beta.float() if (beta is not None and not rms) else xf
        xh = yv / gamma.float() if gamma is not None else yv
    else:
        xh = (xf - (0.0 if rms else mean.reshape(bshape))) * iv
    g = dout.float() * (gamma.float() if gamma is not None else 1.0)
    m2 = (g * xh).mean(d, keepdim=True)
    dx = iv * (g - (0.0 if rms else g.mean(d, keepdim=True)) - xh * m2)
    red = tuple(range(0, xin.dim() - len(shape)))
    gg = (dout.float() * xh).sum(red).to(gamma.dtype) if gamma is not None else None
    gb = dout.float().sum(red).to(beta.dtype) if (beta is not None and not rms) else None
    return dx.to(xin.dtype), gg, gb


def forward_affine(input, normalized_shape, gamma, beta, eps):
    if input.is_cuda:
        return _n().forward_affine(input, normalized_shape, gamma, beta, eps)
    return _ref_fwd(input, normalized_shape, gamma, beta, eps, False, input.dtype)


def forward_affine_mixed_dtypes(input, normalized_shape, gamma, beta, eps):
    if input.is_cuda:
        return _n().forward_affine_mixed_dtypes(input, normalized_shape, gamma, beta, eps)
    return _ref_fwd(input, normalized_shape, gamma, beta, eps, False, gamma.dtype)


def forward(input, normalized_shape, eps):
    if input.is_cuda:
        return _n().forward(input, normalized_shape, eps)
    return _ref_fwd(input, normalized_shape, None, None, eps, False, input.dtype)


def rms_forward_affine(input, normalized_shape, gamma, eps):
    if input.is_cuda:
        return _n().rms_forward_affine(input, normalized_shape, gamma, eps)
    return _ref_fwd(input, normalized_shape, gamma, None, eps, True, input.dtype)


def rms_forward_affine_mixed_dtypes(input, normalized_shape, gamma, eps):
    if input.is_cuda:
        return _n().rms_forward_affine_mixed_dtypes(input, normalized_shape, gamma, eps)
    return _ref_fwd(input, normalized_shape, gamma, None, eps, True, gamma.dtype)


def rms_forward(input, normalized_shape, eps):
    if input.is_cuda:
        return _n().rms_forward(input, normalized_shape, eps)
    return _ref_fwd(input, normalized_shape, None, None, eps, True, input.dtype)


def _mean_or_empty(mean, ref):
    # memory-efficient backward recomputes x_hat from the output: mean is not needed (None)
    return mean if mean is not None else ref.new_empty(0, dtype=torch.float32)


def backward_affine(dout, mean, invvar, input_or_output, normalized_shape, gamma, beta, eps, memory_efficient=False,
                    dresid=None):
    """(grad_input, grad_gamma, grad_beta). ``dresid`` (input-shaped, the input's dtype): a gradient the
    residual branch sends to the same input, added to grad_input inside the dx kernel (one rounding, no
    separate add pass: the reference's MHA LayerNorm ``dout_resid``, layer_norm.cuh:474,566,603)."""
    if dout.is_cuda:
        return _n().backward_affine(dout, _mean_or_empty(mean, dout), invvar, input_or_output, normalized_shape, gamma, beta, eps,
                                    memory_efficient, dresid)
    gi, gg, gb = _ref_bwd(dout, mean, invvar, input_or_output, normalized_shape, gamma, beta, eps, False, memory_efficient)
    if dresid is not None:
        gi = (gi.float() + dresid.float()).to(gi.dtype)
    return gi, gg, gb


def backward(dout, mean, invvar, input_or_output, normalized_shape, eps, memory_efficient=False):
    if dout.is_cuda:
        return _n().backward(dout, _mean_or_empty(mean, dout), invvar, input_or_output, normalized_shape, eps, memory_efficient)
    return _ref_bwd(dout, mean, invvar, input_or_output, normalized_shape, None, None, eps, False, memory_efficient)[0]


def rms_backward_affine(dout, invvar, input_or_output, normalized_shape, gamma, eps, memory_efficient=False):
    if dout.is_cuda:
        return _n().rms_backward_affine(dout, invvar, input_or_output, normalized_shape, gamma, eps, memory_efficient)
    r = _ref_bwd(dout, None, invvar, input_or_output, normalized_shape, gamma, None, eps, True, memory_efficient)
    return r[0], r[1]


def rms_backward(dout, invvar, input_or_output, normalized_shape, eps, memory_efficient=False):
    if dout.is_cuda:
        return _n().rms_backward(dout, invvar, input_or_output, normalized_shape, eps, memory_efficient)
    return _ref_bwd(dout, None, invvar, input_or_output, normalized_shape, None, None, eps, True, memory_efficient)[0]
