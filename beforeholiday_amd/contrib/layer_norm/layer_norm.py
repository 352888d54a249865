"""FastLayerNorm (reference: apex/contrib/layer_norm/layer_norm.py:8-63, fast_layer_norm ext).

The reference registers a launcher per hidden size (768 ... 65536); the gfx950 LayerNorm kernels
(kernels/layer_norm.hip) handle any hidden size with a wave-per-row (<= 8192 wide rows in
registers) or workgroup-per-row schedule, so ``fast_layer_norm.ln_fwd / ln_bwd`` here are thin
adapters over ``fused_layer_norm_cuda`` with the reference's call signature.
"""
import types

import torch
from torch.nn import init

from ..._autocast_utils import _cast_if_autocast_enabled
from ...ops import fused_layer_norm_cuda as _ln


def ln_fwd(x, gamma, beta, epsilon):
    """(y, mu, rsigma) for a [rows, hidden] input."""
    shape = (gamma.numel(),)
    if gamma.dtype != x.dtype:
        y, mu, rs = _ln.forward_affine_mixed_dtypes(x, shape, gamma, beta, epsilon)
        return y.to(x.dtype), mu, rs
    return tuple(_ln.forward_affine(x, shape, gamma, beta, epsilon))


def ln_bwd(dy, x, mu, rsigma, gamma, beta=None, epsilon=1e-5):
    """(dx, dgamma, dbeta, dgamma_part, dbeta_part) — the partial buffers are folded into the
    deterministic column reduction, returned as the final values."""
    shape = (gamma.numel(),)
    b = beta if beta is not None else torch.zeros_like(gamma)
    dx, dg, db = _ln.backward_affine(dy, mu, rsigma, x, shape, gamma, b, epsilon, False)
    return dx, dg, db, dg, db


fast_layer_norm = types.SimpleNamespace(ln_fwd=ln_fwd, ln_bwd=ln_bwd)


class FastLayerNormFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, epsilon):
        x = x.contiguous()
        gamma, beta = gamma.contiguous(), beta.contiguous()
        xmat = x.view(-1, gamma.numel())
        y, mu, rsigma = ln_fwd(xmat, gamma, beta, epsilon)
        ctx.save_for_backward(x, gamma, beta, mu, rsigma)
        ctx.epsilon = epsilon
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x, gamma, beta, mu, rsigma = ctx.saved_tensors
        xmat = x.view(-1, gamma.numel())
        dx, dgamma, dbeta, _, _ = ln_bwd(dy.contiguous().view(xmat.shape), xmat, mu, rsigma, gamma, beta,
                                          ctx.epsilon)
        return dx.view(x.shape), dgamma, dbeta, None


def _fast_layer_norm(x, weight, bias, epsilon):
    args = _cast_if_autocast_enabled(x, weight, bias, epsilon)
    with torch.autocast("cuda", enabled=False):
        return FastLayerNormFN.apply(*args)


class FastLayerNorm(torch.nn.Module):
    def __init__(self, hidden_size, eps=1e-5):
        super().__init__()
        self.epsilon = eps
        self.weight = torch.nn.Parameter(torch.empty(hidden_size))
        self.bias = torch.nn.Parameter(torch.empty(hidden_size))
        self.reset_parameters()

    def reset_parameters(self):
        init.ones_(self.weight)
        init.zeros_(self.bias)

    def forward(self, x):
        return _fast_layer_norm(x, self.weight, self.bias, self.epsilon)
