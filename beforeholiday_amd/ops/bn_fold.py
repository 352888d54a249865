"""BatchNorm backward folded into its 1x1 convolution by linear algebra (``_C.bn_fold``, kernels/bn_fold.hip).

For a training BatchNorm after a 1x1 convolution ``y = a @ W.T`` (``a [M, K]`` the convolution input, ``W [N, K]``)
and the BatchNorm's output gradient ``g [M, N]`` (already ReLU-masked), the input gradient is

    gx = A * g + B * y + D          (per channel n; A, B, D from the batch statistics and two sums)

and everything the convolution's backward needs follows from ``g``, ``a`` and small matrices -- ``y`` and ``gx``
are never read or written (:func:`combine`):

    sum_m g            = colsum(g)                       (mask_colsum's partials)
    sum_m g * y        = rowdot(W, P),   P = g.T @ a      (the raw weight-gradient product, fp32)
    dW                 = A * P + B * (W @ Gm) + D (x) S_a,  Gm = a.T @ a, S_a = colsum(a)   (gram)

so the BatchNorm's backward-reduce pass and the weight gradient's read of ``gx`` disappear, and the data
gradient ``gx @ W`` forms ``gx`` per fragment from ``(g, y)`` inside its GEMM (conv_bn's ``bnb`` prologue) --
``gx`` is never written. (``da`` could also be written without ``y`` as ``g @ (A W) + a @ (W.T diag(B) W) +
W.T @ D``, but those terms cancel after the 16-bit rounding of the small matrices: 40x less accurate on an
ill-conditioned gradient, tests/test_bn_fold.py.)

The reference reaches the same place with separate passes: ``reduce_bn_c_last`` then
``batchnorm_backward_c_last`` over the [M, N] tensors (/root/reference/csrc/welford.cu:739,895), and cuDNN's
fused dgrad + dReLU + dBN-scale for the bottleneck (/root/reference/apex/contrib/csrc/bottleneck/
bottleneck.cpp:760,1370,1414).

GPU tensors run the HIP kernels; CPU tensors run the fp32 references (what the GPU tests compare against).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import submodule


def _bn():
    return submodule("bn_fold")


def gram(a: torch.Tensor, pro_scale: Optional[torch.Tensor] = None,
         pro_shift: Optional[torch.Tensor] = None, s2=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(a'.T @ a', colsum(a'))`` in fp32 for ``a [M, K]``, ``a' = relu(a * pro_scale + pro_shift)`` rounded to
    a's dtype when a prologue is given (the activation a folded BatchNorm + ReLU never wrote). ``s2=(H, W)``:
    the rows are the even pixels (2y, 2x) of ``a`` viewed as ``[.., H, W, K]``."""
    if a.is_cuda:
        gp, cp = _bn().gram(a, pro_scale, pro_shift, *(s2 or (0, 0)))
        return gp.sum(0), cp.sum(0)
    if s2 is not None:
        H, W = s2
        a = a.view(-1, H, W, a.size(1))[:, ::2, ::2, :].reshape(-1, a.size(1))
    af = a.float()
    if pro_scale is not None:
        af = torch.relu(af * pro_scale + pro_shift).to(a.dtype).float()
    return af.t() @ af, af.sum(0)


def mask_colsum(g: torch.Tensor, bits: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(g * mask, colsum(g * mask))`` for ``g [M, N]`` and the ReLU bit mask ``bits [M, N/8]`` of
    ``syncbn.forward_mask`` (bit n % 8 of byte n / 8)."""
    if g.is_cuda:
        out, part = _bn().mask_colsum(g, bits)
        return out, part.sum(0)
    M, N = g.shape
    m = ((bits.view(M, N // 8, 1).to(torch.int32) >> torch.arange(8, dtype=torch.int32)) & 1).view(M, N)
    out = torch.where(m.bool(), g, torch.zeros_like(g))
    return out, out.float().sum(0)


def wgrad_f32(x: torch.Tensor, dy: torch.Tensor, pro_scale: Optional[torch.Tensor] = None,
              pro_shift: Optional[torch.Tensor] = None, stride: int = 1) -> torch.Tensor:
    """``dy.T @ x'`` over the pixels of two channels_last NCHW tensors (1x1 convolution, stride 1 or 2) as fp32
    ``[K_out, C_in]``, never rounded to 16 bits (kernels/conv_wgrad.hip partials, summed here)."""
    k = dy.size(1)
    c = x.size(1)
    if x.is_cuda:
        ws = submodule("conv_cuda").conv_wgrad_f32(x, dy, 1, stride, pro_scale, pro_shift)
        return ws.sum(0).view(k, c)
    if stride == 2:
        x = x[:, :, ::2, ::2]
    xf = x.permute(0, 2, 3, 1).reshape(-1, c).float()
    if pro_scale is not None:
        xf = torch.relu(xf * pro_scale + pro_shift).to(x.dtype).float()
    return dy.permute(0, 2, 3, 1).reshape(-1, k).float().t() @ xf


def local_sums(W: torch.Tensor, P: torch.Tensor, Sg: torch.Tensor, mean: torch.Tensor) -> torch.Tensor:
    """This rank's ``[sum g, sum g (y - mean)]`` (``[2N]`` fp32) of the BatchNorm after ``y = a @ W.T``."""
    Wf = W.float()
    return torch.cat([Sg, (Wf * P).sum(1) - mean * Sg])


def combine(W: torch.Tensor, P: torch.Tensor, Gm: torch.Tensor, Sa: torch.Tensor, sums: torch.Tensor,
            mean: torch.Tensor, invstd: torch.Tensor, weight: Optional[torch.Tensor], count: torch.Tensor):
    """From the (all-reduced) sums and this rank's ``P``, ``Gm``, ``S_a``: ``(dW [N, K], abd [3N])`` with the
    BatchNorm input gradient ``gx = A g + B y + D`` (``abd = (A, B, D)``, in P's dtype)."""
    N = W.size(0)
    Wf = W.to(P.dtype)  # fp32 (fp64 in the algebra test)
    n = count.to(P.dtype).reshape(-1)[0]
    mdy, mdyx = sums[:N] / n, sums[N:] / n
    wv = weight.to(P.dtype) if weight is not None else torch.ones_like(invstd)
    A = invstd * wv
    B = -invstd * invstd * A * mdyx
    D = A * (mean * invstd * invstd * mdyx - mdy)
    dW = A[:, None] * P + (B[:, None] * Wf) @ Gm + D[:, None] * Sa[None, :]
    return dW, torch.cat([A, B, D])


# ------------------------------------------------------------------------------ GPU fast path
# The node in models/resnet.py keeps every intermediate as fp32 partials and finishes the algebra in a few
# fixed-order kernels (no torch elementwise chains): mask_colsum / gram / weight-gradient partials ->
# reduce (P, Gm, S_a, sums, BatchNorm grads) -> [all-reduce of sums] -> finish (dW, Wa, H, c).


def mask_colsum_partials(g: torch.Tensor, bits: torch.Tensor):
    """GPU: ``(g * mask, column-sum partials [S, N])``."""
    return _bn().mask_colsum(g, bits)


def gram_partials(a: torch.Tensor, pro_scale=None, pro_shift=None, s2=None):
    """GPU: ``(Gram partials [S, K, K], column-sum partials [S, K])`` of ``a'`` (``s2``: see :func:`gram`)."""
    return _bn().gram(a, pro_scale, pro_shift, *(s2 or (0, 0)))


def wgrad_partials(x: torch.Tensor, dy: torch.Tensor, pro_scale=None, pro_shift=None, stride: int = 1) -> torch.Tensor:
    """GPU: ``dy.T @ x'`` as fp32 split partials ``[parts, K_out * C_in]``."""
    return submodule("conv_cuda").conv_wgrad_f32(x, dy, 1, stride, pro_scale, pro_shift)


def fold_reduce(W, p_ws, g_ws, sa_ws, sg_ws, mean, invstd):
    """GPU: ``(P, Gm, S_a, sums [2N], bn_grads [2N] = (dgamma, dbeta) of this rank)``."""
    return _bn().fold_reduce(W, p_ws, g_ws, sa_ws, sg_ws, mean, invstd)


def fold_finish(W, sums, count, mean, invstd, weight, P, Gm, Sa):
    """GPU: ``(dW, abd)`` (see :func:`combine`) from the all-reduced sums."""
    w = weight.float().contiguous() if weight is not None else None
    return _bn().fold_finish(W, sums, count.float().reshape(1), mean, invstd, w, P, Gm, Sa)
