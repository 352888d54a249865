"""1x1 convolution GEMMs with BatchNorm folded in (kernels/conv_bn.hip, ``_C.conv_bn``).

All tensors are ``[pixels, channels]`` views of NHWC activations. ``c1x1`` returns ``(C, part)``:

* ``C = f(A) @ B.T`` (+ ``resid``) rounded to A's dtype, with ``f(a) = relu(a * pro_scale + pro_shift)``
  per input channel when a prologue is given (the producing layer's BatchNorm + ReLU, never written);
* ``s2=(H, W)``: output row (n, y, x) reads input row (n, 2y, 2x) of an ``[N, H, W, K]`` input
  (1x1 / stride-2 convolution);
* ``epi="stats"``: ``part [2, G, N]`` holds per-workgroup sums of ``C - kshift`` and ``(C - kshift)^2``
  (C as stored) -- :func:`sum_parts` turns them into the ``[2N+1]`` payload of
  ``syncbn.stats_local_sums``;
* ``epi="bwd"``: with ``by`` (the raw input of the previous BatchNorm, same shape as C), ``dz = C *
  (by * bscale + bshift > 0)``: sums of ``dz`` and ``dz * (by - bmean)`` -- that BatchNorm's backward
  reduction (``syncbn.backward_reduce``'s sums), computed as the data gradient is produced.

GPU tensors run the HIP kernel (no silent fallback: unsupported shapes raise); CPU tensors run the
fp32 reference below, which is also what the GPU tests compare against.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .._native import available, submodule

_EPI = {"plain": 0, "stats": 1, "bwd": 2, "affine": 3, "mask": 4}


def _gather_s2(a: torch.Tensor, s2) -> torch.Tensor:
    H, W = s2
    K = a.size(1)
    return a.view(-1, H, W, K)[:, ::2, ::2, :].reshape(-1, K)


def _bit_mask(bits, M, N):
    return ((bits.view(M, N // 8, 1).to(torch.int32) >> torch.arange(8, dtype=torch.int32)) & 1).view(M, N).bool()


def _reference(a, b, pro_scale, pro_shift, resid, s2, epi, kshift, by, bscale, bshift, bmean, brelu, bnb=None,
               bnb_y=None, mbits=None):
    if s2 is not None:
        a = _gather_s2(a, s2)
    af = a.float()
    if pro_scale is not None:
        af = torch.relu(af * pro_scale + pro_shift).to(a.dtype).float()
    if bnb is not None:
        K = a.size(1)
        af = (af * bnb[:K] + bnb_y.float() * bnb[K:2 * K] + bnb[2 * K:]).to(a.dtype).float()
    c = af @ b.float().t()
    if resid is not None:
        c = c + resid.float()
    N = b.size(0)
    if epi == "mask":
        c = torch.where(_bit_mask(mbits, c.size(0), N), c, torch.zeros_like(c))
    c = c.to(a.dtype)
    cf = c.float()
    if epi == "stats":
        d = cf - (kshift if kshift is not None else 0.0)
        part = torch.stack([d.sum(0), (d * d).sum(0)]).view(2, 1, N)
    elif epi == "mask":
        part = torch.stack([cf.sum(0), torch.zeros_like(cf[0])]).view(2, 1, N)
    elif epi == "bwd":
        y = by.float()
        dz = cf * ((y * bscale + bshift) > 0).float() if brelu else cf
        part = torch.stack([dz.sum(0), (dz * (y - bmean)).sum(0)]).view(2, 1, N)
    else:
        part = torch.empty(0)
    return c, part


def c1x1(a: torch.Tensor, b: torch.Tensor, pro_scale: Optional[torch.Tensor] = None,
         pro_shift: Optional[torch.Tensor] = None, resid: Optional[torch.Tensor] = None, s2=None,
         epi: str = "plain", kshift: Optional[torch.Tensor] = None, by: Optional[torch.Tensor] = None,
         bscale: Optional[torch.Tensor] = None, bshift: Optional[torch.Tensor] = None,
         bmean: Optional[torch.Tensor] = None, brelu: bool = True,
         b_trans: bool = False, s2_scatter: bool = False, bnb: Optional[torch.Tensor] = None,
         bnb_y: Optional[torch.Tensor] = None, mbits: Optional[torch.Tensor] = None,
         lda: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """``b_trans``: ``b`` is given as ``[K, N]`` (e.g. a forward weight for the data gradient).
    ``bnb`` (fp32 ``[3K]`` = A, B, D) with ``bnb_y`` (shaped like ``a``): the BatchNorm-backward prologue
    ``f(a) = A * a + B * bnb_y + D`` per input channel, rounded to a's dtype (ops/bn_fold.py).
    ``epi="mask"`` with ``mbits`` (uint8 ``[M, N/8]``, syncbn.forward_mask's ReLU bits): C is masked and
    ``part[0]`` holds its column-sum partials. ``lda``: ``a`` (and ``bnb_y``) are column slices of row-major
    tensors with that row stride (a split-K data gradient).
    ``s2_scatter`` (with ``s2=(H, W)`` and ``resid`` the full-resolution ``[N*H*W, N]`` tensor): row
    (n, y, x) of ``a @ b.T`` is ADDED in place into row (n, 2y, 2x) of ``resid``, which is returned --
    the 1x1 / stride-2 data gradient accumulated onto the other branch's gradient."""
    rows = a.size(0)
    M = rows // 4 if (s2 is not None and not s2_scatter) else rows
    if not a.is_cuda:
        bb = b.t() if b_trans else b
        if s2_scatter:
            H, W = s2
            add = a.float() @ bb.float().t()
            view = resid.view(-1, H, W, resid.size(1))[:, ::2, ::2, :]
            view.copy_((view.float() + add.view(view.shape)).to(resid.dtype))
            return resid, torch.empty(0)
        return _reference(a, bb, pro_scale, pro_shift, resid, s2, epi, kshift, by, bscale, bshift, bmean, brelu, bnb,
                          bnb_y, mbits)
    H, W = s2 if s2 is not None else (0, 0)
    return submodule("conv_bn").c1x1(a, b, b_trans, M, pro_scale, pro_shift, resid, H, W, _EPI[epi], kshift, by,
                                     bscale, bshift, bmean, brelu, s2_scatter, bnb=bnb, bnb_y=bnb_y, mbits=mbits,
                                     lda=lda)


def c1x1_affine(a: torch.Tensor, b: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, relu: bool = True,
                r: Optional[torch.Tensor] = None, r_mul: bool = False, s2=None) -> torch.Tensor:
    """``relu?(a @ b.T * scale + shift (+ r)) (* r if r_mul)`` in one kernel (1x1 conv + bias / frozen
    BatchNorm (+ residual) (+ ReLU) (x mask)); ``s2=(H, W)`` reads the stride-2 pixels of ``a``."""
    if not a.is_cuda:
        aa = _gather_s2(a, s2) if s2 is not None else a
        y = (aa.float() @ b.float().t()) * scale + shift
        if r is not None and not r_mul:
            y = y + r.float()
        if relu:
            y = torch.relu(y)
        if r is not None and r_mul:
            y = y * r.float()
        return y.to(a.dtype)
    M = a.size(0) // 4 if s2 is not None else a.size(0)
    H, W = s2 if s2 is not None else (0, 0)
    return submodule("conv_bn").c1x1(a, b, False, M, None, None, r, H, W, _EPI["affine"], None, None, None, None,
                                     None, True, False, scale, shift, relu, r_mul)[0]


def supported(a: torch.Tensor, b: torch.Tensor, pro: bool = False, resid: bool = False, s2=None,
              epi: str = "plain", b_trans: bool = False, s2_scatter: bool = False, bnb: bool = False) -> bool:
    if not (a.is_cuda and available()):
        return False
    H, W = s2 if s2 is not None else (0, 0)
    M = a.size(0) // 4 if (s2 is not None and not s2_scatter) else a.size(0)
    return submodule("conv_bn").c1x1_supported(a, b, b_trans, M, pro, resid, H, W, _EPI[epi], s2_scatter, bnb)


def preferred(K: int, N: int, M: int, s2: bool = False) -> bool:
    """Whether the strip kernel beats hipBLASLt + a separate BatchNorm pass for a ``[M, K] x [K, N]``
    layer (microbenchmark: profiles/conv_bn_vs_unfused.jsonl). It wins the HBM-bound shapes -- both
    channel counts <= 256 on 56x56 / 28x28 pixels, and the stride-2 gather from 256 channels -- and
    loses the MFMA-bound ones (a K >= 512 layer keeps its whole weight slice in LDS, so the column
    slices get narrow and the activation is re-read per slice)."""
    if s2:  # against MIOpen's stride-2 kernel (or a strided gather + GEMM) plus the statistics pass
        return K <= 256
    return K <= 256 and N <= 256 and M >= 100000


def sum_parts(part: torch.Tensor, count: float = -1.0) -> torch.Tensor:
    """``[2N+1]`` = (sum over partial rows of both statistics, count) when ``count >= 0``, else ``[2N]``."""
    if part.is_cuda:
        return submodule("conv_bn").sum_parts(part, float(count))
    out = part.sum(1).reshape(-1)
    if count >= 0:
        out = torch.cat([out, torch.tensor([float(count)], dtype=out.dtype)])
    return out


def sum_parts_grads(part: torch.Tensor, invstd: torch.Tensor, weight: Optional[torch.Tensor], need: bool,
                    count: float = -1.0):
    """(sums, gw, gb) of a BatchNorm's backward: :func:`sum_parts` plus the parameter gradients gw = sum(dy
    x_hat) = sums[N:] * invstd and gb = sum(dy) (a separate tensor: the sums may be all-reduced in place
    later). fp32 parameters on the GPU get both from the summing launch itself; gw / gb are None when
    ``need`` is False."""
    n = part.size(2)
    if need and part.is_cuda and weight is not None and weight.dtype == torch.float32:
        sums, gw, gb = submodule("conv_bn").sum_parts_grads(part, float(count), invstd.contiguous())
        return sums, gw, gb
    sums = sum_parts(part, count)
    if not need or weight is None:
        return sums, None, None
    return sums, (sums[n:2 * n] * invstd).to(weight.dtype), sums[:n].to(weight.dtype, copy=True)


def s2_gather(x: torch.Tensor) -> torch.Tensor:
    """``x[:, :, ::2, ::2]`` of a channels_last NCHW-shaped tensor as a channels_last tensor (16-byte vector
    accesses on the GPU; torch's strided copy otherwise)."""
    if (x.is_cuda and x.dtype in (torch.float16, torch.bfloat16) and x.size(1) % 8 == 0 and x.size(2) % 2 == 0
            and x.size(3) % 2 == 0 and x.is_contiguous(memory_format=torch.channels_last)):
        return submodule("conv_bn").s2_gather(x)
    return x[:, :, ::2, ::2].contiguous(memory_format=torch.channels_last)


def s2_scatter_add(full2d: torch.Tensor, quarter2d: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    """``full[n, h, w, c]`` (as ``[n*h*w, c]``) += ``quarter`` at the even pixels, in place."""
    c = full2d.size(1)
    if (full2d.is_cuda and full2d.dtype in (torch.float16, torch.bfloat16) and c % 8 == 0 and h % 2 == 0
            and w % 2 == 0 and full2d.is_contiguous() and quarter2d.is_contiguous()
            and quarter2d.dtype == full2d.dtype):
        return submodule("conv_bn").s2_scatter_add(full2d, quarter2d, n, h, w)
    full2d.view(n, h, w, c)[:, ::2, ::2, :].add_(quarter2d.view(n, h // 2, w // 2, c))
    return full2d


def gemm_bn(a: torch.Tensor, b: torch.Tensor, epi: str = "stats", kshift=None, by=None, bscale=None, bshift=None,
            bmean=None, brelu: bool = True, resid: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``C = a @ b.T (+ resid)`` on the tiled MFMA GEMM (kernels/gemm.hip: ping-pong 256x256, 128x128 /
    256x128 / 256x256 tiles) with the same BatchNorm epilogues as :func:`c1x1` (``epi`` "plain", "stats"
    or "bwd"; partials per 64-row slab): the compute-bound 1x1 layers (K or N >= 512) that the strip
    kernel runs at low MFMA rates. ``resid`` needs ``K % 64 == 0``. Returns ``(C, part)`` (``part`` None
    for "plain")."""
    if not a.is_cuda:
        c, part = _reference(a, b, None, None, resid, None, epi, kshift, by, bscale, bshift, bmean, brelu)
        return c, (part if epi != "plain" else None)
    return tuple(submodule("conv_bn").gemm_bn(a, b, _EPI[epi], kshift, by, bscale, bshift, bmean, brelu, resid))


def gemm_bn_supported(a: torch.Tensor, b: torch.Tensor, resid: bool = False) -> bool:
    """Shapes :func:`gemm_bn` takes on the GPU: 16-bit ``a [M, K]`` / ``b [N, K]``, K % 8 == 0 (K % 64
    with a residual), N % 64 == 0."""
    K, N = a.size(1), b.size(0)
    return (a.is_cuda and available() and a.dtype in (torch.float16, torch.bfloat16) and b.dtype == a.dtype
            and K % (64 if resid else 8) == 0 and N % 64 == 0)
