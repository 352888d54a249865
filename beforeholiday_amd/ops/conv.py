"""Direct 3x3 / stride 1 / pad 1 NHWC convolution on MFMA (kernels/conv.hip, ``_C.conv_cuda``).

``conv3x3(x, w)`` runs the HIP kernel for channels_last fp16 / bf16 CUDA tensors with C and K
multiples of 64 and falls back to ``F.conv2d`` otherwise. ``conv3x3_dgrad(dy, w)`` is the data
gradient of that conv: the same kernel applied to dy with the spatially flipped, in/out-swapped
weights (for stride 1 / pad 1 dX = conv(dY, flip(W)^T)), read in place from ``w``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import available, submodule


def supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    return x.is_cuda and available() and submodule("conv_cuda").supported(x, w)


def conv3x3(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    if supported(x, w):
        return submodule("conv_cuda").conv3x3_forward(x, w)
    return F.conv2d(x, w, stride=1, padding=1)


def dgrad_weight(w: torch.Tensor) -> torch.Tensor:
    """[K, C, 3, 3] -> [C, K, 3, 3] with W'[c, k, r, s] = W[k, c, 2-r, 2-s], channels_last."""
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


def conv3x3_dgrad(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX of conv3x3(x, w) from dY: the kernel reads w in place (transposed LDS reads of the
    flipped slices); reference path conv(dY, dgrad_weight(w))."""
    if dy.is_cuda and available() and supported(dy, w.transpose(0, 1)):
        return submodule("conv_cuda").conv3x3_dgrad(dy, w)
    return F.conv2d(dy, dgrad_weight(w), stride=1, padding=1)


def wgrad_supported(x: torch.Tensor, dy: torch.Tensor, r: int, stride: int = 1) -> bool:
    return x.is_cuda and available() and submodule("conv_cuda").wgrad_supported(x, dy, r, stride)


def conv_wgrad_s2(x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """Weight gradient of a 1x1 / stride-2 convolution (the ResNet downsample) on the MFMA wgrad
    kernel, reading x at the even pixels straight from memory (no gathered copy)."""
    if wgrad_supported(x, dy, 1, 2):
        return submodule("conv_cuda").conv_wgrad(x, dy, 1, 2)
    w = torch.empty(dy.size(1), x.size(1), 1, 1, device=x.device, dtype=x.dtype)
    return torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [0, 0], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def bn_relu_apply(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor) -> torch.Tensor:
    """``relu(x * scale + shift)`` per channel (NCHW-indexed), rounded to x's dtype: the activation a
    folded BatchNorm never materialises, as the reference paths compute it."""
    s = scale.float().view(1, -1, *([1] * (x.dim() - 2)))
    b = shift.float().view(1, -1, *([1] * (x.dim() - 2)))
    return torch.relu(x.float() * s + b).to(x.dtype)


def s2_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    """The stride-2 3x3 / pad-1 kernels (kernels/conv_igemm.hip forward and data gradient,
    kernels/conv_wgrad.hip weight gradient) cover (x, w): channels_last fp16 / bf16, C and K
    multiples of 64, even H and W."""
    return x.is_cuda and available() and submodule("conv_cuda").s2_supported(x, w)


def conv3x3_s2(x: torch.Tensor, w: torch.Tensor, pro_scale: torch.Tensor = None, pro_shift: torch.Tensor = None,
               stats: bool = False, kshift: torch.Tensor = None):
    """``conv2d(x', w, stride=2, padding=1)`` on the implicit-GEMM MFMA kernel, x' = x or
    ``relu(x * pro_scale + pro_shift)`` (a BatchNorm + ReLU folded into the convolution; the padding
    stays zero). Returns ``(y, part)``: part is the [2, G, K] statistics partials of y about kshift
    when ``stats`` (empty otherwise). Fallback: ``F.conv2d`` (+ a statistics pass)."""
    if s2_supported(x, w):
        y, part = submodule("conv_cuda").conv3x3_s2_forward(x, w, pro_scale, pro_shift, stats, kshift)
        return y, part
    xin = bn_relu_apply(x, pro_scale, pro_shift) if pro_scale is not None else x
    y = F.conv2d(xin, w, stride=2, padding=1)
    part = torch.empty(0, device=x.device)
    if stats:
        yf = y.float().transpose(0, 1).reshape(y.size(1), -1)
        if kshift is not None:
            yf = yf - kshift.view(-1, 1)
        part = torch.stack([yf.sum(1), yf.square().sum(1)]).view(2, 1, -1)
    return y, part


def conv3x3_s2_dgrad(dy: torch.Tensor, w: torch.Tensor, hw) -> torch.Tensor:
    """dX [N, C, H, W] of ``conv2d(x, w, stride=2, padding=1)`` from dY: four stride-1 phase
    convolutions of dY (1, 2, 2 and 4 taps) in one launch of the implicit-GEMM kernel."""
    H, W = hw
    if dy.is_cuda and available() and H % 2 == 0 and W % 2 == 0 and dy.is_contiguous(memory_format=torch.channels_last) \
            and dy.dtype in (torch.float16, torch.bfloat16) and dy.size(1) % 64 == 0 and w.size(1) % 64 == 0:
        return submodule("conv_cuda").conv3x3_s2_dgrad(dy, w, H, W)
    x = torch.empty(dy.size(0), w.size(1), H, W, device=dy.device, dtype=dy.dtype)
    return torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                                               [True, False, False])[0]


def conv_wgrad_deferred(x: torch.Tensor, dy: torch.Tensor, r: int, pro_scale: torch.Tensor = None,
                        pro_shift: torch.Tensor = None, stride: int = 1):
    """:func:`conv_wgrad` on the MFMA kernel without its split-partials sum: ``(out, ws)``. With ``ws``
    not None, ``out`` is written only by :func:`conv_wgrad_reduce` ``(ws, out)`` -- which may run on
    another stream (models/resnet.py sums them on a side stream: nothing on the critical path waits
    for a weight gradient). Only for shapes :func:`wgrad_supported` covers."""
    out, ws = submodule("conv_cuda").conv_wgrad_deferred(x, dy, r, stride, pro_scale, pro_shift)
    return out, ws


def conv_wgrad_reduce(ws: torch.Tensor, out: torch.Tensor) -> None:
    submodule("conv_cuda").conv_wgrad_reduce(ws, out)


def conv_wgrad(x: torch.Tensor, dy: torch.Tensor, r: int, pro_scale: torch.Tensor = None,
               pro_shift: torch.Tensor = None, stride: int = 1) -> torch.Tensor:
    """Weight gradient of ``conv2d(x', w, stride, padding=(r-1)//2)`` for r in {1, 3}, where x' is x or,
    with ``pro_scale`` / ``pro_shift``, ``relu(x * pro_scale + pro_shift)`` per channel (a BatchNorm +
    ReLU folded into the convolution, applied to the staged tiles in LDS): the MFMA kernel of
    kernels/conv_wgrad.hip (both operands read through LDS transposes, fp32 split partials summed in a
    fixed order; stride 2: 1x1, or 3x3 at output widths 28 / 14 / 7) for channels_last fp16 / bf16
    with C, K multiples of 64; otherwise
    ``torch.ops.aten.convolution_backward``. Returns [K, C, r, r] (channels_last on the kernel path)."""
    if wgrad_supported(x, dy, r, stride):
        return submodule("conv_cuda").conv_wgrad(x, dy, r, stride, pro_scale, pro_shift)
    if pro_scale is not None:
        x = bn_relu_apply(x, pro_scale, pro_shift)
    w_shape = [dy.size(1), x.size(1), r, r]
    p = (r - 1) // 2
    return torch.ops.aten.convolution_backward(dy, x, torch.empty(w_shape, device=x.device, dtype=x.dtype), None,
                                               [stride, stride], [p, p], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def stem_supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    return x.is_cuda and available() and submodule("conv_cuda").stem_supported(x, w)


def stem_conv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """ResNet stem ``conv2d(x, w, stride=2, padding=3)`` (3 -> 64 channels, 224x224): the MFMA kernel of
    kernels/conv_stem.hip for channels_last fp16 / bf16, ``F.conv2d`` otherwise."""
    if stem_supported(x, w):
        return submodule("conv_cuda").stem_forward(x, w)
    return F.conv2d(x, w, stride=2, padding=3)


def stem_wgrad(x: torch.Tensor, dy: torch.Tensor) -> torch.Tensor:
    """Weight gradient of :func:`stem_conv` (kernels/conv_stem.hip, MFMA over transposed LDS reads of
    dY and of the staged input rows); ``convolution_backward`` otherwise."""
    w = torch.empty(dy.size(1), x.size(1), 7, 7, device=x.device, dtype=x.dtype)
    if stem_supported(x, w) and dy.is_contiguous(memory_format=torch.channels_last):
        return submodule("conv_cuda").stem_wgrad(x, dy)
    return torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                               [False, True, False])[1]


def gemm_n64_supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    return a.is_cuda and available() and submodule("conv_cuda").gemm_n64_supported(a, b)


def gemm_n64(a: torch.Tensor, b: torch.Tensor, resid: torch.Tensor = None) -> torch.Tensor:
    """``a @ b.t() (+ resid)`` for ``b`` of 64 rows: the streaming MFMA kernel of kernels/gemm_n64.hip
    (the 64-channel side of the 56x56 1x1 convolutions), torch.mm elsewhere."""
    if gemm_n64_supported(a, b):
        return submodule("conv_cuda").gemm_n64(a, b, resid)
    out = torch.mm(a, b.t())
    return out if resid is None else out.add_(resid)
