"""FusedLayerNorm / FusedRMSNorm and mixed-dtype variants (reference:
apex/normalization/fused_layer_norm.py:32-437).

Autograd functions call ``ops.fused_layer_norm_cuda`` (HIP kernels on GPU, fp32 PyTorch on CPU).
``memory_efficient=True`` saves the OUTPUT instead of the input and recomputes x_hat from it in the
backward. Under autocast, inputs/params are cast to the autocast dtype first (``_cast_if_autocast_enabled``).
"""
from __future__ import annotations

import numbers

import torch
from torch.nn import init
from torch.nn.parameter import Parameter

from .._autocast_utils import _cast_if_autocast_enabled
from ..ops import fused_layer_norm_cuda as _ln


def manual_rms_norm(input, normalized_shape, weight, eps):
    """Reference RMSNorm in fp32 (the reference's version reads ``self.weight`` in a free
    function; fixed here)."""
    dims = tuple(i for i in range(-1, -len(normalized_shape) - 1, -1))
    variance = input.to(torch.float32).pow(2).mean(dims, keepdim=True)
    input = input * torch.rsqrt(variance + eps)
    if weight is None:
        return input
    if weight.dtype in (torch.float16, torch.bfloat16):
        input = input.to(weight.dtype)
    return weight * input


class FusedLayerNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        bias_ = bias.contiguous()
        output, mean, invvar = _ln.forward_affine(input_, ctx.normalized_shape, weight_, bias_, ctx.eps)
        if memory_efficient:
            ctx.save_for_backward(output, weight_, bias_, None, invvar)
        else:
            ctx.save_for_backward(input_, weight_, bias_, mean, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        input_or_output, weight_, bias_, mean, invvar = ctx.saved_tensors
        grad_input, grad_weight, grad_bias = _ln.backward_affine(
            grad_output.contiguous(), mean, invvar, input_or_output, ctx.normalized_shape, weight_, bias_, ctx.eps,
            ctx.memory_efficient)
        return grad_input, grad_weight, grad_bias, None, None, None


class FusedRMSNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        output, invvar = _ln.rms_forward_affine(input_, ctx.normalized_shape, weight_, ctx.eps)
        ctx.save_for_backward(output if memory_efficient else input_, weight_, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        input_or_output, weight_, invvar = ctx.saved_tensors
        grad_input, grad_weight = _ln.rms_backward_affine(grad_output.contiguous(), invvar, input_or_output,
                                                          ctx.normalized_shape, weight_, ctx.eps, ctx.memory_efficient)
        return grad_input, grad_weight, None, None, None


class FusedLayerNormAffineMixedDtypesFunction(FusedLayerNormAffineFunction):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        bias_ = bias.contiguous()
        output, mean, invvar = _ln.forward_affine_mixed_dtypes(input_, ctx.normalized_shape, weight_, bias_, ctx.eps)
        if memory_efficient:
            ctx.save_for_backward(output, weight_, bias_, None, invvar)
        else:
            ctx.save_for_backward(input_, weight_, bias_, mean, invvar)
        return output


class FusedRMSNormAffineMixedDtypesFunction(FusedRMSNormAffineFunction):
    @staticmethod
    def forward(ctx, input, weight, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        weight_ = weight.contiguous()
        output, invvar = _ln.rms_forward_affine_mixed_dtypes(input_, ctx.normalized_shape, weight_, ctx.eps)
        ctx.save_for_backward(output if memory_efficient else input_, weight_, invvar)
        return output


class FusedLayerNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        output, mean, invvar = _ln.forward(input_, ctx.normalized_shape, ctx.eps)
        if memory_efficient:
            ctx.save_for_backward(output, None, invvar)
        else:
            ctx.save_for_backward(input_, mean, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        input_or_output, mean, invvar = ctx.saved_tensors
        grad_input = _ln.backward(grad_output.contiguous(), mean, invvar, input_or_output, ctx.normalized_shape,
                                  ctx.eps, ctx.memory_efficient)
        return grad_input, None, None, None


class FusedRMSNormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, normalized_shape, eps, memory_efficient=False):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        input_ = input.contiguous()
        output, invvar = _ln.rms_forward(input_, ctx.normalized_shape, ctx.eps)
        ctx.save_for_backward(output if memory_efficient else input_, invvar)
        return output

    @staticmethod
    def backward(ctx, grad_output):
        input_or_output, invvar = ctx.saved_tensors
        grad_input = _ln.rms_backward(grad_output.contiguous(), invvar, input_or_output, ctx.normalized_shape,
                                      ctx.eps, ctx.memory_efficient)
        return grad_input, None, None, None


def fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, weight, bias, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedLayerNormAffineFunction.apply(*args)


def fused_layer_norm(input, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedLayerNormFunction.apply(*args)


def mixed_dtype_fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, weight, bias, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedLayerNormAffineMixedDtypesFunction.apply(*args)


def fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, weight, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedRMSNormAffineFunction.apply(*args)


def fused_rms_norm(input, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedRMSNormFunction.apply(*args)


def mixed_dtype_fused_rms_norm_affine(input, weight, normalized_shape, eps=1e-6, memory_efficient=False):
    args = _cast_if_autocast_enabled(input, weight, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedRMSNormAffineMixedDtypesFunction.apply(*args)


def _shape(normalized_shape):
    if isinstance(normalized_shape, numbers.Integral):
        normalized_shape = (normalized_shape,)
    return torch.Size(normalized_shape)


class FusedLayerNorm(torch.nn.Module):
    """LayerNorm over the trailing ``normalized_shape`` dims, fused forward/backward kernels.

    Same constructor as ``torch.nn.LayerNorm`` (plus ``memory_efficient``); the CPU path runs the same
    math through the PyTorch reference implementation."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, memory_efficient=False):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        self.memory_efficient = memory_efficient
        if self.elementwise_affine:
            self.weight = Parameter(torch.empty(*self.normalized_shape))
            self.bias = Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)
            init.zeros_(self.bias)

    def forward(self, input):
        if self.elementwise_affine:
            return fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps,
                                           self.memory_efficient)
        return fused_layer_norm(input, self.normalized_shape, self.eps, self.memory_efficient)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class FusedRMSNorm(torch.nn.Module):
    """RMSNorm (x / sqrt(mean(x^2) + eps) * weight) with fused kernels."""

    def __init__(self, normalized_shape, eps=1e-5, elementwise_affine=True, memory_efficient=False):
        super().__init__()
        self.normalized_shape = _shape(normalized_shape)
        self.eps = eps
        self.elementwise_affine = elementwise_affine
        self.memory_efficient = memory_efficient
        if self.elementwise_affine:
            self.weight = Parameter(torch.empty(*self.normalized_shape))
        else:
            self.register_parameter("weight", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.elementwise_affine:
            init.ones_(self.weight)

    def forward(self, input):
        if self.elementwise_affine:
            return fused_rms_norm_affine(input, self.weight, self.normalized_shape, self.eps, self.memory_efficient)
        return fused_rms_norm(input, self.normalized_shape, self.eps, self.memory_efficient)

    def extra_repr(self):
        return "{normalized_shape}, eps={eps}, elementwise_affine={elementwise_affine}".format(**self.__dict__)


class MixedFusedLayerNorm(FusedLayerNorm):
    """Output dtype follows the parameters (e.g. fp32 params on a bf16 input -> fp32 output)."""

    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        if "elementwise_affine" in kwargs:
            import warnings

            warnings.warn("MixedFusedLayerNorm does not support `elementwise_affine` argument")
            if not kwargs.pop("elementwise_affine"):
                raise RuntimeError("MixedFusedLayerNorm does not support `elementwise_affine = False`")
        super().__init__(normalized_shape=normalized_shape, eps=eps, elementwise_affine=True, **kwargs)

    def forward(self, input: torch.Tensor):
        return mixed_dtype_fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps,
                                                   self.memory_efficient)


class MixedFusedRMSNorm(FusedRMSNorm):
    def __init__(self, normalized_shape, eps=1e-5, **kwargs):
        if "elementwise_affine" in kwargs:
            import warnings

            warnings.warn("MixedFusedRMSNorm does not support `elementwise_affine` argument")
            if not kwargs.pop("elementwise_affine"):
                raise RuntimeError("MixedFusedRMSNorm does not support `elementwise_affine = False`")
        super().__init__(normalized_shape=normalized_shape, eps=eps, elementwise_affine=True, **kwargs)

    def forward(self, input: torch.Tensor):
        return mixed_dtype_fused_rms_norm_affine(input, self.weight, self.normalized_shape, self.eps,
                                                 self.memory_efficient)
