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


class ResidualGradLink(object):
    """Pairs a pre-LN block's LayerNorm with the bias-dropout-add that takes the LayerNorm's INPUT as its
    residual (models/transformer_lm.py ``ParallelTransformerLayer``). The add's backward parks its residual
    gradient here instead of returning it, and the LayerNorm backward adds it inside its dx kernel: autograd
    then never sums the two branch gradients of that input in a separate pass (the reference's fused
    norm-add LayerNorm backward, apex/contrib/csrc/multihead_attn/layer_norm.cuh:474,566,603).

    ``armed`` is set by the add's forward (only its native path parks gradients); the LayerNorm backward
    raises if an armed link holds no gradient (the add's backward did not run first), so a changed graph
    fails loudly instead of dropping the residual gradient."""

    __slots__ = ("armed", "g")

    def __init__(self):
        self.armed, self.g = False, None

    def take(self):
        if not self.armed:
            return None
        g, self.g, self.armed = self.g, None, False
        if g is None:
            raise RuntimeError("ResidualGradLink: the residual add's backward did not run before the LayerNorm's")
        return g


class FusedLayerNormAffineFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, normalized_shape, eps, memory_efficient=False, resid_link=None):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        ctx.resid_link = resid_link
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
        link = getattr(ctx, "resid_link", None)
        dres = link.take() if link is not None else None
        grad_input, grad_weight, grad_bias = _ln.backward_affine(
            grad_output.contiguous(), mean, invvar, input_or_output, ctx.normalized_shape, weight_, bias_, ctx.eps,
            ctx.memory_efficient, dres)
        # (as many gradients as inputs: callers that do not pass resid_link apply six)
        return (grad_input, grad_weight, grad_bias, None, None, None, None)[:len(ctx.needs_input_grad)]


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
    def forward(ctx, input, weight, bias, normalized_shape, eps, memory_efficient=False, resid_link=None):
        ctx.normalized_shape = normalized_shape
        ctx.eps = eps
        ctx.memory_efficient = memory_efficient
        ctx.resid_link = resid_link
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


def fused_layer_norm_affine(input, weight, bias, normalized_shape, eps=1e-6, memory_efficient=False, resid_link=None):
    args = _cast_if_autocast_enabled(input, weight, bias, normalized_shape, eps, memory_efficient)
    with torch.amp.autocast("cuda", enabled=False):
        return FusedLayerNormAffineFunction.apply(*args, resid_link)


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

    def forward(self, input, resid_link=None):
        """``resid_link`` (:class:`ResidualGradLink`, affine only): the residual add that takes ``input``
        parks its gradient there and this backward adds it inside the dx kernel."""
        if self.elementwise_affine:
            return fused_layer_norm_affine(input, self.weight, self.bias, self.normalized_shape, self.eps,
                                           self.memory_efficient, resid_link)
        assert resid_link is None, "resid_link needs the affine LayerNorm"
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
