"""Conv + bias (+ mask) (+ ReLU) with fused epilogues (reference: apex/contrib/conv_bias_relu/conv_bias_relu.py,
cuDNN-frontend fusions).

The convolution runs on MIOpen (torch conv2d); the epilogue (per-channel scale/bias, optional
mask, ReLU) is one pass of the channel-owned BN-apply kernel (kernels/batchnorm.hip via
``ops.syncbn.forward``), and the backward's ReLU mask + bias-gradient reduction is one pass of
the dense epilogue kernel over the channels_last [N*H*W, C] view (kernels/dense.hip).
Inputs are cast to fp16 under autocast like the reference's ``custom_fwd(cast_inputs=torch.half)``.
"""
import torch
import torch.nn.functional as F

from ...ops import fused_dense as _fd
from ...ops import syncbn as _bn


def _as_rows(t):
    """[N, C, H, W] channels_last -> [N*H*W, C] view (no copy)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.size(1))


def _bias_relu_bwd(grad, y, relu, need_bias):
    g = grad.contiguous(memory_format=torch.channels_last)
    y = y.contiguous(memory_format=torch.channels_last)
    rows = _as_rows(g)
    dx, db = _fd.act_backward(rows, _as_rows(y), _fd.ACT_RELU if relu else _fd.ACT_NONE, need_bias)
    dpre = dx.view(g.size(0), g.size(2), g.size(3), g.size(1)).permute(0, 3, 1, 2)
    return dpre, db


def _conv_grads(x, w, dpre, padding, stride):
    gx = torch.nn.grad.conv2d_input(x.shape, w, dpre, stride=stride, padding=padding)
    gw = torch.nn.grad.conv2d_weight(x, w.shape, dpre, stride=stride, padding=padding)
    return gx, gw


class ConvBiasReLU_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, padding, stride):
        c = F.conv2d(x, weight, None, stride, padding)
        ones = torch.ones(c.size(1), device=c.device, dtype=torch.float32)
        y = _bn.forward(c, None, ones, bias.float().reshape(-1), True)
        ctx.save_for_backward(x, weight, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, y = ctx.saved_tensors
        dpre, db = _bias_relu_bwd(grad_output, y, True, True)
        gx, gw = _conv_grads(x, w, dpre, ctx.padding, ctx.stride)
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None


class ConvBiasMaskReLU_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, mask, padding, stride):
        c = F.conv2d(x, weight, None, stride, padding)
        ones = torch.ones(c.size(1), device=c.device, dtype=torch.float32)
        y = _bn.forward(c, None, ones, bias.float().reshape(-1), True) * mask.to(c.dtype)
        ctx.save_for_backward(x, weight, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, y = ctx.saved_tensors
        dpre, db = _bias_relu_bwd(grad_output, y, True, True)  # y == 0 where masked or ReLU-clipped
        gx, gw = _conv_grads(x, w, dpre, ctx.padding, ctx.stride)
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None, None


class ConvBias_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, padding, stride):
        ctx.save_for_backward(x, weight)
        ctx.padding, ctx.stride = padding, stride
        return F.conv2d(x, weight, bias.reshape(-1), stride, padding)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w = ctx.saved_tensors
        dpre, db = _bias_relu_bwd(grad_output, grad_output, False, True)
        gx, gw = _conv_grads(x, w, dpre, ctx.padding, ctx.stride)
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None


class ConvFrozenScaleBiasReLU_(torch.autograd.Function):
    """relu(conv(x, w) * scale + bias) with frozen (non-trainable) per-channel scale / bias."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, scale, bias, padding, stride):
        c = F.conv2d(x, weight, None, stride, padding)
        y = _bn.forward(c, None, scale.float().reshape(-1), bias.float().reshape(-1), True)
        ctx.save_for_backward(x, weight, scale, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, scale, y = ctx.saved_tensors
        dpre, _ = _bias_relu_bwd(grad_output, y, True, False)
        dpre = dpre * scale.reshape(1, -1, 1, 1).to(dpre.dtype)
        gx, gw = _conv_grads(x, w, dpre, ctx.padding, ctx.stride)
        return gx, gw, None, None, None, None


ConvBiasReLU = ConvBiasReLU_.apply
ConvBiasMaskReLU = ConvBiasMaskReLU_.apply
ConvBias = ConvBias_.apply
ConvFrozenScaleBiasReLU = ConvFrozenScaleBiasReLU_.apply
