"""ResNet bottleneck block with frozen BN, fused epilogues, optional spatial (H-split) parallelism
(reference: apex/contrib/bottleneck/bottleneck.py:15-760, cuDNN-frontend fused kernels).

conv (MIOpen) + frozen-BN scale/bias (+ residual) + ReLU epilogues run as single fused passes of
the BN-apply kernel (kernels/batchnorm.hip). ``SpatialBottleneck`` splits H over
``spatial_group_size`` ranks and exchanges one halo row before the 3x3 convolution (and the halo
gradients in backward) with an exchanger from ``halo_exchangers``. ``explicit_nhwc=True`` takes
and returns physical [N, H, W, C] tensors (viewed as channels_last NCHW without copies).
"""
import torch
import torch.distributed as dist
from torch import nn

from ...ops import syncbn as _bn
from ..conv_bias_relu.conv_bias_relu import (ConvFrozenScaleBias, ConvFrozenScaleBiasAddReLU,
                                             ConvFrozenScaleBiasReLU)
from .halo_exchangers import HaloExchangerSendRecv


def kaiming_uniform_(tensor, a=0, mode="fan_in", nonlinearity="leaky_relu"):
    return nn.init.kaiming_uniform_(tensor, a=a, mode=mode, nonlinearity=nonlinearity)


class FrozenBatchNorm2d(nn.Module):
    """BatchNorm2d with fixed statistics and affine parameters: y = x * scale + bias."""

    def __init__(self, n):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))

    def get_scale_bias(self, nhwc=False):
        scale = self.weight * self.running_var.rsqrt()
        bias = self.bias - self.running_mean * scale
        if nhwc:
            return scale.reshape(1, 1, 1, -1), bias.reshape(1, 1, 1, -1)
        return scale.reshape(1, -1, 1, 1), bias.reshape(1, -1, 1, 1)

    def forward(self, x):
        scale, bias = self.get_scale_bias(False)
        return x * scale.to(x.dtype) + bias.to(x.dtype)


def compute_scale_bias_one(nhwc, weight, bias, running_mean, running_var, w_scale, w_bias):
    scale = weight * running_var.rsqrt()
    b = bias - running_mean * scale
    w_scale.copy_(scale.view_as(w_scale))
    w_bias.copy_(b.view_as(w_bias))


class _ScaleBiasAddReLU(torch.autograd.Function):
    """relu(x * scale + bias + z) in one pass; frozen scale / bias."""

    @staticmethod
    def forward(ctx, x, scale, bias, z):
        y = _bn.forward(x, z, scale.float().reshape(-1), bias.float().reshape(-1), True)
        ctx.save_for_backward(scale, y)
        return y

    @staticmethod
    def backward(ctx, g):
        scale, y = ctx.saved_tensors
        gz = g * (y > 0).to(g.dtype)
        return gz * scale.reshape(1, -1, 1, 1).to(g.dtype), None, None, gz


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation, groups=groups, bias=False,
                     dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class Bottleneck(nn.Module):
    """1x1 (stride) -> 3x3 -> 1x1 with frozen BN, residual, ReLU (ResNet v1 stride placement)."""

    def __init__(self, in_channels, bottleneck_channels, out_channels, stride=1, groups=1, dilation=1,
                 norm_func=None, use_cudnn=False, explicit_nhwc=False):
        super().__init__()
        if groups != 1:
            raise RuntimeError("Only support groups == 1")
        if dilation != 1:
            raise RuntimeError("Only support dilation == 1")
        if norm_func is not None:
            raise RuntimeError("Only support frozen BN now.")
        norm_func = FrozenBatchNorm2d
        self.downsample = (nn.Sequential(conv1x1(in_channels, out_channels, stride), norm_func(out_channels))
                           if stride != 1 or in_channels != out_channels else None)
        self.conv1 = conv1x1(in_channels, bottleneck_channels, stride)
        self.conv2 = conv3x3(bottleneck_channels, bottleneck_channels)
        self.conv3 = conv1x1(bottleneck_channels, out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.stride = stride
        self.bn1 = norm_func(bottleneck_channels)
        self.bn2 = norm_func(bottleneck_channels)
        self.bn3 = norm_func(out_channels)
        self.use_cudnn = use_cudnn
        self.explicit_nhwc = explicit_nhwc
        self.w_conv = [self.conv1.weight, self.conv2.weight, self.conv3.weight]
        if self.downsample is not None:
            self.w_conv.append(self.downsample[0].weight)
        for w in self.w_conv:
            kaiming_uniform_(w, a=1)

    def _to_nchw(self, x):
        return x.permute(0, 3, 1, 2) if self.explicit_nhwc else x

    def _from_nchw(self, y):
        return y.permute(0, 2, 3, 1) if self.explicit_nhwc else y

    def _conv2(self, out):
        s2, b2 = self.bn2.get_scale_bias()
        return ConvFrozenScaleBiasReLU(out, self.conv2.weight, s2, b2, 1, 1)

    def forward(self, x):
        # every conv + frozen BN (+ residual) + ReLU is ONE kernel (conv_bias_relu's affine epilogues on the
        # MFMA 1x1 / 3x3 convolutions) where the shape is covered, MIOpen + one epilogue pass otherwise
        x = self._to_nchw(x)
        s1, b1 = self.bn1.get_scale_bias()
        out = ConvFrozenScaleBiasReLU(x, self.conv1.weight, s1, b1, 0, self.stride)
        out = self._conv2(out)
        if self.downsample is not None:
            sd, bd = self.downsample[1].get_scale_bias()
            identity = ConvFrozenScaleBias(x, self.downsample[0].weight, sd, bd, 0, self.stride)
        else:
            identity = x
        s3, b3 = self.bn3.get_scale_bias()
        y = ConvFrozenScaleBiasAddReLU(out, self.conv3.weight, s3, b3, identity.to(out.dtype), 0, 1)
        return self._from_nchw(y)


class _HaloPad(torch.autograd.Function):
    """Concatenate neighbour halo rows along H (dim 2); backward returns the halo gradients to the
    ranks that own those rows."""

    @staticmethod
    def forward(ctx, y, halo_ex, h):
        ctx.halo_ex, ctx.h = halo_ex, h
        top, bot = y[:, :, :h], y[:, :, -h:]
        li, ri = halo_ex.left_right_halo_exchange(top.contiguous(), bot.contiguous())
        out = torch.cat([li.to(y.dtype), y, ri.to(y.dtype)], dim=2)
        return out.contiguous(memory_format=torch.channels_last) if y.is_contiguous(
            memory_format=torch.channels_last) else out

    @staticmethod
    def backward(ctx, g):
        h = ctx.h
        g_mid = g[:, :, h:-h].clone()
        g_top_halo, g_bot_halo = g[:, :, :h].contiguous(), g[:, :, -h:].contiguous()
        # my top halo came from the left neighbour's bottom rows (and vice versa): send them back
        from_left, from_right = ctx.halo_ex.left_right_halo_exchange(g_top_halo, g_bot_halo)
        if not ctx.halo_ex.left_zero:
            g_mid[:, :, :h] += from_left.to(g.dtype)
        if not ctx.halo_ex.right_zero:
            g_mid[:, :, -h:] += from_right.to(g.dtype)
        return g_mid, None, None


class SpatialBottleneck(Bottleneck):
    """Bottleneck whose activations are split along H over ``spatial_group_size`` consecutive ranks."""

    def __init__(self, in_channels, bottleneck_channels, out_channels, stride=1, groups=1, dilation=1,
                 norm_func=None, use_cudnn=False, explicit_nhwc=False, spatial_parallel_args=None):
        super().__init__(in_channels, bottleneck_channels, out_channels, stride, groups, dilation, norm_func,
                         use_cudnn, explicit_nhwc)
        if spatial_parallel_args is None:
            self.spatial_group_size, self.spatial_group_rank, self.halo_ex = 1, 0, None
        else:
            size, rank, comm, halo_ex = spatial_parallel_args[:4]
            self.spatial_group_size, self.spatial_group_rank = size, rank
            self.halo_ex = halo_ex
        if self.spatial_group_size > 1 and self.halo_ex is None:
            g = dist.get_rank() // self.spatial_group_size * self.spatial_group_size
            self.halo_ex = HaloExchangerSendRecv(list(range(g, g + self.spatial_group_size)), self.spatial_group_rank)

    def _conv2(self, out):
        if self.spatial_group_size <= 1:
            return super()._conv2(out)
        padded = _HaloPad.apply(out, self.halo_ex, 1)
        s2, b2 = self.bn2.get_scale_bias()
        return ConvFrozenScaleBiasReLU(padded, self.conv2.weight, s2, b2, (0, 1), 1)
