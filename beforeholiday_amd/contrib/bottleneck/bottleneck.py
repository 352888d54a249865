"""ResNet bottleneck block with frozen BN, fused epilogues, optional spatial (H-split) parallelism
(reference: apex/contrib/bottleneck/bottleneck.py:15-760, cuDNN-frontend fused kernels).

Every conv + frozen-BN scale / bias (+ residual) + ReLU is ONE MFMA kernel with an affine epilogue
(contrib/conv_bias_relu: the 1x1 strip GEMM, the direct 3x3 convolution); other shapes fall back to
torch conv2d + one epilogue pass.

``SpatialBottleneck`` splits H over ``spatial_group_size`` ranks. Its 3x3 convolution
(:class:`_SpatialConv3x3`) never concatenates a padded copy: the halo rows travel on a side HIP stream
(any exchanger of ``halo_exchangers``) while the compute stream runs the whole local convolution with
zero padding; once the halos land, only the two boundary output rows are recomputed, from 3-row strips
(reference: the interior conv + ``bottleneck_forward_out2_halo`` split, bottleneck.cpp:3113-3176). The
backward likewise runs the local data / weight gradients while the boundary rows of the output gradient
travel, then adds the halo terms -- the neighbours' output-gradient rows into this rank's boundary input
rows, and the halo input rows' products into the weight gradient -- from strip-sized kernels
(reference: the backward halo variants, bottleneck.cpp:3700-3777). ``explicit_nhwc=True`` takes and
returns physical [N, H, W, C] tensors (viewed as channels_last NCHW without copies).
"""
import torch
import torch.distributed as dist
from torch import nn

from ...ops import syncbn as _bn
from ..conv_bias_relu.conv_bias_relu import (ConvFrozenScaleBias, ConvFrozenScaleBiasAddReLU,
                                             ConvFrozenScaleBiasReLU, _dpre, conv_affine, conv_grads)
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


def _row_block(t, i):
    """Row ``i`` of an NCHW-indexed tensor as a contiguous [N, 1, W, C] block (the exchangers' unit)."""
    return t[:, :, i:i + 1].permute(0, 2, 3, 1).contiguous()


def _from_block(b, like):
    """[N, 1, W, C] block -> [N, C, 1, W] in ``like``'s dtype / memory format."""
    t = b.permute(0, 3, 1, 2).to(like.dtype)
    return t.contiguous(memory_format=torch.channels_last) if like.is_contiguous(
        memory_format=torch.channels_last) else t.contiguous()


class _SideExchange(object):
    """One halo exchange issued on a side HIP stream (the compute stream keeps running); ``wait()``
    makes the compute stream wait for it and returns (from_left, from_right) [N, 1, W, C] blocks.
    CPU tensors (gloo tests) exchange synchronously."""

    _streams = {}

    def __init__(self, halo_ex, top, bot):
        self.cuda = top.is_cuda
        if not self.cuda:
            self.out = halo_ex.left_right_halo_exchange(top, bot)
            return
        dev = top.device
        side = self._streams.get(dev)
        if side is None:
            side = self._streams[dev] = torch.cuda.Stream(device=dev)
        self.side = side
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self.out = halo_ex.left_right_halo_exchange(top, bot)
        for t in (top, bot):
            t.record_stream(side)

    def wait(self):
        if self.cuda:
            torch.cuda.current_stream(self.out[0].device).wait_stream(self.side)
            for t in self.out:
                t.record_stream(torch.cuda.current_stream(t.device))
        return self.out


def _strips(rows_a, rows_b, rows_c):
    """Stack 3-row strips [a; b; c] (each [N, C, 1, W]) -> [N, C, 3, W] in a's memory format."""
    s = torch.cat([rows_a, rows_b, rows_c], dim=2)
    return s.contiguous(memory_format=torch.channels_last) if rows_b.is_contiguous(
        memory_format=torch.channels_last) else s


def _dgrad3(dy, wx):
    from ...ops import conv as _conv

    if dy.is_cuda and dy.dtype in (torch.float16, torch.bfloat16) and _conv.supported(dy, wx.transpose(0, 1)):
        return _conv.conv3x3_dgrad(dy.contiguous(memory_format=torch.channels_last), wx)
    return torch.nn.grad.conv2d_input((dy.size(0), wx.size(1), dy.size(2), dy.size(3)), wx, dy, padding=1)


def _wgrad3(x, dy, w):
    from ...ops import conv as _conv

    if _conv.wgrad_supported(x, dy, 3):
        return _conv.conv_wgrad(x, dy, 3).to(w.dtype)
    return torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1)


class _SpatialConv3x3(torch.autograd.Function):
    """``relu(conv3x3(x, w) * scale + bias)`` (stride 1, pad 1, frozen scale / bias) of an H-split
    activation: x holds this rank's rows, the rows above / below live on the left / right neighbour."""

    @staticmethod
    def forward(ctx, x, w, scale, bias, halo_ex):
        H = x.size(2)
        if H < 2:
            raise RuntimeError("SpatialBottleneck: each rank needs at least 2 rows of the split dimension")
        ex = _SideExchange(halo_ex, _row_block(x, 0), _row_block(x, H - 1))
        # the local convolution, zero padded: correct except output rows 0 and H-1 (halo terms missing)
        y = conv_affine(x, w, scale, bias, True, 1, 1)
        from_left, from_right = ex.wait()
        li, ri = _from_block(from_left, x), _from_block(from_right, x)
        fix = []  # (output row, strip) of the boundary rows that have a real neighbour
        if not halo_ex.left_zero:
            fix.append((0, _strips(li, x[:, :, 0:1], x[:, :, 1:2])))
        if not halo_ex.right_zero:
            fix.append((H - 1, _strips(x[:, :, H - 2:H - 1], x[:, :, H - 1:H], ri)))
        if fix:
            ys = conv_affine(torch.cat([s for _, s in fix], dim=0), w, scale, bias, True, 1, 1)
            n = x.size(0)
            for j, (row, _) in enumerate(fix):
                y[:, :, row] = ys[j * n:(j + 1) * n, :, 1]
        ctx.save_for_backward(x, w, scale, y, li, ri)
        ctx.halo_ex = halo_ex
        return y

    @staticmethod
    def backward(ctx, g):
        x, w, scale, y, li, ri = ctx.saved_tensors
        ex_h = ctx.halo_ex
        H, n = x.size(2), x.size(0)
        dpre, _ = _dpre(g, y, True, False)
        # the neighbours need my boundary rows of the output gradient: they travel while the local
        # data / weight gradients run
        ex = _SideExchange(ex_h, _row_block(dpre, 0), _row_block(dpre, H - 1))
        gx, gw = conv_grads(x, w, dpre, 1, 1, scale=scale, need_x=ctx.needs_input_grad[0])
        # weight gradient halo terms: dpre row 0 x the row above (kernel row 0), dpre row H-1 x the row
        # below (kernel row 2) -- 3-row strips where only those products survive
        xs, dys = [], []
        zx, zd = torch.zeros_like(x[:, :, 0:1]), torch.zeros_like(dpre[:, :, 0:1])
        if not ex_h.left_zero:
            xs.append(_strips(li, zx, zx))
            dys.append(_strips(zd, dpre[:, :, 0:1], zd))
        if not ex_h.right_zero:
            xs.append(_strips(zx, zx, ri))
            dys.append(_strips(zd, dpre[:, :, H - 1:H], zd))
        if xs:
            gh = _wgrad3(torch.cat(xs, 0), torch.cat(dys, 0), w)
            gw = gw + gh * scale.reshape(-1, 1, 1, 1).to(gh.dtype)
        from_left, from_right = ex.wait()
        if gx is not None:
            # input rows 0 / H-1 also fed the neighbours' boundary output rows: their output-gradient rows
            # through kernel row 2 (from the left) / row 0 (from the right)
            wx = (w.float() * scale.float().reshape(-1, 1, 1, 1)).to(w.dtype)
            wx = wx.contiguous(memory_format=torch.channels_last) if w.is_contiguous(
                memory_format=torch.channels_last) else wx
            dl, dr = _from_block(from_left, dpre), _from_block(from_right, dpre)
            ds, rows = [], []
            if not ex_h.left_zero:
                ds.append(_strips(dl, zd, zd))
                rows.append(0)
            if not ex_h.right_zero:
                ds.append(_strips(zd, zd, dr))
                rows.append(H - 1)
            if ds:
                gs = _dgrad3(torch.cat(ds, 0), wx)
                for j, row in enumerate(rows):
                    gx[:, :, row] += gs[j * n:(j + 1) * n, :, 1]
        if gw.stride() != w.stride():
            gw = gw.contiguous(memory_format=torch.channels_last) if w.is_contiguous(
                memory_format=torch.channels_last) else gw.contiguous()
        return gx, gw, None, None, None


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
        s2, b2 = self.bn2.get_scale_bias()
        w = self.conv2.weight
        if out.is_cuda and torch.is_autocast_enabled("cuda"):
            out, w = out.half(), w.half()  # (the fused convs' custom_fwd(cast_inputs=torch.half))
        return _SpatialConv3x3.apply(out, w.to(out.dtype), s2, b2, self.halo_ex)
