"""Conv + bias (+ mask) (+ ReLU) fusions (reference: apex/contrib/conv_bias_relu/conv_bias_relu.py and
the cuDNN-frontend graphs of apex/contrib/csrc/conv_bias_relu/conv_bias_relu.cpp:1280-1400).

MI355X design -- one kernel per forward for the ResNet-shaped convolutions:

* 1x1 (stride 1 or 2, no padding): the strip MFMA GEMM of kernels/conv_bn.hip with its affine
  epilogue, ``relu?(conv * scale + bias (+ r)) (* r)``;
* 3x3 / stride 1 / padding 1: the direct MFMA convolution of kernels/conv.hip with the same epilogue;
* anything else: MIOpen (torch conv2d) + the BN-apply pass (kernels/batchnorm.hip).

Backward: one pass of the dense epilogue kernel (kernels/dense.hip) gives the ReLU-masked gradient
and the bias gradient; the data and weight gradients then run on the MFMA kernels (1x1 data gradient
with the weight read transposed in place, stride-2 as a scatter into a zeroed input gradient, the
flipped-weight 3x3 data gradient, the MFMA wgrad kernels); a frozen scale is folded into the weights
of the data gradient and into the weight gradient's rows instead of scaling the activation.
Inputs are cast to fp16 under autocast like the reference's ``custom_fwd(cast_inputs=torch.half)``.
"""
import torch
import torch.nn.functional as F

from ...ops import conv as _conv
from ...ops import conv_bn as _cbn
from ...ops import fused_dense as _fd
from ...ops import syncbn as _bn


def _as_rows(t):
    """[N, C, H, W] channels_last -> [N*H*W, C] view (no copy)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.size(1))


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def _kind(x, w, padding, stride):
    """Which own kernel covers conv2d(x, w, padding, stride): "1x1", "1x1s2", "3x3" or None."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float16, torch.bfloat16) and w.dtype == x.dtype
            and x.is_contiguous(memory_format=torch.channels_last)):
        return None
    p, s = _pair(padding), _pair(stride)
    k, c = w.size(0), w.size(1)
    if w.shape[2:] == (1, 1) and p == (0, 0) and s in ((1, 1), (2, 2)):
        s2 = s == (2, 2)
        if s2 and (x.size(2) % 2 or x.size(3) % 2):
            return None
        a = _as_rows(x)
        ok = _cbn.supported(a, w.view(k, c), resid=True, s2=(x.size(2), x.size(3)) if s2 else None, epi="affine")
        return ("1x1s2" if s2 else "1x1") if ok else None
    if w.shape[2:] == (3, 3) and p == (1, 1) and s == (1, 1) and _conv.supported(x, w):
        return "3x3"
    return None


def _r_rows(r, like):
    if r is None:
        return None
    r = r.to(like.dtype).contiguous(memory_format=torch.channels_last)
    return r


def conv_affine(x, w, scale, shift, relu, padding, stride, r=None, r_mul=False):
    """``relu?(conv2d(x, w) * scale + shift (+ r)) (* r if r_mul)``: one kernel when the shape is covered."""
    kind = _kind(x, w, padding, stride)
    scale = scale.float().reshape(-1).contiguous()
    shift = shift.float().reshape(-1).contiguous()
    n, c, h, wd = x.shape
    k = w.size(0)
    if kind in ("1x1", "1x1s2"):
        s2 = kind == "1x1s2"
        ho, wo = (h // 2, wd // 2) if s2 else (h, wd)
        rr = _r_rows(r, x)
        y2d = _cbn.c1x1_affine(_as_rows(x), w.reshape(k, c), scale, shift, relu,
                               _as_rows(rr) if rr is not None else None, r_mul, s2=(h, wd) if s2 else None)
        return y2d.view(n, ho, wo, k).permute(0, 3, 1, 2)
    if kind == "3x3":
        from ..._native import submodule

        rr = _r_rows(r, x)
        return submodule("conv_cuda").conv3x3_affine(x, w, scale, shift, relu, rr, r_mul)
    c_out = F.conv2d(x, w, None, stride, padding)
    if r is not None and r_mul:
        return _bn.forward(c_out, None, scale, shift, relu) * r.to(c_out.dtype)
    return _bn.forward(c_out, r.to(c_out.dtype) if r is not None else None, scale, shift, relu)


def _dpre(grad, y, relu, need_bias):
    """ReLU-masked gradient and bias gradient in one pass (kernels/dense.hip)."""
    g = grad.contiguous(memory_format=torch.channels_last)
    y = y.contiguous(memory_format=torch.channels_last)
    dx, db = _fd.act_backward(_as_rows(g), _as_rows(y), _fd.ACT_RELU if relu else _fd.ACT_NONE, need_bias)
    return dx.view(g.size(0), g.size(2), g.size(3), g.size(1)).permute(0, 3, 1, 2), db


def conv_grads(x, w, dpre, padding, stride, scale=None, need_x=True):
    """(dX, dW) of ``conv2d(x, w) * scale`` from the gradient ``dpre`` of its output."""
    kind = _kind(x, w, padding, stride)
    k, c = w.size(0), w.size(1)
    if kind is None:
        dconv = dpre * scale.reshape(1, -1, 1, 1).to(dpre.dtype) if scale is not None else dpre
        gx = torch.nn.grad.conv2d_input(x.shape, w, dconv, stride=stride, padding=padding) if need_x else None
        gw = torch.nn.grad.conv2d_weight(x, w.shape, dconv, stride=stride, padding=padding)
        return gx, gw
    dpre = dpre.contiguous(memory_format=torch.channels_last)
    # the frozen scale s multiplies conv's output: dX uses W * s (rows), dW = s * wgrad(x, dpre)
    wx = w if scale is None else (w.float() * scale.float().reshape(-1, 1, 1, 1)).to(w.dtype).contiguous(
        memory_format=torch.channels_last)
    gx = None
    n, _, h, wd = x.shape
    if need_x:
        if kind == "3x3":
            gx = _conv.conv3x3_dgrad(dpre, wx)
        else:
            g2d = _as_rows(dpre)
            w2d = wx.reshape(k, c)
            if kind == "1x1":
                gx2d = _cbn.c1x1(g2d, w2d, b_trans=True)[0] if _cbn.supported(g2d, w2d, b_trans=True) \
                    else torch.mm(g2d, w2d)
            else:
                gx2d = torch.zeros(n * h * wd, c, device=x.device, dtype=x.dtype)
                if _cbn.supported(g2d, w2d, b_trans=True, s2=(h, wd), s2_scatter=True):
                    _cbn.c1x1(g2d, w2d, b_trans=True, s2=(h, wd), s2_scatter=True, resid=gx2d)
                else:
                    gx2d.view(n, h, wd, c)[:, ::2, ::2, :] = torch.mm(g2d, w2d).view(n, h // 2, wd // 2, c)
            gx = gx2d.view(n, h, wd, c).permute(0, 3, 1, 2)
    r = 3 if kind == "3x3" else 1
    st = 2 if kind == "1x1s2" else 1
    if _conv.wgrad_supported(x, dpre, r, st):
        gw = _conv.conv_wgrad_s2(x, dpre) if st == 2 else _conv.conv_wgrad(x, dpre, r)
    else:
        gw = torch.nn.grad.conv2d_weight(x, w.shape, dpre, stride=stride, padding=padding)
    if scale is not None:
        gw = gw * scale.reshape(-1, 1, 1, 1).to(gw.dtype)
    if gw.stride() != w.stride():
        gw = gw.contiguous(memory_format=torch.channels_last) if w.is_contiguous(
            memory_format=torch.channels_last) else gw.contiguous()
    return gx, gw


class ConvBiasReLU_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, padding, stride):
        ones = torch.ones(weight.size(0), device=x.device, dtype=torch.float32)
        y = conv_affine(x, weight, ones, bias, True, padding, stride)
        ctx.save_for_backward(x, weight, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, y = ctx.saved_tensors
        dpre, db = _dpre(grad_output, y, True, True)
        gx, gw = conv_grads(x, w, dpre, ctx.padding, ctx.stride, need_x=ctx.needs_input_grad[0])
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None


class ConvBiasMaskReLU_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, mask, padding, stride):
        ones = torch.ones(weight.size(0), device=x.device, dtype=torch.float32)
        y = conv_affine(x, weight, ones, bias, True, padding, stride, r=mask, r_mul=True)
        ctx.save_for_backward(x, weight, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, y = ctx.saved_tensors
        dpre, db = _dpre(grad_output, y, True, True)  # y == 0 where masked or ReLU-clipped
        gx, gw = conv_grads(x, w, dpre, ctx.padding, ctx.stride, need_x=ctx.needs_input_grad[0])
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None, None


class ConvBias_(torch.autograd.Function):
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, bias, padding, stride):
        ones = torch.ones(weight.size(0), device=x.device, dtype=torch.float32)
        ctx.save_for_backward(x, weight)
        ctx.padding, ctx.stride = padding, stride
        return conv_affine(x, weight, ones, bias, False, padding, stride)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w = ctx.saved_tensors
        dpre, db = _dpre(grad_output, grad_output, False, True)
        gx, gw = conv_grads(x, w, dpre, ctx.padding, ctx.stride, need_x=ctx.needs_input_grad[0])
        return gx, gw, db.view(1, -1, 1, 1).to(w.dtype), None, None


class ConvFrozenScaleBiasReLU_(torch.autograd.Function):
    """relu(conv(x, w) * scale + bias) with frozen (non-trainable) per-channel scale / bias."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, scale, bias, padding, stride):
        y = conv_affine(x, weight, scale, bias, True, padding, stride)
        ctx.save_for_backward(x, weight, scale, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, scale, y = ctx.saved_tensors
        dpre, _ = _dpre(grad_output, y, True, False)
        gx, gw = conv_grads(x, w, dpre, ctx.padding, ctx.stride, scale=scale, need_x=ctx.needs_input_grad[0])
        return gx, gw, None, None, None, None


class ConvFrozenScaleBiasAddReLU_(torch.autograd.Function):
    """relu(conv(x, w) * scale + bias + z), frozen scale / bias: the last conv of a frozen-BN bottleneck
    with its residual add in the same kernel; the gradient of z is the ReLU-masked output gradient."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, scale, bias, z, padding, stride):
        y = conv_affine(x, weight, scale, bias, True, padding, stride, r=z)
        ctx.save_for_backward(x, weight, scale, y)
        ctx.padding, ctx.stride = padding, stride
        return y

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, scale, y = ctx.saved_tensors
        dpre, _ = _dpre(grad_output, y, True, False)
        gx, gw = conv_grads(x, w, dpre, ctx.padding, ctx.stride, scale=scale, need_x=ctx.needs_input_grad[0])
        return gx, gw, None, None, dpre, None, None


class ConvFrozenScaleBias_(torch.autograd.Function):
    """conv(x, w) * scale + bias with frozen scale / bias (a frozen-BN downsample branch)."""

    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda", cast_inputs=torch.half)
    def forward(ctx, x, weight, scale, bias, padding, stride):
        ctx.save_for_backward(x, weight, scale)
        ctx.padding, ctx.stride = padding, stride
        return conv_affine(x, weight, scale, bias, False, padding, stride)

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, grad_output):
        x, w, scale = ctx.saved_tensors
        gx, gw = conv_grads(x, w, grad_output, ctx.padding, ctx.stride, scale=scale,
                            need_x=ctx.needs_input_grad[0])
        return gx, gw, None, None, None, None


ConvBiasReLU = ConvBiasReLU_.apply
ConvBiasMaskReLU = ConvBiasMaskReLU_.apply
ConvBias = ConvBias_.apply
ConvFrozenScaleBiasReLU = ConvFrozenScaleBiasReLU_.apply
ConvFrozenScaleBiasAddReLU = ConvFrozenScaleBiasAddReLU_.apply
ConvFrozenScaleBias = ConvFrozenScaleBias_.apply
