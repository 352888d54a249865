"""``syncbn``: batch-norm statistics / normalisation ops.

GPU tensors run ``beforeholiday_amd._C.syncbn`` (kernels/batchnorm.hip); CPU tensors run the
PyTorch reference below with identical semantics. The second half of this module provides the
reference extension's function names (csrc/syncbn.cpp:98-109: ``welford_mean_var``,
``welford_parallel``, ``batchnorm_forward``, ``reduce_bn``, ``batchnorm_backward`` and the
``_c_last`` variants, ``relu_bw_c_last``) on top of the fused ops.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._native import submodule


def _native():
    return submodule("syncbn")


def _bcast(v: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    return v.view([1, -1] + [1] * (x.dim() - 2))


def _reduce_dims(x):
    return [0] + list(range(2, x.dim()))


# --------------------------------------------------------------------------------- reference


def _ref_stats(x):
    xf = x.float()
    dims = _reduce_dims(x)
    mean = xf.mean(dims)
    var_b = xf.var(dims, unbiased=False)
    n = float(x.numel() // x.size(1))
    return mean, var_b, n


def _ref_final(mean, var_b, n, w, b, rm, rv, momentum, eps, num_batches=None):
    if momentum < 0:  # momentum=None: cumulative average over num_batches_tracked + 1 batches
        momentum = 1.0 / (float(num_batches.item()) + 1.0) if num_batches is not None else 1.0
    invstd = torch.rsqrt(var_b + eps)
    wv = w.float() if w is not None else torch.ones_like(mean)
    bv = b.float() if b is not None else torch.zeros_like(mean)
    scale = wv * invstd
    shift = bv - mean * scale
    if rm is not None:
        unb = var_b * n / (n - 1) if n > 1 else var_b
        rm.copy_(((1 - momentum) * rm.float() + momentum * mean).to(rm.dtype))
        rv.copy_(((1 - momentum) * rv.float() + momentum * unb).to(rv.dtype))
    count = torch.full((1,), n, dtype=torch.float32, device=mean.device)
    return [mean, invstd, scale, shift, count]


def stats_local(x):
    if x.is_cuda:
        return _native().stats_local(x)
    mean, var_b, n = _ref_stats(x)
    return torch.cat([mean, var_b, torch.tensor([n], dtype=torch.float32, device=x.device)])


def stats_single(x, weight, bias, running_mean, running_var, momentum, eps, num_batches=None):
    """Single-rank statistics -> [mean, invstd, scale, shift, count]; updates running stats with
    ``momentum`` (< 0: cumulative average using ``num_batches`` = num_batches_tracked)."""
    if x.is_cuda:
        return _native().stats_single(x, weight, bias, running_mean, running_var, momentum, eps, num_batches)
    mean, var_b, n = _ref_stats(x)
    return _ref_final(mean, var_b, n, weight, bias, running_mean, running_var, momentum, eps, num_batches)


def merge_ranks(gathered, weight, bias, running_mean, running_var, momentum, eps, num_batches=None):
    if gathered.is_cuda:
        return _native().merge_ranks(gathered, weight, bias, running_mean, running_var, momentum, eps, num_batches)
    C = (gathered.size(1) - 1) // 2
    means, vars_b, ns = gathered[:, :C], gathered[:, C:2 * C], gathered[:, 2 * C:]
    n = ns.sum()
    mean = (means * ns).sum(0) / n
    m2 = (vars_b * ns).sum(0) + (ns * (means - mean) ** 2).sum(0)
    var_b = m2 / n
    return _ref_final(mean, var_b, float(n), weight, bias, running_mean, running_var, momentum, eps, num_batches)


def stats_local_sums(x, running_mean=None):
    """Local ``[sum(x-K) (C), sum((x-K)^2) (C), count (1)]`` about ``K = running_mean`` (0 if None).

    This is the ``all_reduce(SUM)`` payload of the multi-rank forward: one fixed-size collective
    instead of an all_gather of W rows plus a merge. ``K`` must be the same on every rank (the
    running mean is: it starts at 0 and is updated from the reduced statistics only), and keeps the
    sums centred so ``E[(x-K)^2] - E[x-K]^2`` does not cancel."""
    if x.is_cuda:
        return _native().stats_local_sums(x, running_mean)
    mean, var_b, n = _ref_stats(x)
    k = running_mean.float() if running_mean is not None else torch.zeros_like(mean)
    d = mean - k
    return torch.cat([n * d, n * var_b + n * d * d, torch.tensor([n], dtype=torch.float32, device=x.device)])


def merge_sums(sums, weight, bias, running_mean, running_var, momentum, eps, num_batches=None):
    """Final stats from all-reduced :func:`stats_local_sums` -> [mean, invstd, scale, shift, count]."""
    if sums.is_cuda:
        return _native().merge_sums(sums, weight, bias, running_mean, running_var, momentum, eps, num_batches)
    C = (sums.numel() - 1) // 2
    s1, s2, n = sums[:C], sums[C:2 * C], float(sums[2 * C])
    k = running_mean.float() if running_mean is not None else torch.zeros_like(s1)
    dm = s1 / n
    mean = k + dm
    var_b = torch.clamp(s2 - s1 * dm, min=0) / n
    return _ref_final(mean, var_b, n, weight, bias, running_mean, running_var, momentum, eps, num_batches)


def merge_parts(part, count, weight, bias, running_mean, running_var, momentum, eps, num_batches=None, bump=False):
    """Single rank: :func:`merge_sums` straight from a convolution epilogue's partials ``part [2, G, C]``
    (sums of ``x - running_mean`` and its square per workgroup) over ``count`` elements per channel --
    one kernel on the GPU (two from 1024 partial rows) instead of ``conv_bn.sum_parts`` + ``merge_sums``. ``bump`` (fixed momentum
    only) also advances ``num_batches`` by one in the same launch."""
    if part.is_cuda:
        return _native().merge_parts(part, float(count), weight, bias, running_mean, running_var, momentum, eps,
                                     num_batches, bump)
    C = part.size(2)
    sums = torch.cat([part.sum(1).reshape(-1), torch.tensor([float(count)], dtype=part.dtype)])
    assert sums.numel() == 2 * C + 1
    out = merge_sums(sums, weight, bias, running_mean, running_var, momentum, eps, num_batches)
    if bump and num_batches is not None:
        num_batches += 1
    return out


def forward(x, z, scale, shift, relu, out_dtype=None, num_batches=None):
    """y = x*scale + shift (+z) (relu); increments ``num_batches`` (num_batches_tracked) if given."""
    if x.is_cuda:
        return _native().forward(x, z, scale, shift, relu, out_dtype, num_batches)
    if num_batches is not None:
        num_batches += 1
    y = x.float() * _bcast(scale, x) + _bcast(shift, x)
    if z is not None:
        y = y + z.float()
    if relu:
        y = torch.relu(y)
    return y.to(out_dtype or x.dtype)


def mask_ok(x, z):
    """Whether :func:`forward_mask` applies: a GPU NHWC (C % 8 == 0) input with a same-dtype residual."""
    return x.is_cuda and z is not None and z.dtype == x.dtype and z.shape == x.shape and _native().mask_ok(x)


def forward_mask(x, z, scale, shift, num_batches=None, zscale=None, zshift=None):
    """Fused ``relu(x*scale + shift + z)`` that also returns the ReLU mask packed 8 channels per byte
    (uint8 ``[rows, C/8]``); backward then reads 1 bit per element instead of the residual ``z``. With
    ``zscale / zshift`` the residual is ``z*zscale + zshift`` (a second BatchNorm normalised in the same pass)."""
    if not x.is_cuda:
        zz = z.float() if zscale is None else z.float() * _bcast(zscale, z) + _bcast(zshift, z)
        if num_batches is not None:
            num_batches += 1
        pre = x.float() * _bcast(scale, x) + _bcast(shift, x) + zz
        out = torch.relu(pre).to(x.dtype).contiguous(memory_format=torch.channels_last)
        pos = (pre > 0).permute(0, 2, 3, 1).reshape(-1, x.size(1) // 8, 8).to(torch.int32)
        bits = (pos << torch.arange(8, dtype=torch.int32)).sum(-1).to(torch.uint8)
        return out, bits
    return _native().forward_mask(x, z, scale, shift, num_batches, zscale, zshift)


def _pool_out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


def maxpool_forward(x, scale, shift, relu, kernel_size, stride, padding, want_idx=True, num_batches=None):
    """Max pool (NHWC) of ``(relu)(x*scale + shift)`` (scale/shift may be None). Returns ``(y, idx)``:
    ``idx`` holds the window offset ``kh*k + kw`` of each maximum as uint8 (None if not wanted);
    increments ``num_batches`` if given."""
    if x.is_cuda:
        y, idx = _native().maxpool_forward(x, scale, shift, relu, kernel_size, stride, padding, want_idx,
                                           num_batches)
        return y, (idx if want_idx else None)
    if num_batches is not None:
        num_batches += 1
    v = x.float()
    if scale is not None:
        v = v * _bcast(scale, x) + _bcast(shift, x)
    if relu:
        v = torch.relu(v)
    y, flat = torch.nn.functional.max_pool2d(v, kernel_size, stride, padding, return_indices=True)
    y = y.to(x.dtype).contiguous(memory_format=torch.channels_last)
    if not want_idx:
        return y, None
    W = x.size(3)
    OH, OW = y.shape[2], y.shape[3]
    oh = torch.arange(OH, device=x.device).view(1, 1, OH, 1)
    ow = torch.arange(OW, device=x.device).view(1, 1, 1, OW)
    kh = flat // W - (oh * stride - padding)
    kw = flat % W - (ow * stride - padding)
    return y, (kh * kernel_size + kw).to(torch.uint8).contiguous(memory_format=torch.channels_last)


def maxpool_backward(grad_output, idx, H, W, kernel_size, stride, padding):
    """Gradient of :func:`maxpool_forward` w.r.t. its pooled input (pre-ReLU masking is the caller's)."""
    if grad_output.is_cuda:
        return _native().maxpool_backward(grad_output, idx, H, W, kernel_size, stride, padding)
    N, C, OH, OW = grad_output.shape
    off = idx.long()
    oh = torch.arange(OH).view(1, 1, OH, 1)
    ow = torch.arange(OW).view(1, 1, 1, OW)
    ih = oh * stride - padding + off // kernel_size
    iw = ow * stride - padding + off % kernel_size
    flat = (ih * W + iw).reshape(N, C, -1)
    gx = torch.zeros(N, C, H * W, dtype=torch.float32)
    gx.scatter_add_(2, flat, grad_output.float().reshape(N, C, -1))
    return gx.view(N, C, H, W).to(grad_output.dtype).contiguous(memory_format=torch.channels_last)


def _ref_masked_dy(dy, x, z, scale, shift, relu):
    g = dy.float()
    if relu:
        pre = x.float() * _bcast(scale, x) + _bcast(shift, x)
        if z is not None:
            pre = pre + z.float()
        g = torch.where(pre > 0, g, torch.zeros_like(g))
    return g


def backward_reduce(dy, x, z, mean, invstd, scale, shift, relu, weight, need_weight_grads, mask=None):
    if x.is_cuda:
        return _native().backward_reduce(dy, x, z, mean, invstd, scale, shift, relu, weight, need_weight_grads, mask)
    g = _ref_masked_dy(dy, x, z, scale, shift, relu)
    dims = _reduce_dims(x)
    sum_dy = g.sum(dims)
    sum_dy_xmu = (g * (x.float() - _bcast(mean, x))).sum(dims)
    gw = gb = None
    if need_weight_grads and weight is not None:
        gw = (sum_dy_xmu * invstd).to(weight.dtype)
        gb = sum_dy.to(weight.dtype)
    return [torch.cat([sum_dy, sum_dy_xmu]), gw, gb]


def backward_dgrad(dy, x, z, mean, invstd, weight, sums, count, scale, shift, relu, need_dz, mask=None):
    if x.is_cuda:
        return _native().backward_dgrad(dy, x, z, mean, invstd, weight, sums, count, scale, shift, relu, need_dz,
                                        mask)
    C = x.size(1)
    g = _ref_masked_dy(dy, x, z, scale, shift, relu)
    n = count.float().reshape(-1)[0]
    mdy, mdyx = sums[:C] / n, sums[C:] / n
    wv = weight.float() if weight is not None else torch.ones_like(mean)
    dx = (g - _bcast(mdy, x) - (x.float() - _bcast(mean, x)) * _bcast(invstd * invstd * mdyx, x)) * _bcast(invstd * wv, x)
    dz = g.to(z.dtype if z is not None else x.dtype) if need_dz else None
    return [dx.to(x.dtype), dz]


# ------------------------------------------------------------------- reference-compatible API


def welford_mean_var(input):
    """Returns (mean, biased var) per channel (NCHW input)."""
    local = stats_local(input)
    C = input.size(1)
    return local[:C], local[C:2 * C]


welford_mean_var_c_last = welford_mean_var


def welford_parallel(mean_feature_nodes, var_biased_feature_nodes, numel, eps):
    """Merge per-rank stats -> (mean, unbiased var, inv_std) (reference welford_kernel_parallel)."""
    W, C = mean_feature_nodes.shape
    g = torch.cat([mean_feature_nodes.float(), var_biased_feature_nodes.float(),
                   numel.float().reshape(W, 1).to(mean_feature_nodes.device)], dim=1)
    mean, invstd, _, _, count = merge_ranks(g, None, None, None, None, 0.0, eps)
    n = count.reshape(-1)[0]
    var_b = 1.0 / (invstd * invstd) - eps
    var = var_b * n / torch.clamp(n - 1, min=1)
    return mean, var, invstd


def _scale_shift(mean, inv_std, weight, shift):
    w = weight.float() if weight is not None else torch.ones_like(mean)
    b = shift.float() if shift is not None else torch.zeros_like(mean)
    sc = w * inv_std
    return sc.contiguous(), (b - mean * sc).contiguous()


def batchnorm_forward(input, mean, inv_std, weight=None, shift=None):
    sc, sh = _scale_shift(mean.float(), inv_std.float(), weight, shift)
    return forward(input, None, sc, sh, False)


def batchnorm_forward_c_last(input, z, mean, inv_std, weight=None, shift=None, fuse_relu=False):
    sc, sh = _scale_shift(mean.float(), inv_std.float(), weight, shift)
    return forward(input, z, sc, sh, fuse_relu)


def reduce_bn(grad_output, input, mean, inv_std, weight=None):
    sums, gw, gb = backward_reduce(grad_output, input, None, mean.float().contiguous(), inv_std.float().contiguous(),
                                   None, None, False, weight, weight is not None)
    C = input.size(1)
    return sums[:C], sums[C:], gw, gb


reduce_bn_c_last = reduce_bn


def batchnorm_backward(grad_output, input, mean, inv_std, weight, sum_dy, sum_dy_xmu, count):
    """``count``: per-rank element counts (int tensor) or a total; the reference divides by sum(count)."""
    total = count.float().sum().reshape(1).to(input.device)
    sums = torch.cat([sum_dy.float(), sum_dy_xmu.float()])
    dx, _ = backward_dgrad(grad_output, input, None, mean.float().contiguous(), inv_std.float().contiguous(),
                           weight, sums, total, None, None, False, False)
    return dx


batchnorm_backward_c_last = batchnorm_backward


def relu_bw_c_last(grad_output, input, z, mean, inv_std, weight=None, shift=None):
    sc, sh = _scale_shift(mean.float(), inv_std.float(), weight, shift)
    pre = forward(input, z, sc, sh, False, torch.float32)
    return torch.where(pre > 0, grad_output, torch.zeros_like(grad_output))
