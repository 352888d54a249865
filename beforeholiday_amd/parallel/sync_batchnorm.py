"""Python-only SyncBatchNorm (reference: apex/parallel/sync_batchnorm.py:9-134).

Statistics with two all_reduces of [sum(x), sum(x^2)] in fp32 and plain PyTorch math; kept as the
"no native extension" path and as an independent oracle for the fused implementation.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.nn import functional as F
from torch.nn.modules.batchnorm import _BatchNorm


def _world(pg):
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(pg)


class SyncBatchnormFunctionPy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, weight, bias, running_mean, running_var, eps, process_group, world_size, momentum):
        C = input.size(1)
        dims = [0] + list(range(2, input.dim()))
        xf = input.float()
        n_local = input.numel() // C
        sums = torch.stack([xf.sum(dims), (xf * xf).sum(dims)])
        count = torch.tensor([float(n_local)], device=input.device)
        if world_size > 1:
            dist.all_reduce(sums, group=process_group)
            dist.all_reduce(count, group=process_group)
        n = count.item()
        mean = sums[0] / n
        var = torch.clamp(sums[1] / n - mean * mean, min=0.0)
        if running_mean is not None:
            running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
            running_var.mul_(1 - momentum).add_((var * n / max(n - 1, 1)).to(running_var.dtype), alpha=momentum)
        invstd = torch.rsqrt(var + eps)
        shape = [1, -1] + [1] * (input.dim() - 2)
        out = (xf - mean.view(shape)) * invstd.view(shape)
        if weight is not None:
            out = out * weight.float().view(shape) + bias.float().view(shape)
        ctx.save_for_backward(input, weight, mean, invstd)
        ctx.process_group, ctx.world_size, ctx.n = process_group, world_size, n
        return out.to(input.dtype)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight, mean, invstd = ctx.saved_tensors
        dims = [0] + list(range(2, input.dim()))
        shape = [1, -1] + [1] * (input.dim() - 2)
        g = grad_output.float()
        xmu = input.float() - mean.view(shape)
        sums = torch.stack([g.sum(dims), (g * xmu).sum(dims)])
        grad_weight = (sums[1] * invstd).to(weight.dtype) if weight is not None else None
        grad_bias = sums[0].to(weight.dtype) if weight is not None else None
        if ctx.world_size > 1:
            dist.all_reduce(sums, group=ctx.process_group)
        mdy, mdyx = sums[0] / ctx.n, sums[1] / ctx.n
        w = weight.float() if weight is not None else torch.ones_like(mean)
        gi = (g - mdy.view(shape) - xmu * (invstd * invstd * mdyx).view(shape)) * (invstd * w).view(shape)
        return gi.to(input.dtype), grad_weight, grad_bias, None, None, None, None, None, None


class SyncBatchNorm(_BatchNorm):
    warned = False

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, channel_last=False, fuse_relu=False):
        if channel_last or fuse_relu:
            raise AttributeError("channel_last / fuse_relu are only supported by the fused SyncBatchNorm")
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats)
        self.process_group = process_group

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError("expected at least 2D input (got {}D input)".format(input.dim()))

    def forward(self, input):
        if not self.training and self.track_running_stats:
            return F.batch_norm(input, self.running_mean, self.running_var, self.weight, self.bias, False, 0.0,
                                self.eps)
        momentum = self.momentum if self.momentum is not None else 0.0
        if self.training and self.track_running_stats:
            self.num_batches_tracked += 1
            if self.momentum is None:
                momentum = 1.0 / float(self.num_batches_tracked)
        rm = self.running_mean if self.training and self.track_running_stats else None
        rv = self.running_var if self.training and self.track_running_stats else None
        return SyncBatchnormFunctionPy.apply(input, self.weight, self.bias, rm, rv, self.eps, self.process_group,
                                             _world(self.process_group), momentum)
