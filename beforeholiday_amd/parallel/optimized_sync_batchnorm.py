"""SyncBatchNorm (reference: apex/parallel/optimized_sync_batchnorm.py:9-85 and
optimized_sync_batchnorm_kernel.py:7-119).

Training forward: local Welford statistics (HIP kernel) -> ONE fixed-size [2C+1] SUM all-reduce of
sums centred on the running mean (``BH_SYNCBN_STATS=allgather`` selects the reference's all_gather of
[mean, var_biased, count] rows + Welford merge instead) -> finalize + running-stat update +
per-channel scale/shift (one tiny kernel) -> a single fused  y = x*scale + shift (+ z) (ReLU)  pass. Backward: one reduce
kernel (ReLU mask recomputed from x, no masked-dy tensor), all_reduce of [sum_dy, sum_dy_xmu],
one dgrad kernel that also emits dz for the fused residual branch (BN + add + ReLU saves a 1-bit
ReLU mask in the forward, so neither backward pass reads z). With a single rank the
collectives are skipped and the merge is fused into the statistics finalize.
"""
from __future__ import annotations


import torch
import torch.distributed as dist
from torch.nn import functional as F
from torch.nn.modules.batchnorm import _BatchNorm

from ..ops import conv_bn as conv_bn_ops
from ..ops import syncbn
from . import comm_stats

def stats_mode() -> str:
    """How ranks combine forward statistics (``Config.syncbn_stats``): ``"allreduce"`` (default; one
    [2C+1] SUM all-reduce of shifted sums) or ``"allgather"`` (the reference's [W, 2C+1] all_gather +
    Welford merge)."""
    from .. import config

    return config.get().syncbn_stats


def set_stats_mode(mode: str) -> None:
    from .. import config

    if mode not in ("allreduce", "allgather"):
        raise ValueError(f"SyncBatchNorm stats mode must be 'allreduce' or 'allgather', got {mode!r}")
    config.set(syncbn_stats=mode)


def _world(pg):
    if hasattr(pg, "all_reduce_"):  # a reducer object, e.g. contrib.peer_memory.PeerAllReduce (IPC)
        return pg.size
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(pg)


def _all_reduce(t, pg):
    if hasattr(pg, "all_reduce_"):
        pg.all_reduce_(t)
    else:
        dist.all_reduce(t, group=pg)


class _WorkHandle:
    def __init__(self, work, t):
        self.work, self.t = work, t

    def wait(self):
        self.work.wait()
        return self.t


def _all_reduce_async(t, pg):
    """Start the SUM all-reduce of ``t`` without blocking the current stream: the IPC reducer's side
    stream, or an async RCCL / gloo collective. ``.wait()`` on the result before using ``t``."""
    if hasattr(pg, "all_reduce_async"):
        return pg.all_reduce_async(t)
    if hasattr(pg, "all_reduce_"):
        pg.all_reduce_(t)
        return _WorkHandle(_NoWork(), t)
    return _WorkHandle(dist.all_reduce(t, group=pg, async_op=True), t)


class _NoWork:
    def wait(self):
        return True


class SyncBatchnormFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, z, weight, bias, running_mean, running_var, eps, momentum, process_group,
                channel_last, fuse_relu, num_batches=None, pool=None):
        input = input.contiguous(memory_format=torch.channels_last) if (channel_last and input.dim() == 4) else input
        world = _world(process_group)
        if world > 1 and (stats_mode() == "allreduce" or hasattr(process_group, "all_reduce_")):
            # one fixed-size [2C+1] SUM all-reduce of shifted sums (K = running mean, shared by all ranks)
            sums = syncbn.stats_local_sums(input, running_mean)
            with comm_stats.timed("syncbn_fwd", sums):
                _all_reduce(sums, process_group)
            mean, invstd, scale, shift, count = syncbn.merge_sums(sums, weight, bias, running_mean, running_var,
                                                                  momentum, eps, num_batches)
        elif world > 1:
            # reference form (optimized_sync_batchnorm_kernel.py:34-43): all_gather [W, 2C+1] + Welford merge
            local = syncbn.stats_local(input)
            gathered = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
            with comm_stats.timed("syncbn_fwd", local):
                dist.all_gather_into_tensor(gathered, local, group=process_group)
            gathered = gathered.view(world, local.numel())
            mean, invstd, scale, shift, count = syncbn.merge_ranks(gathered, weight, bias, running_mean,
                                                                   running_var, momentum, eps, num_batches)
        else:
            mean, invstd, scale, shift, count = syncbn.stats_single(input, weight, bias, running_mean,
                                                                    running_var, momentum, eps, num_batches)
        # the normalisation kernel also bumps num_batches_tracked (no separate add kernel)
        mask = None
        if pool is not None:
            # BN + ReLU + max pool in one pass: the normalised activation is never written
            out, idx = syncbn.maxpool_forward(input, scale, shift, fuse_relu, *pool, True, num_batches)
        elif fuse_relu and syncbn.mask_ok(input, z):
            # BN + add + ReLU: keep a 1-bit ReLU mask instead of re-reading z in both backward passes
            (out, mask), idx = syncbn.forward_mask(input, z, scale, shift, num_batches), None
        else:
            out, idx = syncbn.forward(input, z, scale, shift, fuse_relu, None, num_batches), None
        ctx.save_for_backward(input, None if mask is not None else z, weight, mean, invstd, scale, shift, count, idx,
                              mask)
        ctx.pool = pool
        ctx.process_group = process_group
        ctx.world = world
        ctx.fuse_relu = fuse_relu
        ctx.has_z = z is not None
        return out

    @staticmethod
    def backward(ctx, grad_output):
        input, z, weight, mean, invstd, scale, shift, count, idx, mask = ctx.saved_tensors
        if ctx.pool is not None:
            grad_output = syncbn.maxpool_backward(grad_output, idx, input.size(2), input.size(3), *ctx.pool)
        need_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        sums, gw, gb = syncbn.backward_reduce(grad_output, input, z, mean, invstd, scale, shift, ctx.fuse_relu,
                                              weight, need_w, mask)
        grad_input = grad_z = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            if ctx.world > 1:
                with comm_stats.timed("syncbn_bwd", sums):
                    _all_reduce(sums, ctx.process_group)
            grad_input, grad_z = syncbn.backward_dgrad(grad_output, input, z, mean, invstd, weight, sums, count,
                                                       scale, shift, ctx.fuse_relu,
                                                       ctx.has_z and ctx.needs_input_grad[1], mask)
        return grad_input, grad_z, (gw if need_w else None), (gb if need_w else None), None, None, None, None, None, \
            None, None, None, None


class BNLink(object):
    """One BatchNorm -> convolution boundary of the conv-folded ResNet path (models/resnet.py).

    The BatchNorm's forward records its raw input ``y`` and per-channel ``scale / shift / mean``; the
    consuming convolution's backward reads them to reduce the BatchNorm's backward sums inside its
    data-gradient epilogue and leaves them in ``sums`` (``[sum_dz, sum_dz*(y-mean)]``, local to this
    rank); the BatchNorm's backward then skips its own reduction pass over ``dA`` and ``y``. The forward also
    records ``invstd`` and the BatchNorm ``weight``, so the launch that sums the epilogue partials can emit
    the fp32 parameter gradients too (``grads`` = (gw, gb), ops.conv_bn.sum_parts_grads)."""

    __slots__ = ("y", "scale", "shift", "mean", "relu", "sums", "invstd", "weight", "grads")

    def __init__(self):
        self.y = self.scale = self.shift = self.mean = self.sums = self.invstd = self.weight = self.grads = None
        self.relu = True

    def take_part(self, part):
        """Sum a consumer's epilogue partials into ``sums`` (+ ``grads`` for fp32 parameters that need them)."""
        from ..ops import conv_bn as _cb

        need = self.weight is not None and self.weight.requires_grad and self.invstd is not None
        self.sums, gw, gb = _cb.sum_parts_grads(part, self.invstd, self.weight, need)
        self.grads = (gw, gb) if gw is not None else None


class SyncBatchnormFromStats(torch.autograd.Function):
    """Training-mode SyncBatchNorm whose local statistics arrive as the producing convolution's
    epilogue partials (``part [2, G, C]``: sums of ``x - running_mean`` and its square, see
    ops/conv_bn.py) instead of a statistics pass over ``input``: partials -> ``[2C+1]`` sums -> (one
    all-reduce across ranks) -> merge / running-stat update -> the fused normalise (+z)(ReLU) pass.
    With ``link``, the backward reduction may already have been done by the consuming convolution."""

    @staticmethod
    def forward(ctx, input, part, z, weight, bias, running_mean, running_var, eps, momentum, process_group,
                fuse_relu, num_batches, link, pool=None):
        world = _world(process_group)
        C = input.size(1)
        count = float(input.numel() // C)
        if world > 1:
            sums = conv_bn_ops.sum_parts(part, count)
            with comm_stats.timed("syncbn_fwd", sums):
                _all_reduce(sums, process_group)
            mean, invstd, scale, shift, count_t = syncbn.merge_sums(sums, weight, bias, running_mean, running_var,
                                                                    momentum, eps, num_batches)
        else:  # one rank: partials -> statistics in one launch
            mean, invstd, scale, shift, count_t = syncbn.merge_parts(part, count, weight, bias, running_mean,
                                                                     running_var, momentum, eps, num_batches)
        mask = idx = None
        if pool is not None:  # BN (+ ReLU) + max pool in one pass (the ResNet stem): the normalised
            out, idx = syncbn.maxpool_forward(input, scale, shift, fuse_relu, *pool, True, num_batches)
        elif fuse_relu and syncbn.mask_ok(input, z):
            out, mask = syncbn.forward_mask(input, z, scale, shift, num_batches)
        else:
            out = syncbn.forward(input, z, scale, shift, fuse_relu, None, num_batches)
        if link is not None:
            link.y, link.scale, link.shift, link.mean, link.relu = input, scale, shift, mean, fuse_relu
            link.invstd, link.weight = invstd, weight
            link.sums = link.grads = None
        ctx.save_for_backward(input, None if mask is not None else z, weight, mean, invstd, scale, shift, count_t, mask,
                              idx)
        ctx.pool = pool
        ctx.process_group = process_group
        ctx.world = world
        ctx.fuse_relu = fuse_relu
        ctx.has_z = z is not None
        ctx.link = link
        ctx.mark_non_differentiable(part)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        input, z, weight, mean, invstd, scale, shift, count, mask, idx = ctx.saved_tensors
        if ctx.pool is not None:
            grad_output = syncbn.maxpool_backward(grad_output, idx, input.size(2), input.size(3), *ctx.pool)
        link = ctx.link
        need_w = weight is not None and (ctx.needs_input_grad[3] or ctx.needs_input_grad[4])
        if link is not None and link.sums is not None:
            sums = link.sums  # reduced by the consuming convolution's data-gradient epilogue
            grads, link.sums, link.grads = link.grads, None, None
            C = input.size(1)
            if need_w and grads is not None:
                gw, gb = grads  # from the summing launch (fp32 parameters)
            else:
                gw = (sums[C:] * invstd).to(weight.dtype) if need_w else None
                # a copy: `sums` is all-reduced in place below, the bias gradient stays this rank's own
                gb = sums[:C].to(weight.dtype, copy=True) if need_w else None
        else:
            sums, gw, gb = syncbn.backward_reduce(grad_output, input, z, mean, invstd, scale, shift, ctx.fuse_relu,
                                                  weight, need_w, mask)
        if link is not None:
            link.y = link.invstd = link.weight = None  # release the saved references
        if ctx.world > 1:
            with comm_stats.timed("syncbn_bwd", sums):
                _all_reduce(sums, ctx.process_group)
        grad_input, grad_z = syncbn.backward_dgrad(grad_output, input, z, mean, invstd, weight, sums, count, scale,
                                                   shift, ctx.fuse_relu, ctx.has_z and ctx.needs_input_grad[2], mask)
        return grad_input, None, grad_z, (gw if need_w else None), (gb if need_w else None), None, None, None, None, \
            None, None, None, None, None


class SyncBatchNorm(_BatchNorm):
    """Synchronized batch norm over ``process_group`` (default: WORLD).

    ``channel_last=True`` expects/keeps NHWC (channels_last) activations; ``fuse_relu=True`` applies
    ReLU after the optional residual input ``z`` (``forward(input, z=None)``).
    ``fuse_maxpool=(kernel, stride, padding)`` additionally max-pools the (ReLU'd) output in the same
    pass (the ResNet stem); the module then returns the pooled tensor.
    """

    warned = False

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, channel_last=False, fuse_relu=False, fuse_maxpool=None):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats)
        self.process_group = process_group
        self.channel_last = channel_last
        self.fuse_relu = fuse_relu
        self.fuse_maxpool = tuple(fuse_maxpool) if fuse_maxpool is not None else None

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def _specify_channel_last(self, channel_last):
        self.channel_last = channel_last

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError("expected at least 2D input (got {}D input)".format(input.dim()))

    def _pool_ok(self, input, z):
        return (self.fuse_maxpool is not None and z is None and input.dim() == 4 and input.size(1) % 8 == 0
                and self.channel_last and input.is_contiguous(memory_format=torch.channels_last))

    def forward(self, input, z=None):
        self._check_input_dim(input)
        if self.fuse_maxpool is not None and not self._pool_ok(input, z):
            return F.max_pool2d(self._bn(input, z, None), *self.fuse_maxpool)
        return self._bn(input, z, self.fuse_maxpool)

    def forward_from_stats(self, input, part, z=None, link=None):
        """Training forward from the producing convolution's statistics partials (see
        :class:`SyncBatchnormFromStats`); ``part`` must be centred on ``self.running_mean``. With
        ``fuse_maxpool`` the pooled tensor is returned (BN + ReLU + max pool in one pass)."""
        exp_avg = self.momentum if self.momentum is not None else -1.0
        pool = self.fuse_maxpool if (self.fuse_maxpool is not None and self._pool_ok(input, z)) else None
        return SyncBatchnormFromStats.apply(input, part, z, self.weight, self.bias, self.running_mean, self.running_var,
                                            self.eps, exp_avg, self.process_group, self.fuse_relu,
                                            self.num_batches_tracked, link, pool)

    def _bn(self, input, z, pool):
        if not self.training and self.track_running_stats:
            # inference: fold running stats into scale/shift, one fused pass (z / relu / pool included)
            w = self.weight.float() if self.weight is not None else torch.ones_like(self.running_mean, dtype=torch.float32)
            b = self.bias.float() if self.bias is not None else torch.zeros_like(self.running_mean, dtype=torch.float32)
            invstd = torch.rsqrt(self.running_var.float() + self.eps)
            scale = (w * invstd).contiguous()
            shift = (b - self.running_mean.float() * scale).contiguous()
            if pool is not None:
                return syncbn.maxpool_forward(input, scale, shift, self.fuse_relu, *pool, False)[0]
            return syncbn.forward(input, z, scale, shift, self.fuse_relu)
        tracking = self.training and self.track_running_stats
        # momentum=None -> cumulative average, computed on the device from num_batches_tracked
        exp_avg = (self.momentum if self.momentum is not None else -1.0) if tracking else 0.0
        rm = self.running_mean if tracking else None
        rv = self.running_var if tracking else None
        nbt = self.num_batches_tracked if tracking else None
        return SyncBatchnormFunction.apply(input, z, self.weight, self.bias, rm, rv, self.eps, exp_avg,
                                           self.process_group, self.channel_last, self.fuse_relu, nbt, pool)
