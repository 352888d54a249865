"""NHWC batch norm with optional fused add + ReLU, synchronised over groups of ``bn_group`` GPUs
(reference: apex/contrib/groupbn/batch_norm.py:135-260, ``bnp`` extension with IPC peer buffers).

MI355X: the statistics exchange uses the same Welford-partials all-gather as SyncBatchNorm, over a
process group of ``bn_group`` consecutive ranks (RCCL over xGMI) — no IPC handle registry or
spin-wait CTAs. Inputs are physical NHWC [N, H, W, C] tensors (or channels_last NCHW with
``torch_channels_last=True``); kernels are the channel-owned BN kernels of kernels/batchnorm.hip.
"""
import torch
import torch.distributed as dist
from torch.nn.modules.batchnorm import _BatchNorm

from ...parallel.optimized_sync_batchnorm import SyncBatchnormFunction
from ...ops import syncbn as _bn

_GROUPS = {}


def _bn_group(size):
    if size <= 1 or not dist.is_initialized():
        return None
    if size not in _GROUPS:
        world, rank = dist.get_world_size(), dist.get_rank()
        assert world >= size and world % size == 0
        mine = None
        for start in range(0, world, size):
            g = dist.new_group(list(range(start, start + size)))
            if start <= rank < start + size:
                mine = g
        _GROUPS[size] = mine
    return _GROUPS[size]


class BatchNorm2d_NHWC(_BatchNorm):
    def __init__(self, num_features, fuse_relu=False, bn_group=1, torch_channels_last=False, max_cta_per_sm=2,
                 cta_launch_margin=12, multi_stream=False):
        super().__init__(num_features)
        self.fuse_relu = fuse_relu
        self.torch_channels_last = torch_channels_last
        self.multi_stream = multi_stream
        self.bn_group = bn_group
        self.process_group = _bn_group(bn_group)

    def _to_nchw(self, x):
        return x if self.torch_channels_last else x.permute(0, 3, 1, 2)

    def _from_nchw(self, y):
        return y if self.torch_channels_last else y.permute(0, 2, 3, 1)

    def forward(self, x, z=None):
        xn = self._to_nchw(x)
        zn = self._to_nchw(z) if z is not None else None
        if not self.training:
            invstd = torch.rsqrt(self.running_var.float() + self.eps)
            scale = (self.weight.float() * invstd).contiguous()
            shift = (self.bias.float() - self.running_mean.float() * scale).contiguous()
            return self._from_nchw(_bn.forward(xn, zn, scale, shift, self.fuse_relu))
        y = SyncBatchnormFunction.apply(xn, zn, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                        self.momentum, self.process_group, True, self.fuse_relu,
                                        self.num_batches_tracked)
        return self._from_nchw(y)
