"""NHWC batch norm with optional fused add + ReLU, synchronised over groups of ``bn_group`` GPUs
(reference: apex/contrib/groupbn/batch_norm.py:135-260, ``bnp`` extension with IPC peer buffers).

MI355X: like the reference, the ``bn_group`` consecutive ranks of a node exchange statistics through
IPC-mapped peer memory: one :class:`~beforeholiday_amd.contrib.peer_memory.PeerAllReduce` per group
size (a HIP-IPC pool shared by the group, a single-workgroup push + epoch-flag + rank-ordered sum
kernel), used for the forward [2C+1] shifted sums and the backward [2C] sums -- no RCCL launch per
layer. ``BH_GROUPBN_IPC=0`` (or CPU tensors / no native extension) uses an RCCL / gloo process group of
the same ranks instead. Inputs are physical NHWC [N, H, W, C] tensors (or channels_last NCHW with
``torch_channels_last=True``); kernels are the channel-owned BN kernels of kernels/batchnorm.hip.
"""

import torch
import torch.distributed as dist
from torch.nn.modules.batchnorm import _BatchNorm

from ... import _native
from ... import config as _config
from ...parallel.optimized_sync_batchnorm import SyncBatchnormFunction
from ...ops import syncbn as _bn

_GROUPS = {}
_IPC = {}
_IPC_CAPACITY = 1 << 14  # floats per slot row: 2C+1 for C <= 8191 channels


def _ipc_reducer(size):
    """The IPC reducer of this rank's group of ``size`` consecutive ranks, or None."""
    if (size <= 1 or not dist.is_initialized() or not torch.cuda.is_available() or not _native.available()
            or not _config.get().groupbn_ipc):
        return None
    if size not in _IPC:
        from ..peer_memory import PeerAllReduce, PeerMemoryPool

        start = dist.get_rank() // size * size
        pool = PeerMemoryPool(2 * size * _IPC_CAPACITY * 4 + 4096, 0, peer_ranks=list(range(start, start + size)))
        _IPC[size] = PeerAllReduce(pool, capacity=_IPC_CAPACITY, group=_bn_group(size))
    return _IPC[size]


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
        group = self.process_group
        if xn.is_cuda and self.bn_group > 1:
            group = _ipc_reducer(self.bn_group) or group
        y = SyncBatchnormFunction.apply(xn, zn, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                        self.momentum, group, True, self.fuse_relu, self.num_batches_tracked)
        return self._from_nchw(y)
