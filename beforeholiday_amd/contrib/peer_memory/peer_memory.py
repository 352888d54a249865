"""Peer-memory pool and 1-D halo exchanger (reference: apex/contrib/peer_memory/{peer_memory,
peer_halo_exchanger_1d}.py, csrc/peer_memory: hipIpc-shared buffers + push/pull kernels with
flag signalling).

MI355X: the host driver here only supports dmabuf IPC, and RCCL already drives the xGMI peer links
directly, so the pool hands out ordinary device tensors (one per peer slot) and the exchanger moves
halos with grouped RCCL send/recv between neighbours — the same data movement without IPC
handles, spin-wait flags or a resident copy kernel.
"""
import torch
import torch.distributed as dist

from ..nccl_p2p.nccl_p2p import _exchange


class PeerMemoryPool(object):
    def __init__(self, static_size, dynamic_size, peer_ranks=None):
        self.peer_ranks = peer_ranks if peer_ranks is not None else list(range(dist.get_world_size()))
        self.peer_rank = self.peer_ranks.index(dist.get_rank()) if dist.get_rank() in self.peer_ranks else 0
        self.static_size = static_size
        self.dynamic_size = dynamic_size
        self._static = []
        self._dynamic = []

    def __del__(self):
        self._static = self._dynamic = []

    def reset(self):
        self._dynamic = []

    def allocate_peer_tensors(self, shape, dtype, channels_last, dynamic):
        fmt = torch.channels_last if channels_last and len(shape) == 4 else torch.contiguous_format
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        ts = [torch.zeros(shape, dtype=dtype, device=dev).contiguous(memory_format=fmt) for _ in self.peer_ranks]
        (self._dynamic if dynamic else self._static).append(ts)
        return ts


class PeerHaloExchanger1d:
    """In-place halo exchange along H (or W) of a padded activation ``y`` ([N, C, H+2h, W] channels_last
    or explicit NHWC [N, H+2h, W, C]); first/last ranks get zero halos."""

    def __init__(self, ranks, rank_in_group, peer_pool, half_halo):
        self.peer_group_size = len(ranks)
        self.ranks = ranks
        self.rank_in_group = rank_in_group
        self.peer_pool = peer_pool
        self.half_halo = half_halo
        self.left_rank = ranks[rank_in_group - 1] if rank_in_group > 0 else -1
        self.right_rank = ranks[rank_in_group + 1] if rank_in_group < len(ranks) - 1 else -1

    def __call__(self, y, H_split=True, explicit_nhwc=False, numSM=0, diagnostics=False):
        h = self.half_halo
        dim = (1 if H_split else 2) if explicit_nhwc else (2 if H_split else 3)
        n = y.size(dim)
        left_out = y.narrow(dim, h, h)
        right_out = y.narrow(dim, n - 2 * h, h)
        left_in = y.narrow(dim, 0, h)
        right_in = y.narrow(dim, n - h, h)
        li = torch.empty_like(left_in, memory_format=torch.contiguous_format)
        ri = torch.empty_like(right_in, memory_format=torch.contiguous_format)
        _exchange(dist.group.WORLD, self.left_rank, self.right_rank, left_out, right_out, li, ri)
        left_in.copy_(li)
        right_in.copy_(ri)
