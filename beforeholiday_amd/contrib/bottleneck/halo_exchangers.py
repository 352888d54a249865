"""Halo exchangers for spatially-parallel convolutions (reference: apex/contrib/bottleneck/halo_exchangers.py:11-170).

``left_right_halo_exchange(left_output_halo, right_output_halo[, left_input_halo, right_input_halo])``:
send my boundary rows to the left / right neighbour in ``ranks`` and receive theirs; edge ranks
receive zeros. Variants: no communication (single rank, wraps), one all-gather over a sub-group,
and point-to-point (grouped RCCL send/recv — also used for the reference's IPC 'Peer' variant).
"""
import torch
import torch.distributed as dist

from ..nccl_p2p.nccl_p2p import _exchange


class HaloExchanger(object):
    def __init__(self, ranks, rank_in_group):
        self.group_size = len(ranks)
        self.ranks = ranks
        self.rank_in_group = rank_in_group
        self.wrap_around_left_rank_in_group = (rank_in_group + self.group_size - 1) % self.group_size
        self.wrap_around_right_rank_in_group = (rank_in_group + 1) % self.group_size
        self.left_rank = ranks[rank_in_group - 1] if rank_in_group > 0 else -1
        self.left_zero = rank_in_group == 0
        self.right_rank = ranks[rank_in_group + 1] if rank_in_group < self.group_size - 1 else -1
        self.right_zero = rank_in_group == self.group_size - 1


class HaloExchangerNoComm(HaloExchanger):
    def left_right_halo_exchange(self, left_output_halo, right_output_halo, left_input_halo=None,
                                 right_input_halo=None):
        if left_input_halo is None:
            return right_output_halo, left_output_halo
        left_input_halo.copy_(right_output_halo)
        right_input_halo.copy_(left_output_halo)


class HaloExchangerAllGather(HaloExchanger):
    def __init__(self, ranks, rank_in_group, comm):
        super().__init__(ranks, rank_in_group)
        self.comm = comm

    def left_right_halo_exchange(self, left_output_halo, right_output_halo, left_input_halo=None,
                                 right_input_halo=None):
        N, Hh, W, C = left_output_halo.shape
        send = torch.cat([left_output_halo.contiguous(), right_output_halo.contiguous()], dim=1)
        gathered = torch.empty((self.group_size,) + tuple(send.shape), dtype=send.dtype, device=send.device)
        dist.all_gather_into_tensor(gathered.view(-1), send.reshape(-1), group=self.comm)
        ag_left = gathered[self.wrap_around_left_rank_in_group][:, Hh:]
        ag_right = gathered[self.wrap_around_right_rank_in_group][:, :Hh]
        if self.left_zero:
            ag_left = torch.zeros_like(ag_left)
        if self.right_zero:
            ag_right = torch.zeros_like(ag_right)
        if left_input_halo is None:
            return ag_left, ag_right
        left_input_halo.copy_(ag_left)
        right_input_halo.copy_(ag_right)


class HaloExchangerSendRecv(HaloExchanger):
    def __init__(self, ranks, rank_in_group, group=None):
        super().__init__(ranks, rank_in_group)
        self.group = group if group is not None else dist.group.WORLD

    def left_right_halo_exchange(self, left_output_halo, right_output_halo, left_input_halo=None,
                                 right_input_halo=None):
        li = torch.empty_like(right_output_halo, memory_format=torch.contiguous_format)
        ri = torch.empty_like(left_output_halo, memory_format=torch.contiguous_format)
        _exchange(self.group, self.left_rank, self.right_rank, left_output_halo, right_output_halo, li, ri)
        if left_input_halo is None:
            return li, ri
        left_input_halo.copy_(li)
        right_input_halo.copy_(ri)


class HaloExchangerPeer(HaloExchangerSendRecv):
    """The reference pushes halos through IPC-mapped peer buffers; here the same exchange runs as
    grouped RCCL send/recv over xGMI (see contrib.peer_memory)."""

    def __init__(self, ranks, rank_in_group, peer_pool, explicit_nhwc, numSM=1):
        super().__init__(ranks, rank_in_group)
        self.peer_pool = peer_pool
        self.explicit_nhwc = explicit_nhwc
        self.numSM = numSM


class HaloPadder:
    """Pad ``y`` along H (or W) with ``half_halo`` rows from each neighbour."""

    def __init__(self, halo_ex):
        self.halo_ex = halo_ex

    def __call__(self, y, half_halo, explicit_nhwc, H_split):
        dim = (1 if H_split else 2) if explicit_nhwc else (2 if H_split else 3)
        n = y.size(dim)
        left_out = y.narrow(dim, 0, half_halo)
        right_out = y.narrow(dim, n - half_halo, half_halo)
        if explicit_nhwc and H_split:
            li, ri = self.halo_ex.left_right_halo_exchange(left_out, right_out)
        else:
            # exchangers work on [N, Hh, W, C]-like blocks: move the split dim to position 1
            perm = list(range(y.dim()))
            perm[1], perm[dim] = perm[dim], perm[1]
            li, ri = self.halo_ex.left_right_halo_exchange(left_out.permute(perm).contiguous(),
                                                           right_out.permute(perm).contiguous())
            li, ri = li.permute(perm), ri.permute(perm)
        out = torch.cat([li.to(y.dtype), y, ri.to(y.dtype)], dim=dim)
        if not explicit_nhwc and y.is_contiguous(memory_format=torch.channels_last):
            out = out.contiguous(memory_format=torch.channels_last)
        return out
