"""Halo exchangers for spatially-parallel convolutions (reference: apex/contrib/bottleneck/halo_exchangers.py:11-170).

``left_right_halo_exchange(left_output_halo, right_output_halo[, left_input_halo, right_input_halo])``:
send my boundary rows to the left / right neighbour in ``ranks`` and receive theirs; edge ranks
receive zeros. Variants: no communication (single rank, wraps), one all-gather over a sub-group,
point-to-point (grouped RCCL send/recv on a private communicator, as the reference's nccl_p2p), and
'Peer' (direct loads / stores into IPC-mapped neighbour memory through peer_memory_cuda).
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
    """Grouped send/recv on a private communicator (reference: get_unique_nccl_id + broadcast +
    init_nccl_comm, halo_exchangers.py:69-88); ``group`` overrides it."""

    def __init__(self, ranks, rank_in_group, group=None):
        super().__init__(ranks, rank_in_group)
        if group is None:
            from ..nccl_p2p import get_unique_nccl_id, init_nccl_comm

            uid = get_unique_nccl_id(1)
            if dist.get_backend() == "nccl":
                uid = uid.cuda()
            dist.broadcast(uid, 0)
            group = init_nccl_comm(uid.cpu(), dist.get_rank(), dist.get_world_size())
        self.group = group

    def left_right_halo_exchange(self, left_output_halo, right_output_halo, left_input_halo=None,
                                 right_input_halo=None):
        li = torch.empty_like(right_output_halo, memory_format=torch.contiguous_format)
        ri = torch.empty_like(left_output_halo, memory_format=torch.contiguous_format)
        _exchange(self.group, self.left_rank, self.right_rank, left_output_halo, right_output_halo, li, ri)
        if left_input_halo is None:
            return li, ri
        left_input_halo.copy_(li)
        right_input_halo.copy_(ri)


class HaloExchangerPeer(HaloExchanger):
    """Halos moved through IPC-mapped neighbour memory (peer_memory_cuda.push_pull_halos_1d) when the
    pool is native; otherwise grouped send/recv over the default group."""

    def __init__(self, ranks, rank_in_group, peer_pool, explicit_nhwc, numSM=1):
        super().__init__(ranks, rank_in_group)
        self.peer_pool = peer_pool
        self.explicit_nhwc = explicit_nhwc
        self.numSM = numSM
        self._peer = None
        if getattr(peer_pool, "native", False):
            from ..peer_memory import PeerHaloExchanger1d

            self._peer = PeerHaloExchanger1d(ranks, rank_in_group, peer_pool, 0)

    def left_right_halo_exchange(self, left_output_halo, right_output_halo, left_input_halo=None,
                                 right_input_halo=None):
        ret = left_input_halo is None
        if ret:
            left_input_halo = torch.empty_like(right_output_halo)
            right_input_halo = torch.empty_like(left_output_halo)
        if self._peer is not None and left_output_halo.is_cuda:
            self._peer.exchange_views(left_output_halo, right_output_halo, left_input_halo, right_input_halo)
        else:
            li = torch.empty_like(right_output_halo, memory_format=torch.contiguous_format)
            ri = torch.empty_like(left_output_halo, memory_format=torch.contiguous_format)
            _exchange(dist.group.WORLD, self.left_rank, self.right_rank, left_output_halo, right_output_halo, li, ri)
            left_input_halo.copy_(li)
            right_input_halo.copy_(ri)
        if ret:
            return left_input_halo, right_input_halo


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
