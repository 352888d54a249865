"""Neighbour halo exchange on a private communicator (reference: apex/contrib/csrc/nccl_p2p/nccl_p2p_cuda.cu,
``nccl_p2p_cuda``: ``ncclGetUniqueId`` + ``ncclCommInitRank`` of a second communicator + grouped
send/recv).

On ROCm the torch.distributed "nccl" backend IS RCCL: ``init_nccl_comm`` creates a dedicated process
group over the ranks, i.e. its own RCCL communicator (own streams, never queued behind the default
group's gradient all-reduces), keyed by the unique id every rank received from rank 0. One
``batch_isend_irecv`` group then moves both halos (RCCL coalesces the sends / receives into one
launch on the xGMI links between neighbouring GPUs).
"""
import os

import torch
import torch.distributed as dist

_COMMS = {}


def get_unique_nccl_id(n):
    """``n`` random 128-byte communicator ids (uint8 [n, 128]); rank 0's are broadcast by the caller."""
    return torch.frombuffer(bytearray(os.urandom(128 * n)), dtype=torch.uint8).view(n, 128).clone()


def init_nccl_comm(unique_id, my_rank, num_ranks):
    """Collective: the private communicator (process group over ranks 0..num_ranks-1) for ``unique_id``."""
    key = bytes(unique_id.cpu().contiguous().view(-1)[:128].tolist())
    if key not in _COMMS:
        assert dist.get_rank() == my_rank, "init_nccl_comm: my_rank must be this process's global rank"
        _COMMS[key] = dist.new_group(ranks=list(range(num_ranks)))
    return _COMMS[key]


def _exchange(handle, left_rank, right_rank, left_out, right_out, left_in, right_in):
    ops = []
    if left_rank >= 0:
        ops.append(dist.P2POp(dist.isend, left_out.contiguous(), left_rank, handle))
        ops.append(dist.P2POp(dist.irecv, left_in, left_rank, handle))
    if right_rank >= 0:
        ops.append(dist.P2POp(dist.isend, right_out.contiguous(), right_rank, handle))
        ops.append(dist.P2POp(dist.irecv, right_in, right_rank, handle))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    if left_rank < 0:
        left_in.zero_()
    if right_rank < 0:
        right_in.zero_()


def left_right_halo_exchange(handle, left_rank, right_rank, left_output_halo, right_output_halo):
    """Send my left/right boundary rows, receive the neighbours' -> (left_input_halo, right_input_halo).
    A rank of -1 means no neighbour (its input halo is zero)."""
    left_in = torch.empty_like(right_output_halo, memory_format=torch.contiguous_format)
    right_in = torch.empty_like(left_output_halo, memory_format=torch.contiguous_format)
    _exchange(handle, left_rank, right_rank, left_output_halo, right_output_halo, left_in, right_in)
    return left_in, right_in


def left_right_halo_exchange_inplace(handle, left_rank, right_rank, left_output_halo, right_output_halo,
                                     left_input_halo, right_input_halo):
    li = torch.empty_like(left_input_halo, memory_format=torch.contiguous_format)
    ri = torch.empty_like(right_input_halo, memory_format=torch.contiguous_format)
    _exchange(handle, left_rank, right_rank, left_output_halo, right_output_halo, li, ri)
    left_input_halo.copy_(li)
    right_input_halo.copy_(ri)


def add_delay(delay):
    """Reference debugging hook: enqueue a ``delay`` ns busy kernel on the current stream (GPU only)."""
    if torch.cuda.is_available():
        torch.cuda._sleep(max(1, int(delay * 2.4)))  # ~2.4 GHz shader clock on MI355X
