"""Neighbour halo exchange over the process group (reference: apex/contrib/csrc/nccl_p2p/nccl_p2p_cuda.cu,
``nccl_p2p_cuda``: private NCCL communicator + grouped send/recv).

On ROCm the torch.distributed "nccl" backend IS RCCL, so no second communicator is created: a
"handle" is a process group, and one ``batch_isend_irecv`` group moves both halos (RCCL coalesces
the sends/receives into one launch on the xGMI links between neighbouring GPUs).
"""
import torch
import torch.distributed as dist


def get_unique_nccl_id(n):
    """API shim: RCCL communicators come from torch.distributed; returns a dummy id tensor."""
    return torch.zeros(n, 128, dtype=torch.uint8)


def init_nccl_comm(unique_id, my_rank, num_ranks):
    """Returns the communicator handle (the default process group)."""
    return dist.group.WORLD


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
    """Reference debugging hook (spin kernel); a no-op here."""
    return None
