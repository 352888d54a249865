"""Shared helpers for tensor/pipeline parallel (reference: apex/transformer/utils.py:7-48)."""
import torch

from . import parallel_state


def ensure_divisibility(numerator, denominator):
    assert numerator % denominator == 0, f"{numerator} is not divisible by {denominator}"


def divide(numerator, denominator):
    ensure_divisibility(numerator, denominator)
    return numerator // denominator


def split_tensor_into_1d_equal_chunks(tensor):
    """This TP rank's contiguous 1/tp slice of the flattened tensor."""
    data = tensor.view(-1)
    part = data.numel() // parallel_state.get_tensor_model_parallel_world_size()
    start = part * parallel_state.get_tensor_model_parallel_rank()
    return data[start:start + part]


def gather_split_1d_tensor(tensor):
    """Inverse of :func:`split_tensor_into_1d_equal_chunks`: one all-gather into a flat buffer."""
    world = parallel_state.get_tensor_model_parallel_world_size()
    out = torch.empty(world * tensor.numel(), dtype=tensor.dtype, device=tensor.device)
    torch.distributed.all_gather_into_tensor(out, tensor.contiguous().view(-1),
                                             group=parallel_state.get_tensor_model_parallel_group())
    return out
