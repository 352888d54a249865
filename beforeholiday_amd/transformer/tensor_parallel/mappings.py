"""Autograd-aware TP / sequence-parallel collectives (reference: apex/transformer/tensor_parallel/mappings.py:23-304).

Each region mapping is a pair of conjugate collectives (forward op, its adjoint in backward):

  copy_to       identity        / all-reduce
  reduce_from   all-reduce      / identity
  scatter_to    split last dim  / all-gather last dim
  gather_from   all-gather last / split last dim
  scatter_to_sequence  split dim 0 / all-gather dim 0
  gather_from_sequence all-gather dim 0 / reduce-scatter dim 0 (or split when not feeding a TP region)
  reduce_scatter_to_sequence reduce-scatter dim 0 / all-gather dim 0

All gathers use ONE ``all_gather_into_tensor`` into a flat buffer (contiguous dim-0 concatenation) and
all reductions one ``reduce_scatter_tensor`` / ``all_reduce``: on RCCL over xGMI a single large
collective per call is the efficient shape; the last-dim gather permutes the dim-0 result in one copy.
"""
import torch

from .. import parallel_state
from .utils import split_tensor_along_last_dim


def _tp_group():
    return parallel_state.get_tensor_model_parallel_group()


def _tp_world():
    return parallel_state.get_tensor_model_parallel_world_size()


def _reduce(input_: torch.Tensor) -> torch.Tensor:
    if _tp_world() == 1:
        return input_
    torch.distributed.all_reduce(input_, group=_tp_group())
    return input_


def _split_along_last_dim(input_: torch.Tensor) -> torch.Tensor:
    world = _tp_world()
    if world == 1:
        return input_
    return split_tensor_along_last_dim(input_, world)[parallel_state.get_tensor_model_parallel_rank()].contiguous()


def _split_along_first_dim(input_: torch.Tensor) -> torch.Tensor:
    world = _tp_world()
    if world == 1:
        return input_
    n = input_.size(0)
    assert n % world == 0, "First dimension of the tensor should be divisible by tensor parallel size"
    part = n // world
    r = parallel_state.get_tensor_model_parallel_rank()
    return input_[r * part:(r + 1) * part].contiguous()


def all_gather_first_dim(input_: torch.Tensor, group=None, async_op=False):
    """[n, ...] per rank -> [world*n, ...]; returns (out, work)."""
    group = group if group is not None else _tp_group()
    world = torch.distributed.get_world_size(group=group)
    input_ = input_.contiguous()
    out = torch.empty((world * input_.size(0),) + tuple(input_.shape[1:]), dtype=input_.dtype, device=input_.device)
    work = torch.distributed.all_gather_into_tensor(out.view(-1), input_.view(-1), group=group, async_op=async_op)
    return out, work


def reduce_scatter_first_dim(input_: torch.Tensor, group=None, async_op=False):
    """[world*n, ...] per rank -> sum over ranks of this rank's [n, ...] block; returns (out, work)."""
    group = group if group is not None else _tp_group()
    world = torch.distributed.get_world_size(group=group)
    input_ = input_.contiguous()
    assert input_.size(0) % world == 0, "First dimension of the tensor should be divisible by tensor parallel size"
    out = torch.empty((input_.size(0) // world,) + tuple(input_.shape[1:]), dtype=input_.dtype, device=input_.device)
    work = torch.distributed.reduce_scatter_tensor(out.view(-1), input_.view(-1), group=group, async_op=async_op)
    return out, work


def _gather_along_last_dim(input_: torch.Tensor) -> torch.Tensor:
    world = _tp_world()
    if world == 1:
        return input_
    g, _ = all_gather_first_dim(input_)
    # [world*s, ..., h] -> [s, ..., world*h]
    g = g.view((world,) + tuple(input_.shape))
    return torch.cat(g.unbind(0), dim=-1).contiguous()


def _gather_along_first_dim(input_: torch.Tensor) -> torch.Tensor:
    if _tp_world() == 1:
        return input_
    return all_gather_first_dim(input_)[0]


def _reduce_scatter_along_first_dim(input_: torch.Tensor) -> torch.Tensor:
    if _tp_world() == 1:
        return input_
    return reduce_scatter_first_dim(input_)[0]


class _CopyToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return input_

    @staticmethod
    def backward(ctx, grad_output):
        return _reduce(grad_output)


class _ReduceFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _reduce(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output


class _ScatterToModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _split_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_last_dim(grad_output)


class _GatherFromModelParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _gather_along_last_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _split_along_last_dim(grad_output)


class _ScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _split_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_first_dim(grad_output)


class _GatherFromSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_, to_model_parallel: bool = True):
        ctx.to_model_parallel = to_model_parallel
        return _gather_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        if ctx.to_model_parallel:
            return _reduce_scatter_along_first_dim(grad_output), None
        return _split_along_first_dim(grad_output), None


class _ReduceScatterToSequenceParallelRegion(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input_):
        return _reduce_scatter_along_first_dim(input_)

    @staticmethod
    def backward(ctx, grad_output):
        return _gather_along_first_dim(grad_output)


def copy_to_tensor_model_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _CopyToModelParallelRegion.apply(input_)


def reduce_from_tensor_model_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _ReduceFromModelParallelRegion.apply(input_)


def scatter_to_tensor_model_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _ScatterToModelParallelRegion.apply(input_)


def gather_from_tensor_model_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _GatherFromModelParallelRegion.apply(input_)


def scatter_to_sequence_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _ScatterToSequenceParallelRegion.apply(input_)


def gather_from_sequence_parallel_region(input_: torch.Tensor, to_model_parallel: bool = True) -> torch.Tensor:
    return _GatherFromSequenceParallelRegion.apply(input_, to_model_parallel)


def reduce_scatter_to_sequence_parallel_region(input_: torch.Tensor) -> torch.Tensor:
    return _ReduceScatterToSequenceParallelRegion.apply(input_)


__all__ = [
    "copy_to_tensor_model_parallel_region",
    "reduce_from_tensor_model_parallel_region",
    "scatter_to_tensor_model_parallel_region",
    "gather_from_tensor_model_parallel_region",
    "scatter_to_sequence_parallel_region",
    "gather_from_sequence_parallel_region",
    "reduce_scatter_to_sequence_parallel_region",
]
