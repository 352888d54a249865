"""Megatron tensor-parallel layers (reference: apex/transformer/tensor_parallel/layers.py:69-780).

``ColumnParallelLinear`` splits the weight's output dim, ``RowParallelLinear`` its input dim,
``VocabParallelEmbedding`` the vocabulary. The shared autograd core
(:class:`LinearWithGradAccumulationAndAsyncCommunication`) orders the backward so RCCL collectives
overlap with GEMMs: the sequence-parallel all-gather of the input is issued async and waited only
after dgrad; the dgrad all-reduce / reduce-scatter is issued async and overlapped with the wgrad GEMM.
With ``gradient_accumulation_fusion`` the wgrad GEMM accumulates straight into ``weight.main_grad``
(fp32 or 16-bit) through ``fused_weight_gradient_mlp_cuda``.
"""
import warnings
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch.nn import init
from torch.nn.parameter import Parameter

from ..._autocast_utils import _cast_if_autocast_enabled
from ...ops.fused_dense import bias_grad as _bias_grad
from ...ops.fused_dense import weight_grad as _weight_grad
from ..parallel_state import (get_tensor_model_parallel_group, get_tensor_model_parallel_rank,
                              get_tensor_model_parallel_world_size)
from ..utils import divide
from .mappings import (all_gather_first_dim, copy_to_tensor_model_parallel_region,
                       gather_from_tensor_model_parallel_region, reduce_from_tensor_model_parallel_region,
                       reduce_scatter_first_dim, reduce_scatter_to_sequence_parallel_region,
                       scatter_to_tensor_model_parallel_region)
from .random import get_cuda_rng_tracker
from .utils import VocabUtility

_MODEL_PARALLEL_ATTRIBUTE_DEFAULTS = {"tensor_model_parallel": False, "partition_dim": -1, "partition_stride": 1}

_grad_accum_fusion_available = True


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def param_is_not_tensor_parallel_duplicate(param: torch.Tensor) -> bool:
    return (hasattr(param, "tensor_model_parallel") and param.tensor_model_parallel) or \
        (get_tensor_model_parallel_rank() == 0)


def set_tensor_model_parallel_attributes(tensor: torch.Tensor, is_parallel: bool, dim: int, stride: int) -> None:
    for attribute in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        assert not hasattr(tensor, attribute)
    setattr(tensor, "tensor_model_parallel", is_parallel)
    setattr(tensor, "partition_dim", dim)
    setattr(tensor, "partition_stride", stride)


def set_defaults_if_not_set_tensor_model_parallel_attributes(tensor: torch.Tensor) -> None:
    for attribute, value in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS.items():
        if not hasattr(tensor, attribute):
            setattr(tensor, attribute, value)


def copy_tensor_model_parallel_attributes(destination_tensor: torch.Tensor, source_tensor: torch.Tensor) -> None:
    for attribute in _MODEL_PARALLEL_ATTRIBUTE_DEFAULTS:
        if hasattr(source_tensor, attribute):
            setattr(destination_tensor, attribute, getattr(source_tensor, attribute))


def _initialize_affine_weight_gpu(weight, init_method, partition_dim, stride=1):
    """Initialise this rank's shard in place under the TP RNG stream (shards differ across TP ranks)."""
    set_tensor_model_parallel_attributes(tensor=weight, is_parallel=True, dim=partition_dim, stride=stride)
    with get_cuda_rng_tracker().fork():
        init_method(weight)


def _initialize_affine_weight_cpu(weight, output_size, input_size, per_partition_size, partition_dim, init_method,
                                  stride=1, return_master_weight=False, *, params_dtype=torch.float32):
    """Initialise the full fp32 master weight identically on every rank, keep the strided shard."""
    set_tensor_model_parallel_attributes(tensor=weight, is_parallel=True, dim=partition_dim, stride=stride)
    master = torch.empty(output_size, input_size, dtype=torch.float, requires_grad=False)
    init_method(master)
    master = master.to(dtype=params_dtype)
    pieces = torch.split(master, divide(per_partition_size, stride), dim=partition_dim)
    mine = pieces[get_tensor_model_parallel_rank()::get_tensor_model_parallel_world_size()]
    with torch.no_grad():
        weight.copy_(torch.cat(mine, dim=partition_dim))
    return master if return_master_weight else None


class VocabParallelEmbedding(torch.nn.Module):
    """Embedding whose vocabulary rows are sharded over the TP group; out-of-shard tokens contribute
    zeros and one all-reduce sums the shards."""

    def __init__(self, num_embeddings: int, embedding_dim: int, init_method=init.xavier_normal_, *,
                 params_dtype: torch.dtype = torch.float32, use_cpu_initialization: bool = False):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.embedding_dim = embedding_dim
        self.padding_idx = None
        self.max_norm = None
        self.norm_type = 2.0
        self.scale_grad_by_freq = False
        self.sparse = False
        self._weight = None
        self.tensor_model_parallel_size = get_tensor_model_parallel_world_size()
        self.vocab_start_index, self.vocab_end_index = VocabUtility.vocab_range_from_global_vocab_size(
            num_embeddings, get_tensor_model_parallel_rank(), self.tensor_model_parallel_size)
        self.num_embeddings_per_partition = self.vocab_end_index - self.vocab_start_index
        if use_cpu_initialization:
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, embedding_dim, dtype=params_dtype))
            _initialize_affine_weight_cpu(self.weight, num_embeddings, embedding_dim,
                                          self.num_embeddings_per_partition, 0, init_method,
                                          params_dtype=params_dtype)
        else:
            self.weight = Parameter(torch.empty(self.num_embeddings_per_partition, embedding_dim,
                                                device=_default_device(), dtype=params_dtype))
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0, stride=1)

    def forward(self, input_):
        if self.tensor_model_parallel_size > 1:
            input_mask = (input_ < self.vocab_start_index) | (input_ >= self.vocab_end_index)
            masked_input = (input_ - self.vocab_start_index).masked_fill_(input_mask, 0)
        else:
            masked_input = input_
        if self.max_norm is None and not self.scale_grad_by_freq and not self.sparse:
            from ...ops import fused_dense as _fd

            output_parallel = _fd.embedding(masked_input, self.weight, self.padding_idx)
        else:
            output_parallel = F.embedding(masked_input, self.weight, self.padding_idx, self.max_norm, self.norm_type,
                                          self.scale_grad_by_freq, self.sparse)
        if self.tensor_model_parallel_size > 1:
            output_parallel = output_parallel.masked_fill(input_mask.unsqueeze(-1), 0.0)
        return reduce_from_tensor_model_parallel_region(output_parallel)


def _wgrad_accumulate(total_input_2d, grad_output_2d, main_grad, use_16bit):
    from ...ops import fused_dense as _fd
    if use_16bit:
        _fd.wgrad_gemm_accum_fp16(total_input_2d, grad_output_2d, main_grad)
    else:
        _fd.wgrad_gemm_accum_fp32(total_input_2d, grad_output_2d, main_grad)


class LinearWithGradAccumulationAndAsyncCommunication(torch.autograd.Function):
    """y = x W^T (+ b) with TP/SP communication folded into forward/backward (see module doc)."""

    @staticmethod
    def forward(ctx, input, weight, bias, gradient_accumulation_fusion, async_grad_allreduce,
                sequence_parallel_enabled, use_16bit_in_wgrad_accum_fusion=False):
        ctx.save_for_backward(input, weight)
        ctx.use_bias = bias is not None
        ctx.gradient_accumulation_fusion = gradient_accumulation_fusion
        ctx.async_grad_allreduce = async_grad_allreduce
        ctx.sequence_parallel_enabled = sequence_parallel_enabled
        ctx.use_16bit_in_wgrad_accum_fusion = use_16bit_in_wgrad_accum_fusion
        total_input = all_gather_first_dim(input)[0] if sequence_parallel_enabled else input
        return F.linear(total_input, weight, bias)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        handle = None
        if ctx.sequence_parallel_enabled:
            total_input, handle = all_gather_first_dim(input, async_op=True)
        else:
            total_input = input
        grad_input = grad_output.matmul(weight)
        if handle is not None:
            handle.wait()
        grad_output_2d = grad_output.reshape(-1, grad_output.shape[-1])
        total_input_2d = total_input.reshape(-1, total_input.shape[-1])
        comm = None
        sub_grad_input = None
        if ctx.async_grad_allreduce:
            comm = torch.distributed.all_reduce(grad_input, group=get_tensor_model_parallel_group(), async_op=True)
        if ctx.sequence_parallel_enabled:
            assert not ctx.async_grad_allreduce
            sub_grad_input, comm = reduce_scatter_first_dim(grad_input, async_op=True)
        if ctx.gradient_accumulation_fusion:
            _wgrad_accumulate(total_input_2d, grad_output_2d, weight.main_grad, ctx.use_16bit_in_wgrad_accum_fusion)
            grad_weight = None
        else:
            grad_weight = _weight_grad(grad_output_2d, total_input_2d)
        grad_bias = _bias_grad(grad_output_2d) if ctx.use_bias else None
        if comm is not None:
            comm.wait()
        if ctx.sequence_parallel_enabled:
            return sub_grad_input, grad_weight, grad_bias, None, None, None, None
        return grad_input, grad_weight, grad_bias, None, None, None, None


def linear_with_grad_accumulation_and_async_allreduce(input, weight, bias, gradient_accumulation_fusion,
                                                      async_grad_allreduce, sequence_parallel_enabled):
    args = _cast_if_autocast_enabled(input, weight, bias, gradient_accumulation_fusion, async_grad_allreduce,
                                     sequence_parallel_enabled, False)
    with torch.autocast("cuda", enabled=False):
        return LinearWithGradAccumulationAndAsyncCommunication.apply(*args)


def linear_with_grad_accumulation_and_async_allreduce_in16bit(input, weight, bias, gradient_accumulation_fusion,
                                                              async_grad_allreduce, sequence_parallel_enabled):
    args = _cast_if_autocast_enabled(input, weight, bias, gradient_accumulation_fusion, async_grad_allreduce,
                                     sequence_parallel_enabled, True)
    with torch.autocast("cuda", enabled=False):
        return LinearWithGradAccumulationAndAsyncCommunication.apply(*args)


class ColumnParallelLinear(torch.nn.Module):
    """Y = X A + b with A split along its output (column) dimension: rank i holds A_i and computes
    Y_i = X A_i. ``gather_output`` all-gathers Y; ``skip_bias_add`` returns the bias for fusion.
    Input layout [sequence, batch, hidden]."""

    def __init__(self, input_size, output_size, bias=True, gather_output=True, init_method=init.xavier_normal_,
                 stride=1, keep_master_weight_for_test=False, skip_bias_add=False, *,
                 no_async_tensor_model_parallel_allreduce=False, params_dtype=torch.float32,
                 use_cpu_initialization=False, gradient_accumulation_fusion=False,
                 accumulation_in_fp16: bool = False, sequence_parallel_enabled: bool = False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.gather_output = gather_output
        world_size = get_tensor_model_parallel_world_size()
        self.output_size_per_partition = divide(output_size, world_size)
        self.skip_bias_add = skip_bias_add
        if use_cpu_initialization:
            self.weight = Parameter(torch.empty(self.output_size_per_partition, input_size, dtype=params_dtype))
            self.master_weight = _initialize_affine_weight_cpu(
                self.weight, output_size, input_size, self.output_size_per_partition, 0, init_method, stride=stride,
                return_master_weight=keep_master_weight_for_test, params_dtype=params_dtype)
        else:
            self.weight = Parameter(torch.empty(self.output_size_per_partition, input_size, device=_default_device(),
                                                dtype=params_dtype))
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=0, stride=stride)
        if bias:
            dev = None if use_cpu_initialization else _default_device()
            self.bias = Parameter(torch.empty(self.output_size_per_partition, dtype=params_dtype, device=dev))
            set_tensor_model_parallel_attributes(self.bias, True, 0, stride)
            with torch.no_grad():
                self.bias.zero_()
        else:
            self.register_parameter("bias", None)
        self.async_tensor_model_parallel_allreduce = (not no_async_tensor_model_parallel_allreduce and world_size > 1)
        if sequence_parallel_enabled and world_size <= 1:
            warnings.warn(f"`sequence_parallel_enabled` is set to `True`, but got world_size of {world_size}")
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if gradient_accumulation_fusion and not _grad_accum_fusion_available:
            warnings.warn("`gradient_accumulation_fusion` requested but fused_weight_gradient_mlp_cuda is unavailable")
            gradient_accumulation_fusion = False
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        if self.async_tensor_model_parallel_allreduce and self.sequence_parallel_enabled:
            raise RuntimeError("`async_tensor_model_parallel_allreduce` and `sequence_parallel_enabled` cannot be "
                               "enabled at the same time.")
        self._forward_impl = (linear_with_grad_accumulation_and_async_allreduce_in16bit if accumulation_in_fp16
                              else linear_with_grad_accumulation_and_async_allreduce)

    def forward(self, input_: torch.Tensor) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        bias = self.bias if not self.skip_bias_add else None
        if self.async_tensor_model_parallel_allreduce or self.sequence_parallel_enabled:
            input_parallel = input_
        else:
            input_parallel = copy_to_tensor_model_parallel_region(input_)
        output_parallel = self._forward_impl(
            input=input_parallel, weight=self.weight, bias=bias,
            gradient_accumulation_fusion=self.gradient_accumulation_fusion,
            async_grad_allreduce=self.async_tensor_model_parallel_allreduce,
            sequence_parallel_enabled=self.sequence_parallel_enabled)
        if self.gather_output:
            assert not self.sequence_parallel_enabled
            output = gather_from_tensor_model_parallel_region(output_parallel)
        else:
            output = output_parallel
        return output, (self.bias if self.skip_bias_add else None)


class RowParallelLinear(torch.nn.Module):
    """Y = X A + b with A split along its input (row) dimension and X along its last dimension:
    rank i computes X_i A_i, partial sums are all-reduced (or reduce-scattered along the sequence
    with sequence parallelism). The bias is not split and is added after the reduction."""

    def __init__(self, input_size, output_size, bias=True, input_is_parallel=False, init_method=init.xavier_normal_,
                 stride=1, keep_master_weight_for_test=False, skip_bias_add=False, *, params_dtype=torch.float32,
                 use_cpu_initialization=False, gradient_accumulation_fusion=False,
                 accumulation_in_fp16: bool = False, sequence_parallel_enabled: bool = False):
        super().__init__()
        self.input_size = input_size
        self.output_size = output_size
        self.input_is_parallel = input_is_parallel
        world_size = get_tensor_model_parallel_world_size()
        self.input_size_per_partition = divide(input_size, world_size)
        self.skip_bias_add = skip_bias_add
        self.gradient_accumulation_fusion = gradient_accumulation_fusion
        self.sequence_parallel_enabled = sequence_parallel_enabled
        if self.sequence_parallel_enabled and not self.input_is_parallel:
            raise RuntimeError("To enable `sequence_parallel_enabled`, `input_is_parallel` must be `True`")
        if use_cpu_initialization:
            self.weight = Parameter(torch.empty(output_size, self.input_size_per_partition, dtype=params_dtype))
            self.master_weight = _initialize_affine_weight_cpu(
                self.weight, output_size, input_size, self.input_size_per_partition, 1, init_method, stride=stride,
                return_master_weight=keep_master_weight_for_test, params_dtype=params_dtype)
        else:
            self.weight = Parameter(torch.empty(output_size, self.input_size_per_partition, device=_default_device(),
                                                dtype=params_dtype))
            _initialize_affine_weight_gpu(self.weight, init_method, partition_dim=1, stride=stride)
        if bias:
            dev = None if use_cpu_initialization else _default_device()
            self.bias = Parameter(torch.empty(output_size, dtype=params_dtype, device=dev))
            with torch.no_grad():
                self.bias.zero_()
            setattr(self.bias, "sequence_parallel_enabled", sequence_parallel_enabled)
        else:
            self.register_parameter("bias", None)
        self._forward_impl = (linear_with_grad_accumulation_and_async_allreduce_in16bit if accumulation_in_fp16
                              else linear_with_grad_accumulation_and_async_allreduce)

    def forward(self, input_: torch.Tensor) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        if self.input_is_parallel:
            input_parallel = input_
        else:
            assert not self.sequence_parallel_enabled
            input_parallel = scatter_to_tensor_model_parallel_region(input_)
        output_parallel = self._forward_impl(
            input=input_parallel, weight=self.weight, bias=None,
            gradient_accumulation_fusion=self.gradient_accumulation_fusion, async_grad_allreduce=False,
            sequence_parallel_enabled=False)
        if self.sequence_parallel_enabled:
            output_ = reduce_scatter_to_sequence_parallel_region(output_parallel)
        else:
            output_ = reduce_from_tensor_model_parallel_region(output_parallel)
        if not self.skip_bias_add:
            return (output_ + self.bias if self.bias is not None else output_), None
        return output_, self.bias
