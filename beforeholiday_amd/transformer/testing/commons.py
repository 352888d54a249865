"""Toy models and helpers for pipeline / tensor-parallel tests (reference: apex/transformer/testing/commons.py:40-297)."""
import datetime
import os
import random
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple, Union

import numpy
import torch
import torch.nn as nn

from .. import parallel_state, tensor_parallel
from ..pipeline_parallel.utils import average_losses_across_data_parallel_group
from ..tensor_parallel import ColumnParallelLinear, RowParallelLinear, scatter_to_sequence_parallel_region

TEST_SUCCESS_MESSAGE = ">> passed the test :-)"


class MyLayer(nn.Module):
    def __init__(self, hidden_size: int, pre_process: bool, post_process: bool):
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.layer = nn.Linear(hidden_size, hidden_size)

    def forward(self, x):
        return self.layer(x)


class MyModel(nn.Module):
    def __init__(self, hidden_size: int, pre_process: bool = False, post_process: bool = False, *,
                 add_encoder: bool = False, add_decoder: bool = False) -> None:
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.layer = MyLayer(hidden_size=hidden_size, pre_process=pre_process, post_process=post_process)
        self.input_tensor = None

    def set_input_tensor(self, input_tensor: Union[torch.Tensor, List[torch.Tensor]]) -> None:
        if not isinstance(input_tensor, list):
            input_tensor = [input_tensor]
        self.input_tensor = input_tensor[0]

    def forward(self, x: Optional[torch.Tensor]) -> torch.Tensor:
        return self.layer(x if self.input_tensor is None else self.input_tensor)


class ToyParallelMLP(nn.Module):
    """h -> 4h (column parallel, GELU) -> h (row parallel), optionally sequence parallel."""

    def __init__(self, hidden_size: int, pre_process: bool = False, post_process: bool = False, *,
                 sequence_parallel_enabled: bool = False, add_encoder: bool = False, add_decoder: bool = False,
                 use_cpu_initialization: bool = False) -> None:
        super().__init__()
        self.pre_process = pre_process
        self.post_process = post_process
        self.sequence_parallel_enabled = sequence_parallel_enabled
        ffn = 4 * hidden_size
        self.dense_h_to_4h = ColumnParallelLinear(hidden_size, ffn, gather_output=False, skip_bias_add=True, bias=True,
                                                  sequence_parallel_enabled=sequence_parallel_enabled,
                                                  no_async_tensor_model_parallel_allreduce=True,
                                                  use_cpu_initialization=use_cpu_initialization)
        self.dense_4h_to_h = RowParallelLinear(ffn, hidden_size, input_is_parallel=True, skip_bias_add=False,
                                               bias=True, sequence_parallel_enabled=sequence_parallel_enabled,
                                               use_cpu_initialization=use_cpu_initialization)
        self.activation_func = torch.nn.GELU()
        self.input_tensor = None

    def set_input_tensor(self, input_tensor) -> None:
        if not isinstance(input_tensor, list):
            input_tensor = [input_tensor]
        self.input_tensor = input_tensor[0]

    def forward(self, x: Optional[torch.Tensor]) -> torch.Tensor:
        inp = x if self.input_tensor is None else self.input_tensor
        inter, bias = self.dense_h_to_4h(inp)
        if bias is not None:
            inter = inter + bias
        out, _ = self.dense_4h_to_h(self.activation_func(inter))
        return out


def model_provider_func(hidden_size: int, pre_process: bool, post_process: bool, *, add_encoder: bool = False,
                        add_decoder: bool = False) -> MyModel:
    return MyModel(hidden_size, pre_process, post_process, add_encoder=add_encoder, add_decoder=add_decoder)


def mlp_provider_func(hidden_size: int, pre_process: bool, post_process: bool, *, add_encoder: bool = False,
                      add_decoder: bool = False, sequence_parallel_enabled: bool = False,
                      use_cpu_initialization: bool = False) -> ToyParallelMLP:
    return ToyParallelMLP(hidden_size, pre_process, post_process, add_encoder=add_encoder, add_decoder=add_decoder,
                          sequence_parallel_enabled=sequence_parallel_enabled,
                          use_cpu_initialization=use_cpu_initialization)


def process_batch(batch):
    return batch[0] if isinstance(batch, list) else batch


def _sum_loss(x):
    loss = torch.sum(x)
    return loss, {"avg": average_losses_across_data_parallel_group([loss])}


def fwd_step_func(batch, model):
    return model(process_batch(batch)), _sum_loss


@dataclass(frozen=True)
class ToyParallelMLPFwdBwdStepFunc:
    sequence_parallel_enabled: bool

    def __call__(self, batch, model: torch.nn.Module):
        x = batch[0] if isinstance(batch, list) else batch
        if isinstance(x, torch.Tensor):
            x = x.transpose(0, 1).contiguous()
            if self.sequence_parallel_enabled:
                x = scatter_to_sequence_parallel_region(x)
        return model(x), _sum_loss


class IdentityLayer(torch.nn.Module):
    def __init__(self, size, scale=1.0):
        super().__init__()
        self.weight = torch.nn.Parameter(scale * torch.randn(size))

    def forward(self):
        return self.weight


def set_random_seed(seed):
    random.seed(seed)
    numpy.random.seed(seed)
    torch.manual_seed(seed)
    tensor_parallel.model_parallel_cuda_manual_seed(seed)


def initialize_distributed(backend="nccl"):
    """Init torch.distributed from RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (tcp) and bind the GPU."""
    if backend not in ("nccl", "ucc", "gloo"):
        raise RuntimeError(f"Currently only nccl, ucc & gloo are supported but {backend}")
    rank = int(os.getenv("RANK", "0"))
    world_size = int(os.getenv("WORLD_SIZE", "1"))
    local_rank = os.getenv("LOCAL_RANK")
    if torch.cuda.is_available():
        torch.cuda.set_device(int(local_rank) if local_rank is not None else rank % torch.cuda.device_count())
    init_method = f"tcp://{os.getenv('MASTER_ADDR', '127.0.0.1')}:{os.getenv('MASTER_PORT', '6000')}"
    torch.distributed.init_process_group(backend=backend, world_size=world_size, rank=rank, init_method=init_method,
                                         timeout=datetime.timedelta(seconds=60))


def print_separator(message):
    torch.distributed.barrier()
    filler = "-" * ((78 - len(message)) // 2)
    if torch.distributed.get_rank() == 0:
        print(f"\n{filler} {message} {filler}", flush=True)
    torch.distributed.barrier()
