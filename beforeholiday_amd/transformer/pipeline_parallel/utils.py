"""Pipeline-parallel utilities: global microbatch calculator, microbatch slicing, model helpers,
diagnostics (reference: apex/transformer/pipeline_parallel/utils.py:31-357)."""
from typing import List, Optional, Union

import torch
from torch.nn.parallel import DistributedDataParallel

from .. import parallel_state
from ..enums import ModelType
from ..microbatches import build_num_microbatches_calculator
from ._timers import _Timers

_GLOBAL_ARGS = None
_GLOBAL_NUM_MICROBATCHES_CALCULATOR = None
_GLOBAL_TOKENIZER = None
_GLOBAL_TENSORBOARD_WRITER = None
_GLOBAL_AUTORESUME = None
_GLOBAL_TIMERS = None


def listify_model(model: Union[torch.nn.Module, List[torch.nn.Module]]) -> List[torch.nn.Module]:
    return model if isinstance(model, list) else [model]


def _ensure_var_is_initialized(var, name):
    assert var is not None, f"{name} is not initialized."


def _ensure_var_is_not_initialized(var, name):
    assert var is None, f"{name} is already initialized."


def setup_microbatch_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                micro_batch_size: int, data_parallel_size: int) -> None:
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _ensure_var_is_not_initialized(_GLOBAL_NUM_MICROBATCHES_CALCULATOR, "num microbatches calculator")
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def _reconfigure_microbatch_calculator(rank: int, rampup_batch_size: Optional[List[int]], global_batch_size: int,
                                       micro_batch_size: int, data_parallel_size: int) -> None:
    """Replace the global calculator (tests only)."""
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = build_num_microbatches_calculator(
        rank, rampup_batch_size, global_batch_size, micro_batch_size, data_parallel_size)


def destroy_microbatch_calculator():
    global _GLOBAL_NUM_MICROBATCHES_CALCULATOR
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR = None


def get_micro_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.micro_batch_size


def get_num_microbatches():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get()


def get_current_global_batch_size():
    return _GLOBAL_NUM_MICROBATCHES_CALCULATOR.get_current_global_batch_size()


def update_num_microbatches(consumed_samples, consistency_check=True):
    _GLOBAL_NUM_MICROBATCHES_CALCULATOR.update(consumed_samples, consistency_check)


def _split_batch_into_microbatch(batch: List[torch.Tensor], *, _micro_batch_size: Optional[int] = None,
                                 _global_batch_size: Optional[int] = None):
    mbs = _micro_batch_size or get_micro_batch_size()
    gbs = _global_batch_size or get_current_global_batch_size()
    for i in range(0, gbs, mbs):
        yield [x[i:i + mbs] for x in batch]


def get_kth_microbatch(batch: Optional[List[torch.Tensor]], k: int) -> List[torch.Tensor]:
    """k-th ``micro_batch_size`` slice (dim 0) of every tensor of the local minibatch."""
    if batch is None:
        return batch
    mbs = get_micro_batch_size()
    start, end = k * mbs, (k + 1) * mbs
    out = []
    for x in batch:
        assert x.size(0) > start and x.size(0) >= end
        out.append(x[start:end])
    assert out
    return out


def get_autoresume():
    return _GLOBAL_AUTORESUME


def _set_timers():
    global _GLOBAL_TIMERS
    _ensure_var_is_not_initialized(_GLOBAL_TIMERS, "timers")
    _GLOBAL_TIMERS = _Timers()


def get_timers():
    _ensure_var_is_initialized(_GLOBAL_TIMERS, "timers")
    return _GLOBAL_TIMERS


def print_rank_0(message: str) -> None:
    if torch.distributed.is_initialized():
        if torch.distributed.get_rank() == 0:
            print(message, flush=True)
    else:
        print(message, flush=True)


def is_last_rank():
    return torch.distributed.get_rank() == (torch.distributed.get_world_size() - 1)


def print_rank_last(message):
    if torch.distributed.is_initialized():
        if is_last_rank():
            print(message, flush=True)
    else:
        print(message, flush=True)


def param_is_not_shared(param: torch.nn.Parameter) -> bool:
    return getattr(param, "shared", False) is False


def unwrap_model(model, module_instances=(DistributedDataParallel,)):
    return_list = True
    if not isinstance(model, list):
        model = [model]
        return_list = False
    unwrapped = []
    for m in model:
        while isinstance(m, module_instances):
            m = m.module
        unwrapped.append(m)
    return unwrapped if return_list else unwrapped[0]


def get_model_type(model: torch.nn.Module) -> ModelType:
    return getattr(unwrap_model(model), "model_type", ModelType.encoder_or_decoder)


def calc_params_l2_norm(model: torch.nn.Module, bf16: bool):
    """L2 norm of all non-duplicated parameters across the model-parallel group (one fused l2norm
    launch + one scalar all-reduce)."""
    from ...multi_tensor_apply import multi_tensor_applier
    from ...ops import amp_C
    from ..tensor_parallel.layers import param_is_not_tensor_parallel_duplicate
    models = model if isinstance(model, list) else [model]
    params = []
    for m in models:
        for p in m.parameters():
            if param_is_not_shared(p) and param_is_not_tensor_parallel_duplicate(p):
                params.append(p.data.float() if bf16 else p.data)
    dev = params[0].device if params else torch.device("cpu")
    flag = torch.zeros(1, dtype=torch.int, device=dev)
    norm, _ = multi_tensor_applier(amp_C.multi_tensor_l2norm, flag, [params], False)
    norm_2 = norm * norm
    torch.distributed.all_reduce(norm_2, op=torch.distributed.ReduceOp.SUM,
                                 group=parallel_state.get_model_parallel_group())
    return norm_2.item() ** 0.5


def average_losses_across_data_parallel_group(losses):
    averaged = torch.cat([loss.clone().detach().view(1) for loss in losses])
    torch.distributed.all_reduce(averaged, group=parallel_state.get_data_parallel_group())
    return averaged / torch.distributed.get_world_size(group=parallel_state.get_data_parallel_group())


def report_memory(name):
    mb = 1024.0 * 1024.0
    s = (f"{name} memory (MB) | allocated: {torch.cuda.memory_allocated() / mb} | max allocated: "
         f"{torch.cuda.max_memory_allocated() / mb} | reserved: {torch.cuda.memory_reserved() / mb} | max reserved: "
         f"{torch.cuda.max_memory_reserved() / mb}")
    if parallel_state.get_data_parallel_rank() == 0:
        print(f"[Rank {torch.distributed.get_rank()}] {s}", flush=True)


def print_params_min_max_norm(optimizer, iteration):
    rank = torch.distributed.get_rank()
    s = "iteration, rank, index, tensor-model-parallel, min, max, norm\n"
    opt = getattr(optimizer, "optimizer", optimizer)
    index = 0
    for group in opt.param_groups:
        for p in group["params"]:
            index += 1
            s += (f"{iteration:7d}, {rank:4d}, {index:4d}, {int(getattr(p, 'tensor_model_parallel', False)):2d}, "
                  f"{p.data.min():.6E}, {p.data.max():.6E}, {torch.linalg.norm(p.data):.6E}\n")
    print(s, flush=True)


def get_ltor_masks_and_position_ids(data, eod_token, reset_position_ids, reset_attention_mask, eod_mask_loss):
    """Causal attention mask (True = masked), loss mask and position ids for a left-to-right LM batch,
    optionally restarting positions / attention at every end-of-document token."""
    micro_batch_size, seq_length = data.size()
    att_mask_batch = micro_batch_size if reset_attention_mask else 1
    attention_mask = torch.tril(torch.ones((att_mask_batch, seq_length, seq_length), device=data.device)).view(
        att_mask_batch, 1, seq_length, seq_length)
    loss_mask = torch.ones(data.size(), dtype=torch.float, device=data.device)
    if eod_mask_loss:
        loss_mask[data == eod_token] = 0.0
    position_ids = torch.arange(seq_length, dtype=torch.long, device=data.device).unsqueeze(0).expand_as(data)
    if reset_position_ids:
        position_ids = position_ids.clone()
    if reset_position_ids or reset_attention_mask:
        for b in range(micro_batch_size):
            eod_index = position_ids[b, data[b] == eod_token].tolist()
            prev = 0
            for i in eod_index:
                if reset_attention_mask:
                    attention_mask[b, 0, (i + 1):, :(i + 1)] = 0
                if reset_position_ids:
                    position_ids[b, (i + 1):] -= i + 1 - prev
                    prev = i + 1
    return attention_mask < 0.5, loss_mask, position_ids
