"""Interleaved (virtual-stage) 1F1B schedule
(reference: apex/transformer/pipeline_parallel/schedules/fwd_bwd_pipelining_with_interleaving.py:26-415).

Each rank holds ``num_model_chunks`` non-contiguous model chunks; microbatches visit chunk 0 of every
rank, then chunk 1, ... (the next rank of the last physical stage wraps to rank 0), which shrinks the
pipeline bubble by the number of chunks. Microbatch k in the forward order runs on chunk
``(k mod (pp*chunks)) // pp``; the backward order visits chunks in reverse.
"""
from typing import List, Optional

import torch

from ... import parallel_state
from .. import p2p_communication
from ..utils import get_kth_microbatch, get_model_type, get_num_microbatches
from .common import FwdStepFunc, backward_step, forward_step, free_output_tensor


def _forward_backward_pipelining_with_interleaving(
        forward_step_func: FwdStepFunc, batch, model: List[torch.nn.Module], *, forward_only: bool,
        tensor_shape=None, dtype: Optional[torch.dtype] = None, grad_scaler=None, disable_autocast: bool = False,
        deallocate_pipeline_outputs: bool = False, async_comm: bool = False, sequence_parallel_enabled: bool = False,
        **kwargs):
    if not isinstance(model, list):
        raise RuntimeError("`model` must be a list of `nn.Module`'s'")
    num_model_chunks = len(model)
    input_tensors = [[] for _ in range(num_model_chunks)]
    output_tensors = [[] for _ in range(num_model_chunks)]
    output_tensor_grads = [[] for _ in range(num_model_chunks)]
    curr_iters = [0 for _ in range(num_model_chunks)]
    losses_reduced = []
    if not forward_only:
        output_tensor_grads = [[] for _ in range(num_model_chunks)]

    pp = parallel_state.get_pipeline_model_parallel_world_size()
    rank = parallel_state.get_pipeline_model_parallel_rank()
    model_type = get_model_type(model[0])
    if sequence_parallel_enabled:
        s, b, h = tensor_shape
        tensor_shape = (s // parallel_state.get_tensor_model_parallel_world_size(), b, h)
    comm = dict(dtype=dtype, async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)

    num_microbatches = get_num_microbatches() * num_model_chunks
    all_warmup = False
    if forward_only:
        num_warmup = num_microbatches
    elif get_num_microbatches() == pp:
        num_warmup = num_microbatches
        all_warmup = True
    else:
        num_warmup = min((pp - rank - 1) * 2 + (num_model_chunks - 1) * pp, num_microbatches)
    num_remaining = num_microbatches - num_warmup

    def chunk_id(k: int, forward: bool) -> int:
        c = (k % (pp * num_model_chunks)) // pp
        return c if forward else num_model_chunks - c - 1

    def forward_helper(k: int):
        c = chunk_id(k, True)
        parallel_state.set_virtual_pipeline_model_parallel_rank(c)
        if parallel_state.is_pipeline_first_stage() and len(input_tensors[c]) == len(output_tensors[c]):
            input_tensors[c].append(None)
        out = forward_step(forward_step_func, get_kth_microbatch(batch, curr_iters[c]), model[c],
                           input_tensors[c][-1], losses_reduced, dtype, disable_autocast)
        curr_iters[c] += 1
        output_tensors[c].append(out)
        if forward_only:
            input_tensors[c].pop()
            output_tensors[c].pop()
        return out

    def backward_helper(k: int):
        c = chunk_id(k, False)
        parallel_state.set_virtual_pipeline_model_parallel_rank(c)
        if parallel_state.is_pipeline_last_stage() and len(output_tensor_grads[c]) == 0:
            output_tensor_grads[c].append(None)
        return backward_step(input_tensors[c].pop(0), output_tensors[c].pop(0), output_tensor_grads[c].pop(0),
                             model_type=model_type, grad_scaler=grad_scaler,
                             deallocate_pipeline_outputs=deallocate_pipeline_outputs)

    # warm-up
    parallel_state.set_virtual_pipeline_model_parallel_rank(0)
    input_tensors[0].append(p2p_communication.recv_forward(tensor_shape=tensor_shape, **comm))
    for k in range(num_warmup):
        output_tensor = forward_helper(k)
        next_c = chunk_id(k + 1, True)
        recv_prev = True
        if parallel_state.is_pipeline_first_stage(ignore_virtual=True) and next_c == 0:
            recv_prev = False
        if k == num_microbatches - 1:
            recv_prev = False
        if parallel_state.is_pipeline_last_stage():
            output_tensor = None
        if k == num_warmup - 1 and not forward_only and not all_warmup:
            recv_next = not parallel_state.is_pipeline_last_stage(ignore_virtual=True)
            input_tensor, output_tensor_grad = p2p_communication.send_forward_backward_recv_forward_backward(
                output_tensor, None, recv_prev=recv_prev, recv_next=recv_next, tensor_shape=tensor_shape, **comm)
            output_tensor_grads[num_model_chunks - 1].append(output_tensor_grad)
        else:
            input_tensor = p2p_communication.send_forward_recv_forward(output_tensor, recv_prev=recv_prev,
                                                                       tensor_shape=tensor_shape, **comm)
        input_tensors[next_c].append(input_tensor)
        free_output_tensor(output_tensor, deallocate_pipeline_outputs)

    # steady state: 1F1B
    for k in range(num_remaining):
        forward_k = k + num_warmup
        output_tensor = forward_helper(forward_k)
        backward_k = k
        input_tensor_grad = backward_helper(backward_k)

        parallel_state.set_virtual_pipeline_model_parallel_rank(chunk_id(forward_k, True))
        if parallel_state.is_pipeline_last_stage():
            output_tensor = None
        parallel_state.set_virtual_pipeline_model_parallel_rank(chunk_id(backward_k, False))
        if parallel_state.is_pipeline_first_stage():
            input_tensor_grad = None

        recv_prev = True
        if parallel_state.is_pipeline_first_stage(ignore_virtual=True):
            next_forward_c = chunk_id(forward_k - (pp - 1), True)
            if next_forward_c == num_model_chunks - 1:
                recv_prev = False
            next_forward_c += 1
        else:
            next_forward_c = chunk_id(forward_k + 1, True)
        recv_next = True
        if parallel_state.is_pipeline_last_stage(ignore_virtual=True):
            next_backward_c = chunk_id(backward_k - (pp - 1), False)
            if next_backward_c == 0:
                recv_next = False
            next_backward_c -= 1
        else:
            next_backward_c = chunk_id(backward_k + 1, False)
        if k == num_remaining - 1:
            recv_prev = False

        input_tensor, output_tensor_grad = p2p_communication.send_forward_backward_recv_forward_backward(
            output_tensor, input_tensor_grad, recv_prev=recv_prev, recv_next=recv_next, tensor_shape=tensor_shape,
            **comm)
        free_output_tensor(output_tensor, deallocate_pipeline_outputs)
        if recv_prev:
            input_tensors[next_forward_c].append(input_tensor)
        if recv_next:
            output_tensor_grads[next_backward_c].append(output_tensor_grad)

    # cool-down
    if not forward_only:
        if all_warmup:
            output_tensor_grads[num_model_chunks - 1].append(
                p2p_communication.recv_backward(tensor_shape=tensor_shape, **comm))
        for k in range(num_remaining, num_microbatches):
            input_tensor_grad = backward_helper(k)
            next_backward_c = chunk_id(k + 1, False)
            recv_next = True
            if parallel_state.is_pipeline_last_stage(ignore_virtual=True) and next_backward_c == num_model_chunks - 1:
                recv_next = False
            if k == num_microbatches - 1:
                recv_next = False
            output_tensor_grads[next_backward_c].append(p2p_communication.send_backward_recv_backward(
                input_tensor_grad, recv_next=recv_next, tensor_shape=tensor_shape, **comm))
    parallel_state.set_virtual_pipeline_model_parallel_rank(0)
    return losses_reduced
