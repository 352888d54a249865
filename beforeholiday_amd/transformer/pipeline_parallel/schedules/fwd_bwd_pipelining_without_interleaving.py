"""Non-interleaved 1F1B pipeline schedule
(reference: apex/transformer/pipeline_parallel/schedules/fwd_bwd_pipelining_without_interleaving.py:28-489).

Stage r runs (pp - r - 1) warm-up forwards, then alternates one forward / one backward, then drains
the remaining backwards; at most (pp - r) microbatch activations are alive at once.
"""
from typing import List, Optional, Sequence, Union

import torch

from ... import parallel_state
from ...enums import ModelType
from .. import p2p_communication
from ..utils import get_kth_microbatch, get_model_type, get_num_microbatches, listify_model
from .common import Batch, FwdStepFunc, backward_step, forward_step, free_output_tensor


def get_tensor_shapes(rank: int, model_type: ModelType, *, tensor_shape, decoder_sequence_length: Optional[int] = None,
                      sequence_parallel_enabled: bool = False) -> Sequence[Sequence[int]]:
    """Shapes exchanged by stage ``rank``: one [s, b, h] tensor, or (decoder, encoder) pair after the
    encoder/decoder split of a T5-style model. Sequence parallelism divides s by tp."""
    assert len(tensor_shape) == 3, \
        f"`tensor_shape` should be [sequence_length, micro_batch_size, hidden_size] but {tensor_shape}"
    seq, mbs, hidden = tensor_shape
    tp = parallel_state.get_tensor_model_parallel_world_size()
    s = seq // tp if sequence_parallel_enabled else seq
    if model_type == ModelType.encoder_and_decoder:
        ds = decoder_sequence_length // tp if sequence_parallel_enabled else decoder_sequence_length
        if parallel_state.is_pipeline_stage_before_split(rank):
            return [(s, mbs, hidden)]
        return [(ds, mbs, hidden), (s, mbs, hidden)]
    return [(s, mbs, hidden)]


def recv_forward(tensor_shapes, *, dtype=None, async_comm=False, sequence_parallel_enabled=False):
    return [None if shape is None else p2p_communication.recv_forward(
        tensor_shape=shape, dtype=dtype, async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
        for shape in tensor_shapes]


def recv_backward(tensor_shapes, *, dtype=None, async_comm=False, sequence_parallel_enabled=False):
    return [None if shape is None else p2p_communication.recv_backward(
        tensor_shape=shape, dtype=dtype, async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
        for shape in tensor_shapes]


def send_forward(output_tensors, tensor_shapes, *, dtype=None, async_comm=False, sequence_parallel_enabled=False):
    if not isinstance(output_tensors, list):
        output_tensors = [output_tensors]
    for t, shape in zip(output_tensors, tensor_shapes):
        if shape is None:
            continue
        p2p_communication.send_forward(t, tensor_shape=shape, dtype=dtype, async_comm=async_comm,
                                       sequence_parallel_enabled=sequence_parallel_enabled)


def send_backward(input_tensor_grads, tensor_shapes, *, dtype=None, async_comm=False, sequence_parallel_enabled=False):
    if not isinstance(input_tensor_grads, list):
        input_tensor_grads = [input_tensor_grads]
    for g, shape in zip(input_tensor_grads, tensor_shapes):
        if shape is None:
            continue
        p2p_communication.send_backward(g, tensor_shape=shape, dtype=dtype, async_comm=async_comm,
                                        sequence_parallel_enabled=sequence_parallel_enabled)


def send_forward_recv_backward(output_tensors, tensor_shapes, *, dtype=None, async_comm=False,
                               sequence_parallel_enabled=False):
    if not isinstance(output_tensors, list):
        output_tensors = [output_tensors]
    out = []
    for t, shape in zip(output_tensors, tensor_shapes):
        if shape is None:
            out.append(None)
            continue
        out.append(p2p_communication.send_forward_recv_backward(
            t, tensor_shape=shape, dtype=dtype, async_comm=async_comm,
            sequence_parallel_enabled=sequence_parallel_enabled))
    return out


def send_backward_recv_forward(input_tensor_grads, tensor_shapes, *, dtype=None, async_comm=False,
                               sequence_parallel_enabled=False):
    if not isinstance(input_tensor_grads, list):
        input_tensor_grads = [input_tensor_grads]
    out = []
    for g, shape in zip(input_tensor_grads, tensor_shapes):
        if shape is None:
            out.append(None)
            continue
        out.append(p2p_communication.send_backward_recv_forward(
            g, tensor_shape=shape, dtype=dtype, async_comm=async_comm,
            sequence_parallel_enabled=sequence_parallel_enabled))
    return out


def forward_backward_pipelining_without_interleaving(
        forward_step_func: FwdStepFunc, batch: Optional[Batch], model: Union[torch.nn.Module, List[torch.nn.Module]],
        *, forward_only: bool, tensor_shape=None, decoder_sequence_length: Optional[int] = None,
        dtype: Optional[torch.dtype] = None, grad_scaler=None, disable_autocast: bool = False,
        deallocate_pipeline_outputs: bool = False, async_comm: bool = False, sequence_parallel_enabled: bool = False,
        **kwargs):
    """Returns per-microbatch reduced losses on the last stage, [] elsewhere."""
    model = listify_model(model)
    if len(model) != 1:
        raise RuntimeError(f"`model` is expected be a `nn.Module`, but {type(model)}")
    model = model[0]
    num_microbatches = get_num_microbatches()
    pp = parallel_state.get_pipeline_model_parallel_world_size()
    rank = parallel_state.get_pipeline_model_parallel_rank()
    num_warmup = num_microbatches if forward_only else min(pp - rank - 1, num_microbatches)
    num_remaining = num_microbatches - num_warmup
    model_type = get_model_type(model)
    recv_shapes = get_tensor_shapes(rank - 1, model_type, tensor_shape=tensor_shape,
                                    decoder_sequence_length=decoder_sequence_length,
                                    sequence_parallel_enabled=sequence_parallel_enabled)
    send_shapes = get_tensor_shapes(rank, model_type, tensor_shape=tensor_shape,
                                    decoder_sequence_length=decoder_sequence_length,
                                    sequence_parallel_enabled=sequence_parallel_enabled)
    comm = dict(dtype=dtype, async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
    input_tensors, output_tensors, losses_reduced = [], [], []

    for i in range(num_warmup):
        input_tensor = recv_forward(recv_shapes, **comm)
        output_tensor = forward_step(forward_step_func, get_kth_microbatch(batch, i), model, input_tensor,
                                     losses_reduced, dtype, disable_autocast)
        send_forward(output_tensor, send_shapes, **comm)
        if not forward_only:
            input_tensors.append(input_tensor)
            output_tensors.append(output_tensor)
            free_output_tensor(output_tensor, deallocate_pipeline_outputs)

    input_tensor = recv_forward(recv_shapes, **comm) if num_remaining > 0 else None

    for i in range(num_remaining):
        last = i == num_remaining - 1
        output_tensor = forward_step(forward_step_func, get_kth_microbatch(batch, i + num_warmup), model,
                                     input_tensor, losses_reduced, dtype, disable_autocast)
        if forward_only:
            send_forward(output_tensor, send_shapes, **comm)
            if not last:
                input_tensor = recv_forward(recv_shapes, **comm)
            continue
        output_tensor_grad = send_forward_recv_backward(output_tensor, send_shapes, **comm)
        input_tensors.append(input_tensor)
        output_tensors.append(output_tensor)
        free_output_tensor(output_tensor, deallocate_pipeline_outputs)
        input_tensor = input_tensors.pop(0)
        output_tensor = output_tensors.pop(0)
        input_tensor_grad = backward_step(input_tensor, output_tensor, output_tensor_grad, model_type=model_type,
                                          grad_scaler=grad_scaler,
                                          deallocate_pipeline_outputs=deallocate_pipeline_outputs)
        if last:
            input_tensor = None
            send_backward(input_tensor_grad, recv_shapes, **comm)
        else:
            input_tensor = send_backward_recv_forward(input_tensor_grad, recv_shapes, **comm)

    if not forward_only:
        for _ in range(num_warmup):
            input_tensor = input_tensors.pop(0)
            output_tensor = output_tensors.pop(0)
            output_tensor_grad = recv_backward(send_shapes, **comm)
            input_tensor_grad = backward_step(input_tensor, output_tensor, output_tensor_grad, model_type=model_type,
                                              grad_scaler=grad_scaler,
                                              deallocate_pipeline_outputs=deallocate_pipeline_outputs)
            send_backward(input_tensor_grad, recv_shapes, **comm)
    return losses_reduced
