"""Point-to-point activation / gradient exchange between pipeline stages
(reference: apex/transformer/pipeline_parallel/p2p_communication.py:34-578).

Every exchange is ONE ``batch_isend_irecv`` group over the pipeline group (RCCL groups the sends and
receives into a single launch; neighbouring stages on an MI355X node talk over a direct xGMI link).
Completion is ordered on the device: ``work.wait()`` makes the current stream wait for RCCL's stream,
so no host-side ``synchronize()`` is needed (the reference calls ``torch.cuda.synchronize()`` after
every exchange). With ``async_comm`` the received tensors are returned as :class:`FutureTensor`
whose ``get()`` performs that wait.
"""
import functools
import operator
from typing import List, Optional, Sequence, Tuple, Union

import torch

from .. import parallel_state
from ..utils import gather_split_1d_tensor, split_tensor_into_1d_equal_chunks
from ._timers import _Timers

Shape = Union[List[int], torch.Size, Tuple[int, ...]]


class FutureTensor:
    def __init__(self, tensor: torch.Tensor, waitfunc):
        self.tensor = tensor
        self.waitfunc = waitfunc

    def get(self):
        if self.waitfunc is not None:
            res = self.waitfunc()
            if isinstance(res, torch.Tensor):
                self.tensor = res
            self.waitfunc = None
        return self.tensor


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def _run_p2pops(tensor_send_prev, tensor_send_next, tensor_recv_prev, tensor_recv_next, async_comm=False):
    group = parallel_state.get_pipeline_model_parallel_group()
    prev_rank = parallel_state.get_pipeline_model_parallel_prev_rank()
    next_rank = parallel_state.get_pipeline_model_parallel_next_rank()
    ops, slots = [], []
    if tensor_send_prev is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.isend, tensor_send_prev, prev_rank, group))
        slots.append("send_prev")
    if tensor_recv_prev is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.irecv, tensor_recv_prev, prev_rank, group))
        slots.append("recv_prev")
    if tensor_send_next is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.isend, tensor_send_next, next_rank, group))
        slots.append("send_next")
    if tensor_recv_next is not None:
        ops.append(torch.distributed.P2POp(torch.distributed.irecv, tensor_recv_next, next_rank, group))
        slots.append("recv_next")
    reqs = {"send_prev": None, "recv_prev": None, "send_next": None, "recv_next": None}
    if ops:
        works = torch.distributed.batch_isend_irecv(ops)
        if len(works) == len(ops):
            reqs.update(dict(zip(slots, works)))
        else:  # a coalesced backend returns one work for the whole group
            for s in slots:
                reqs[s] = works[0] if works else None
        if not async_comm:
            for w in set(w for w in works if w is not None):
                w.wait()
    return reqs["send_prev"], reqs["recv_prev"], reqs["send_next"], reqs["recv_next"]


def _communicate(tensor_send_next: Optional[torch.Tensor], tensor_send_prev: Optional[torch.Tensor], recv_prev: bool,
                 recv_next: bool, tensor_shape: Optional[Shape] = None,
                 override_scatter_gather_tensors_in_pipeline: bool = False, dtype_: Optional[torch.dtype] = None, *,
                 scatter_gather_tensors_in_pipeline: bool = True, params_dtype: Optional[torch.dtype] = None,
                 fp32_residual_connection: bool = False, async_comm: bool = False,
                 sequence_parallel_enabled: bool = False):
    """Exchange with neighbour stages. Returns (recv_prev, recv_next) tensors (or FutureTensors).

    With tensor parallelism each TP rank holds the same stage output, so (when the size divides and
    sequence parallelism is off) only a 1/tp slice is sent and the receivers all-gather it over the TP
    group — tp-times fewer bytes over the inter-stage link.
    """
    if tensor_shape is None:
        raise RuntimeError("`tensor_shape` must be specified. Common `tensor_shape` is "
                           "`(seq_length, micro_batch_size, hidden_size)`")
    tp = parallel_state.get_tensor_model_parallel_world_size()
    numel = int(functools.reduce(operator.mul, tensor_shape, 1))
    scatter_gather = (scatter_gather_tensors_in_pipeline and not override_scatter_gather_tensors_in_pipeline and
                      not sequence_parallel_enabled and tp > 1 and numel % tp == 0)
    chunk_shape = [numel // tp] if scatter_gather else list(tensor_shape)
    dtype = params_dtype or torch.float
    if fp32_residual_connection:
        dtype = torch.float
    if dtype_ is not None:
        dtype = dtype_
    dev = _device()
    tensor_recv_prev = torch.empty(chunk_shape, requires_grad=True, device=dev, dtype=dtype) if recv_prev else None
    tensor_recv_next = torch.empty(chunk_shape, requires_grad=True, device=dev, dtype=dtype) if recv_next else None
    if tensor_send_next is not None:
        tensor_send_next = tensor_send_next.contiguous()
        if scatter_gather:
            tensor_send_next = split_tensor_into_1d_equal_chunks(tensor_send_next)
    if tensor_send_prev is not None:
        tensor_send_prev = tensor_send_prev.contiguous()
        if scatter_gather:
            tensor_send_prev = split_tensor_into_1d_equal_chunks(tensor_send_prev)
    _, req_prev, _, req_next = _run_p2pops(tensor_send_prev, tensor_send_next, tensor_recv_prev, tensor_recv_next,
                                           async_comm=async_comm)

    def finish(t):
        if t is None:
            return None
        if scatter_gather:
            return gather_split_1d_tensor(t.detach()).view(tensor_shape).requires_grad_()
        return t

    if not async_comm:
        return finish(tensor_recv_prev), finish(tensor_recv_next)

    def waiter(req, t):
        def wait():
            if req is not None:
                req.wait()
            return finish(t)
        return wait

    fp = FutureTensor(tensor_recv_prev, waiter(req_prev, tensor_recv_prev)) if recv_prev else None
    fn = FutureTensor(tensor_recv_next, waiter(req_next, tensor_recv_next)) if recv_next else None
    return fp, fn


def recv_forward(tensor_shape: Shape, override_scatter_gather_tensors_in_pipeline: bool = False, *,
                 dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                 sequence_parallel_enabled: bool = False, timers: _Timers = None):
    """Receive the activation from the previous stage (None on the first stage)."""
    if parallel_state.is_pipeline_first_stage():
        return None
    out, _ = _communicate(None, None, True, False, tensor_shape, override_scatter_gather_tensors_in_pipeline, dtype,
                          async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def recv_backward(tensor_shape: Shape = None, *, dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                  sequence_parallel_enabled: bool = False, timers: _Timers = None):
    """Receive the output gradient from the next stage (None on the last stage)."""
    if parallel_state.is_pipeline_last_stage():
        return None
    _, out = _communicate(None, None, False, True, tensor_shape, dtype_=dtype, async_comm=async_comm,
                          sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def send_forward(output_tensor: torch.Tensor, override_scatter_gather_tensors_in_pipeline: bool = False,
                 tensor_shape: Shape = None, *, dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                 sequence_parallel_enabled: bool = False, timers: _Timers = None) -> None:
    if parallel_state.is_pipeline_last_stage():
        return
    _communicate(output_tensor, None, False, False, tensor_shape, override_scatter_gather_tensors_in_pipeline, dtype,
                 async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)


def send_backward(input_tensor_grad: torch.Tensor, tensor_shape: Shape, *, dtype: Optional[torch.dtype] = None,
                  async_comm: bool = False, sequence_parallel_enabled: bool = False, timers: _Timers = None) -> None:
    if parallel_state.is_pipeline_first_stage():
        return
    _communicate(None, input_tensor_grad, False, False, tensor_shape, dtype_=dtype, async_comm=async_comm,
                 sequence_parallel_enabled=sequence_parallel_enabled)


def send_forward_recv_backward(output_tensor: torch.Tensor, tensor_shape: Shape, *,
                               dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                               sequence_parallel_enabled: bool = False, timers: _Timers = None):
    if parallel_state.is_pipeline_last_stage():
        return None
    _, out = _communicate(output_tensor, None, False, True, tensor_shape, dtype_=dtype, async_comm=async_comm,
                          sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def send_backward_recv_forward(input_tensor_grad: torch.Tensor, tensor_shape: Shape, *,
                               dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                               sequence_parallel_enabled: bool = False, timers: _Timers = None):
    if parallel_state.is_pipeline_first_stage():
        return None
    out, _ = _communicate(None, input_tensor_grad, True, False, tensor_shape, dtype_=dtype, async_comm=async_comm,
                          sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def send_forward_recv_forward(output_tensor: torch.Tensor, recv_prev: bool, tensor_shape: Shape, *,
                              dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                              sequence_parallel_enabled: bool = False, timers: _Timers = None):
    out, _ = _communicate(output_tensor, None, recv_prev, False, tensor_shape, dtype_=dtype, async_comm=async_comm,
                          sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def send_backward_recv_backward(input_tensor_grad: torch.Tensor, recv_next: bool, tensor_shape: Shape, *,
                                dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                                sequence_parallel_enabled: bool = False, timers: _Timers = None):
    _, out = _communicate(None, input_tensor_grad, False, recv_next, tensor_shape, dtype_=dtype,
                          async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
    return out


def send_forward_backward_recv_forward_backward(output_tensor: torch.Tensor, input_tensor_grad: torch.Tensor,
                                                recv_prev: bool, recv_next: bool, tensor_shape: Shape, *,
                                                dtype: Optional[torch.dtype] = None, async_comm: bool = False,
                                                sequence_parallel_enabled: bool = False, timers: _Timers = None):
    return _communicate(output_tensor, input_tensor_grad, recv_prev, recv_next, tensor_shape, dtype_=dtype,
                        async_comm=async_comm, sequence_parallel_enabled=sequence_parallel_enabled)
