"""Gradient accumulation over microbatches without pipeline stages
(reference: apex/transformer/pipeline_parallel/schedules/fwd_bwd_no_pipelining.py:24-132).

All but the last microbatch run under the DDP ``no_sync`` context, so the gradient all-reduce runs
once, overlapped with the last backward."""
import contextlib
from typing import List, Optional, Union

import torch

from ..utils import get_kth_microbatch, get_model_type, get_num_microbatches, listify_model
from .common import Batch, FwdStepFunc, backward_step, forward_step


@contextlib.contextmanager
def placeholder_handler():
    yield


def forward_backward_no_pipelining(forward_step_func: FwdStepFunc, batch: Batch,
                                   model: Union[torch.nn.Module, List[torch.nn.Module]], *, forward_only: bool,
                                   dtype: Optional[torch.dtype] = None, grad_scaler=None,
                                   disable_autocast: bool = False, custom_sync_context_handler=None, **kwargs):
    """Returns the list of per-microbatch reduced losses (last stage) — here every rank is the last stage."""
    model = listify_model(model)
    if len(model) != 1:
        raise RuntimeError(f"`model` is expected be a `nn.Module`, but {type(model)}")
    model = model[0]
    model_type = get_model_type(model)
    if custom_sync_context_handler is not None:
        context_handler = custom_sync_context_handler
    elif hasattr(model, "no_sync"):
        context_handler = model.no_sync
    else:
        context_handler = placeholder_handler
    losses_reduced = []
    n = get_num_microbatches()
    with context_handler():
        for i in range(n - 1):
            out = forward_step(forward_step_func, get_kth_microbatch(batch, i), model, None, losses_reduced,
                               dtype=dtype, disable_autocast=disable_autocast)
            if not forward_only:
                backward_step(None, out, None, model_type=model_type, grad_scaler=grad_scaler)
    out = forward_step(forward_step_func, get_kth_microbatch(batch, n - 1), model, None, losses_reduced, dtype=dtype,
                       disable_autocast=disable_autocast)
    if not forward_only:
        backward_step(None, out, None, model_type=model_type, grad_scaler=grad_scaler)
    return losses_reduced
