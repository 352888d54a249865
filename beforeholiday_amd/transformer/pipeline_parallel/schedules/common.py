"""Pieces shared by the pipeline schedules: model construction per stage, one forward step, one
backward step, output pseudo-freeing (reference: apex/transformer/pipeline_parallel/schedules/common.py:30-398)."""
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import torch
from torch.autograd.variable import Variable

from ....normalization.fused_layer_norm import FusedLayerNorm
from ... import parallel_state
from ...enums import ModelType
from ...tensor_parallel.layers import set_defaults_if_not_set_tensor_model_parallel_attributes
from ..p2p_communication import FutureTensor
from ..utils import get_model_type, get_num_microbatches, listify_model, unwrap_model

Batch = Union[torch.Tensor, List[torch.Tensor], tuple]
LossFunc = Callable[[torch.Tensor], torch.Tensor]
FwdStepFunc = Callable[[Optional[Batch], torch.nn.Module], tuple]


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def build_model(model_provider_func: Callable[..., torch.nn.Module], wrap_with_ddp: bool = True,
                virtual_pipeline_model_parallel_size: Optional[int] = None,
                model_type: ModelType = ModelType.encoder_or_decoder, *args: Any, **kwargs: Any
                ) -> List[torch.nn.Module]:
    """Instantiate this rank's stage(s): ``model_provider_func(*args, pre_process=..., post_process=...,
    [add_encoder=..., add_decoder=...], **kwargs)`` once per virtual chunk, move to the device and
    optionally wrap each chunk in torch DDP over the data-parallel group."""
    pp = parallel_state.get_pipeline_model_parallel_world_size()
    if pp > 1 and virtual_pipeline_model_parallel_size is not None:
        model = []
        for i in range(virtual_pipeline_model_parallel_size):
            parallel_state.set_virtual_pipeline_model_parallel_rank(i)
            kw = dict(kwargs)
            kw.update(pre_process=parallel_state.is_pipeline_first_stage(),
                      post_process=parallel_state.is_pipeline_last_stage())
            model.append(model_provider_func(*args, **kw))
    else:
        kw = dict(kwargs)
        if model_type == ModelType.encoder_or_decoder:
            kw.update(pre_process=parallel_state.is_pipeline_first_stage(),
                      post_process=parallel_state.is_pipeline_last_stage())
        elif model_type == ModelType.encoder_and_decoder:
            pre = parallel_state.is_pipeline_first_stage()
            post = parallel_state.is_pipeline_last_stage()
            add_encoder = add_decoder = True
            if pp > 1:
                split = parallel_state.get_pipeline_model_parallel_split_rank()
                if split is None:
                    raise RuntimeError("Split rank needs to be specified for model with both encoder and decoder.")
                rank = parallel_state.get_pipeline_model_parallel_rank()
                pre = rank == 0 or rank == split
                post = rank == (split - 1) or rank == (pp - 1)
                add_encoder = parallel_state.is_pipeline_stage_before_split()
                add_decoder = parallel_state.is_pipeline_stage_after_split()
            kw.update(pre_process=pre, post_process=post, add_encoder=add_encoder, add_decoder=add_decoder)
        model = model_provider_func(*args, **kw)
        model.model_type = model_type
    if not isinstance(model, list):
        model = [model]
    for m in model:
        for p in m.parameters():
            set_defaults_if_not_set_tensor_model_parallel_attributes(p)
    if parallel_state.model_parallel_is_initialized() and parallel_state.get_data_parallel_rank() == 0:
        print(f" > number of parameters on (tensor, pipeline) model parallel rank "
              f"({parallel_state.get_tensor_model_parallel_rank()}, "
              f"{parallel_state.get_pipeline_model_parallel_rank()}): {_calc_number_of_params(model)}", flush=True)
    dev = _device()
    for m in model:
        m.to(dev)
    if wrap_with_ddp:
        ids = [dev.index] if dev.type == "cuda" else None
        model = [torch.nn.parallel.DistributedDataParallel(m, device_ids=ids, output_device=ids[0] if ids else None,
                                                           process_group=parallel_state.get_data_parallel_group())
                 for m in model]
    return model


def _calc_number_of_params(model: List[torch.nn.Module]) -> int:
    assert isinstance(model, list)
    return sum(p.nelement() for m in model for p in m.parameters())


def _get_params_for_weight_decay_optimization(model, *, no_weight_decay_modules=(FusedLayerNorm,)):
    """Two param groups: weights (decayed) and biases + norm parameters (weight_decay 0)."""
    decay = {"params": []}
    no_decay = {"params": [], "weight_decay": 0.0}
    for module in listify_model(model):
        for m in module.modules():
            params = [(n, p) for n, p in m._parameters.items() if p is not None]
            if isinstance(m, no_weight_decay_modules):
                no_decay["params"].extend(p for _, p in params)
            else:
                decay["params"].extend(p for n, p in params if n != "bias")
                no_decay["params"].extend(p for n, p in params if n == "bias")
    return decay, no_decay


def free_output_tensor(output_tensors, deallocate_pipeline_outputs: bool = False) -> None:
    """Drop the storage of stage outputs already sent downstream; only their grad_fn is still needed."""
    if not deallocate_pipeline_outputs or output_tensors is None:
        return
    if isinstance(output_tensors, torch.Tensor):
        output_tensors = [output_tensors]
    for t in output_tensors:
        t.data = torch.zeros(1, dtype=t.dtype, device=t.device)


def custom_backward(output: torch.Tensor, grad_output: Optional[torch.Tensor]) -> None:
    """Run the autograd engine directly (skips the shape check against the pseudo-freed output)."""
    assert output.numel() == 1, "output should be pseudo-freed in schedule, to optimize memory consumption"
    if grad_output is None:
        grad_output = torch.ones_like(output, memory_format=torch.preserve_format)
    Variable._execution_engine.run_backward(tensors=(output,), grad_tensors=(grad_output,), keep_graph=False,
                                            create_graph=False, inputs=(), allow_unreachable=True,
                                            accumulate_grad=True)


def forward_step(forward_step_func: FwdStepFunc, batch: Optional[Batch], model: torch.nn.Module,
                 input_tensor, losses_reduced: List[torch.Tensor], dtype: torch.dtype,
                 disable_autocast: bool = False):
    """Feed ``input_tensor`` (stage input) to the model via ``set_input_tensor``, run the user's step;
    on the last stage apply the loss function and scale by 1/num_microbatches."""
    unwrapped = unwrap_model(model)
    model_type = get_model_type(unwrapped)
    unwrap_output = not isinstance(input_tensor, list)
    if unwrap_output:
        input_tensor = [input_tensor]
    input_tensor = [t.get() if isinstance(t, FutureTensor) else t for t in input_tensor]
    unwrapped.set_input_tensor(input_tensor)
    with torch.autocast("cuda", enabled=not disable_autocast and dtype in (torch.half, torch.bfloat16),
                        dtype=dtype if dtype in (torch.half, torch.bfloat16) else torch.half):
        output_tensor, loss_func = forward_step_func(batch, model)
        if parallel_state.is_pipeline_last_stage():
            loss, loss_reduced = loss_func(output_tensor)
            output_tensor = loss / get_num_microbatches()
            losses_reduced.append(loss_reduced)
    if parallel_state.is_pipeline_stage_after_split() and model_type == ModelType.encoder_and_decoder:
        return [output_tensor, input_tensor[-1]]
    return output_tensor if unwrap_output else [output_tensor]


def backward_step(input_tensor, output_tensor, output_tensor_grad, model_type: ModelType, *,
                  grad_scaler=None, deallocate_pipeline_outputs: bool = False):
    """Backprop the stage output (scaled loss on the last stage), return the stage-input gradient(s)."""
    unwrap_grad = not isinstance(input_tensor, list)
    if unwrap_grad:
        input_tensor = [input_tensor]
    input_tensor = [t.get() if isinstance(t, FutureTensor) else t for t in input_tensor]
    for x in input_tensor:
        if x is not None:
            x.retain_grad()
    if not isinstance(output_tensor, list):
        output_tensor = [output_tensor]
    output_tensor = [t.get() if isinstance(t, FutureTensor) else t for t in output_tensor]
    if not isinstance(output_tensor_grad, list):
        output_tensor_grad = [output_tensor_grad]
    output_tensor_grad = [t.get() if isinstance(t, FutureTensor) else t for t in output_tensor_grad]
    if grad_scaler is not None and output_tensor_grad[0] is None:
        output_tensor[0] = grad_scaler.scale(output_tensor[0])
    if deallocate_pipeline_outputs:
        custom_backward(output_tensor[0], output_tensor_grad[0])
    else:
        torch.autograd.backward(output_tensor[0], grad_tensors=output_tensor_grad[0])
    input_tensor_grad = [None if x is None else x.grad for x in input_tensor]
    if (parallel_state.get_pipeline_model_parallel_world_size() > 1 and
            parallel_state.is_pipeline_stage_after_split() and model_type == ModelType.encoder_and_decoder):
        if len(output_tensor_grad) > 1 and output_tensor_grad[1] is not None:
            input_tensor_grad[-1].add_(output_tensor_grad[1])
    return input_tensor_grad[0] if unwrap_grad else input_tensor_grad
