"""amp._initialize (reference: apex/amp/_initialize.py:147-267).

Casts models (keeping BatchNorm fp32 when asked), patches forward to cast inputs/outputs, adds
fp32 state_dict hooks, processes optimizers (master weights / grad stashing) and builds the loss
scalers. Device-agnostic: CPU models work (the reference requires CUDA tensors).
"""
from __future__ import annotations

import collections.abc as container_abcs
import functools
import warnings
from types import MethodType

import numpy as np
import torch

from ._amp_state import _amp_state, warn_or_err
from ._process_optimizer import _process_optimizer
from .scaler import LossScaler

_LOW = (torch.float16, torch.bfloat16)


def to_type(dtype, t):
    if isinstance(t, torch.Tensor):
        if t.is_floating_point():
            return t.to(dtype)
        return t
    return t.to(dtype)


def applier(value, fn):
    if isinstance(value, torch.Tensor):
        return fn(value)
    if isinstance(value, str):
        return value
    if isinstance(value, np.ndarray):
        return value
    if hasattr(value, "to"):  # custom batch classes
        return fn(value)
    if isinstance(value, container_abcs.Mapping):
        return {applier(k, fn): applier(v, fn) for k, v in value.items()}
    if isinstance(value, container_abcs.Iterable):
        return type(value)(applier(v, fn) for v in value)
    return value


def check_models(models):
    from ..parallel.distributed import DistributedDataParallel as bh_DDP

    for model in models:
        parallel_type = None
        if isinstance(model, torch.nn.parallel.DistributedDataParallel):
            parallel_type = "torch.nn.parallel.DistributedDataParallel"
        if isinstance(model, bh_DDP):
            parallel_type = "beforeholiday_amd.parallel.DistributedDataParallel"
        if isinstance(model, torch.nn.parallel.DataParallel):
            parallel_type = "torch.nn.parallel.DataParallel"
        if parallel_type is not None:
            raise RuntimeError("Incoming model is an instance of {}. Parallel wrappers should only be applied "
                               "to the model(s) AFTER \nthe model(s) have been returned from amp.initialize."
                               .format(parallel_type))


def check_params_fp32(models):
    for model in models:
        for name, param in model.named_parameters():
            if param.is_floating_point() and param.dtype in _LOW:
                warn_or_err("Found param {} with type {}, expected torch.float32.\nWhen using amp.initialize, "
                            "you do not need to call .half() or .bfloat16()\non your model before passing it, no "
                            "matter what optimization level you choose.".format(name, param.type()))
        for name, buf in model.named_buffers():
            if buf.is_floating_point() and buf.dtype in _LOW:
                warn_or_err("Found buffer {} with type {}, expected torch.float32.\nWhen using amp.initialize, "
                            "you do not need to call .half() on your model\nbefore passing it, no matter what "
                            "optimization level you choose.".format(name, buf.type()))


def check_optimizers(optimizers):
    from ..fp16_utils import FP16_Optimizer

    for optim in optimizers:
        if isinstance(optim, FP16_Optimizer):
            raise RuntimeError("An incoming optimizer is an instance of fp16_utils.FP16_Optimizer. The "
                               "optimizer(s) passed to amp.initialize() must be bare \ninstances of either ordinary "
                               "Pytorch optimizers, or fused optimizers.\n")


class O2StateDictHook(object):
    """Makes ``model.state_dict()`` return fp32 tensors under O2/O3/O5."""

    def __init__(self, fn):
        self.fn = fn

    def __call__(self, module, state_dict, prefix, local_metadata):
        for key in state_dict:
            param = state_dict[key]
            if isinstance(param, torch.Tensor) and param.dtype in _LOW:
                state_dict[key] = param.to(torch.float32)


def _is_optimizer(o):
    from ..parallel.LARC import LARC

    return isinstance(o, (torch.optim.Optimizer, LARC))


def _initialize(models, optimizers, properties, num_losses=1, cast_model_outputs=None):
    from ..fp16_utils import convert_network
    from .amp import init as amp_init
    from .handle import disable_casts

    optimizers_was_list = False
    if _is_optimizer(optimizers):
        optimizers = [optimizers]
    elif optimizers is None:
        optimizers = []
    elif isinstance(optimizers, list):
        optimizers_was_list = True
        check_optimizers(optimizers)
    else:
        check_optimizers([optimizers])
        raise TypeError("optimizers must be either a single optimizer or a list of optimizers.")

    if isinstance(models, torch.nn.Module):
        models_was_list = False
        models = [models]
    elif isinstance(models, list):
        models_was_list = True
    else:
        raise TypeError("models must be either a single model or a list of models.")

    check_models(models)
    if not _amp_state.allow_incoming_model_not_fp32:
        check_params_fp32(models)

    if properties.cast_model_type:
        if properties.keep_batchnorm_fp32:
            for model in models:
                convert_network(model, properties.cast_model_type)
        else:
            for model in models:
                model.to(properties.cast_model_type)
        input_caster = functools.partial(to_type, properties.cast_model_type)
        output_caster = functools.partial(to_type, cast_model_outputs if cast_model_outputs is not None
                                          else torch.float32)
        for model in models:
            def patch_forward(old_fwd):
                def new_fwd(*args, **kwargs):
                    output = old_fwd(*applier(args, input_caster), **applier(kwargs, input_caster))
                    return applier(output, output_caster)
                return new_fwd
            model.forward = patch_forward(model.forward)
        # recast per-param optimizer state (e.g. momentum buffers) to the new param types
        for optimizer in optimizers:
            optimizer.load_state_dict(optimizer.state_dict())
        for model in models:
            for module in model.modules():
                module._register_state_dict_hook(O2StateDictHook(functools.partial(to_type, torch.float32)))
    elif cast_model_outputs is not None:
        output_caster = functools.partial(to_type, cast_model_outputs)
        for model in models:
            def patch_forward(old_fwd):
                def new_fwd(*args, **kwargs):
                    return applier(old_fwd(*args, **kwargs), output_caster)
                return new_fwd
            model.forward = patch_forward(model.forward)

    for i, optimizer in enumerate(optimizers):
        optimizers[i] = _process_optimizer(optimizer, properties)

    device = None
    for model in models:
        for p in model.parameters():
            device = p.device
            break
    _amp_state.loss_scalers = [LossScaler(properties.loss_scale, min_loss_scale=_amp_state.min_loss_scale,
                                          max_loss_scale=_amp_state.max_loss_scale, device=device)
                               for _ in range(num_losses)]

    if properties.patch_torch_functions:
        # O1/O4: patch torch functions with cast wrappers; the optimizer step runs with casts off
        amp_init(loss_scale=properties.loss_scale, patch_type=properties.patch_torch_functions_type,
                 verbose=(_amp_state.verbosity == 2))
        for optimizer in optimizers:
            def patch_step(old_step):
                def new_step(self, *args, **kwargs):
                    with disable_casts():
                        return old_step(*args, **kwargs)
                return new_step
            optimizer.step = MethodType(patch_step(optimizer.step), optimizer)

    if optimizers_was_list:
        return (models if models_was_list else models[0]), optimizers
    if models_was_list:
        return models if len(optimizers) == 0 else (models, optimizers[0])
    return models[0] if len(optimizers) == 0 else (models[0], optimizers[0])
