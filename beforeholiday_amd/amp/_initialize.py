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


def _as_list(obj, is_item, what):
    """(list, was_list) for the ``models`` / ``optimizers`` argument: one item, a list, or None."""
    if obj is None and what == "optimizers":
        return [], False
    if is_item(obj):
        return [obj], False
    if isinstance(obj, list):
        return obj, True
    raise TypeError(f"{what} must be either a single {what[:-1]} or a list of {what}.")


class _CastingForward(object):
    """Replacement ``model.forward``: floating-point tensors in ``args`` / ``kwargs`` are cast with
    ``cast_in`` (None: untouched), every floating-point tensor of the output with ``cast_out``."""

    def __init__(self, inner, cast_in, cast_out):
        self.inner, self.cast_in, self.cast_out = inner, cast_in, cast_out

    def __call__(self, *args, **kwargs):
        if self.cast_in is not None:
            args, kwargs = applier(args, self.cast_in), applier(kwargs, self.cast_in)
        return applier(self.inner(*args, **kwargs), self.cast_out)


def _cast_models(models, optimizers, properties, cast_model_outputs):
    """O2 / O3 / O5: the model weights in the low dtype (BatchNorms kept fp32 when asked), inputs cast on
    the way in, outputs on the way out (fp32 unless ``cast_model_outputs``), fp32 ``state_dict``."""
    from ..fp16_utils import convert_network

    low = properties.cast_model_type
    out_dtype = cast_model_outputs if cast_model_outputs is not None else torch.float32
    for model in models:
        if properties.keep_batchnorm_fp32:
            convert_network(model, low)
        else:
            model.to(low)
        model.forward = _CastingForward(model.forward, functools.partial(to_type, low),
                                        functools.partial(to_type, out_dtype))
        hook = O2StateDictHook(functools.partial(to_type, torch.float32))
        for module in model.modules():
            module._register_state_dict_hook(hook)
    # state created before the cast (e.g. momentum buffers) follows the parameters' new dtype
    for optimizer in optimizers:
        optimizer.load_state_dict(optimizer.state_dict())


def _casts_off_during_step(optimizer):
    """O1 / O4: the optimizer step runs with the function-cast wrappers disabled."""
    from .handle import disable_casts

    inner = optimizer.step

    def step(self, *args, **kwargs):
        with disable_casts():
            return inner(*args, **kwargs)

    optimizer.step = MethodType(step, optimizer)


def _initialize(models, optimizers, properties, num_losses=1, cast_model_outputs=None):
    from .amp import init as amp_init

    if isinstance(optimizers, list):
        check_optimizers(optimizers)
    elif optimizers is not None and not _is_optimizer(optimizers):
        check_optimizers([optimizers])
    optimizers, optimizers_was_list = _as_list(optimizers, _is_optimizer, "optimizers")
    models, models_was_list = _as_list(models, lambda m: isinstance(m, torch.nn.Module), "models")

    check_models(models)
    if not _amp_state.allow_incoming_model_not_fp32:
        check_params_fp32(models)

    if properties.cast_model_type:
        _cast_models(models, optimizers, properties, cast_model_outputs)
    elif cast_model_outputs is not None:
        for model in models:
            model.forward = _CastingForward(model.forward, None, functools.partial(to_type, cast_model_outputs))

    optimizers = [_process_optimizer(o, properties) for o in optimizers]
    device = next((p.device for m in models for p in m.parameters()), None)
    _amp_state.loss_scalers = [LossScaler(properties.loss_scale, min_loss_scale=_amp_state.min_loss_scale,
                                          max_loss_scale=_amp_state.max_loss_scale, device=device)
                               for _ in range(num_losses)]

    if properties.patch_torch_functions:
        amp_init(loss_scale=properties.loss_scale, patch_type=properties.patch_torch_functions_type,
                 verbose=(_amp_state.verbosity == 2))
        for optimizer in optimizers:
            _casts_off_during_step(optimizer)

    model_ret = models if models_was_list else models[0]
    if optimizers_was_list:
        return model_ret, optimizers
    return model_ret if not optimizers else (model_ret, optimizers[0])
